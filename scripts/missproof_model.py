#!/usr/bin/env python3
"""CPU model of the RC march's miss proof (k_rc_level, tuning rc_mp).

A ray of RadianceCascades.fs:60-92 that hits nothing returns (0,0,0,1) however its march ends, so
a proof that none of its samples can pass the hit test replaces the whole march.  The model marches
sampled rays of every level exactly (distance from an exact EDT of the demo scene, as
scripts/sim_gather_lines.py) and reports, per level:

  * hit fraction, samples per ray without and with the exit proofs of the current kernel;
  * the fraction of rays the coarse trace proves (cells of C texels flagged when a texel passes the
    hit test, Chebyshev cell distance k to the nearest flagged cell, advance (k-1)*C - 1 texels in
    max-norm per step) and its mean / max steps;
  * the samples per ray left with the miss proof on top of the exit proofs.

It also asserts the proof's soundness on the sampled rays (no proved ray hits).
Usage: python scripts/missproof_model.py [size=4096] [cell=64] [N=6] [rayRange=2] [rays=20000]
"""
import math
import sys

import numpy as np
from scipy import ndimage

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from sim_gather_lines import dist_field, march  # noqa: E402


def exit_proof_samples(D, cm, C2, ox, oy, dx, dy, t0, t1, W):
    """samples per ray of the current march with exit proofs (bound k/512 per 64x64-cell grid)"""
    n = ox.size
    t = np.full(n, t0)
    act = np.ones(n, bool)
    cnt = np.zeros(n)
    with np.errstate(divide="ignore", invalid="ignore"):
        Tx = np.where(dx > 0, (1 - ox) / dx, np.where(dx < 0, -ox / dx, np.inf))
        Ty = np.where(dy > 0, (1 - oy) / dy, np.where(dy < 0, -oy / dy, np.inf))
    T = np.minimum(Tx, Ty)
    for _ in range(32):
        px, py = ox + t * dx, oy + t * dy
        live = act & (t <= t1) & (px >= 0) & (py >= 0) & (px <= 1) & (py <= 1)
        ix = np.clip((px * W).astype(int), 0, W - 1)
        iy = np.clip((py * W).astype(int), 0, W - 1)
        dl = cm[iy // C2, ix // C2]
        live &= ~((dl > 0) & (t + dl >= np.minimum(t1, T)))
        if not live.any():
            break
        cnt += live
        d = D[iy, ix]
        act = live & ~(d < 0.001)
        t = np.where(act, t + d, t)
    return cnt


def coarse_trace(dt, C, ox, oy, dx, dy, t0, t1, W):
    """(proved, steps) per ray"""
    n = ox.size
    t = np.full(n, t0)
    proved = np.zeros(n, bool)
    active = np.ones(n, bool)
    steps = np.zeros(n)
    m = np.maximum(np.abs(dx), np.abs(dy))
    for _ in range(32):
        px, py = ox + t * dx, oy + t * dy
        off = (px < 0) | (py < 0) | (px > 1) | (py > 1) | (t > t1)
        proved |= active & off
        active &= ~off
        if not active.any():
            break
        ix = np.clip((px * W).astype(int), 0, W - 1) // C
        iy = np.clip((py * W).astype(int), 0, W - 1) // C
        k = dt[iy, ix]
        active &= k > 1
        steps += active
        t = np.where(active, t + (C * (k - 1) - 1.0) / W / m, t)
    return proved, steps


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    N = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    rr = float(sys.argv[4]) if len(sys.argv) > 4 else 2.0
    n = int(sys.argv[5]) if len(sys.argv) > 5 else 20000
    D = dist_field(W, W)
    G = W // C
    flag = (D < 0.001).reshape(G, C, G, C).any(axis=(1, 3))
    dt = np.minimum(ndimage.distance_transform_cdt(~flag, metric="chessboard"), 255) if flag.any() else \
        np.full((G, G), 255)
    C2 = W // 64
    cmv = D.reshape(64, C2, 64, C2).min(axis=(1, 3))
    cm = np.where(cmv < 0.001, 0, np.floor(cmv * 512) / 512)
    rng = np.random.default_rng(0)
    print(f"{W}^2 N={N} rayRange={rr}, cells of {C} texels, {n} rays per level")
    for L in range(N):
        b = 1 << L
        bd = W // b
        t0 = (4 ** L - 1) / (4 ** N - 1) * rr
        t1 = (4 ** (L + 1) - 1) / (4 ** N - 1) * rr
        cx, cy, ai = rng.integers(0, bd, n), rng.integers(0, bd, n), rng.integers(0, 4 * b * b, n)
        ox, oy = (cx + 0.5) * b / W, (cy + 0.5) * b / W
        th = (ai + 0.5) * 2 * math.pi / (4 * b * b)
        dx, dy = np.cos(th), np.sin(th)
        R = march(D, ox.astype(np.float32), oy.astype(np.float32), dx.astype(np.float32), dy.astype(np.float32),
                  t0, t1, W, W)
        hit = np.zeros(n, bool)
        samples = np.zeros(n)
        for ix, iy, lv in R:
            hit |= lv & (D[iy, ix] < 0.001)
            samples += lv
        ex = exit_proof_samples(D, cm, C2, ox, oy, dx, dy, t0, t1, W)
        proved, steps = coarse_trace(dt, C, ox, oy, dx, dy, t0, t1, W)
        assert not (proved & hit).any(), "a proved ray hits: the proof is unsound"
        print(f"L{L}: hit {hit.mean():.3f}  samples/ray {samples.mean():.3f}, exit proofs {ex.mean():.3f}, "
              f"+ miss proof {ex[~proved].sum() / n:.3f}  | proved {proved.mean():.3f} "
              f"(of the misses {proved.sum() / max(1, (~hit).sum()):.3f}), steps mean {steps.mean():.2f} "
              f"max {steps.max():.0f}")


if __name__ == "__main__":
    main()
