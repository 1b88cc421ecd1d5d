#!/usr/bin/env python3
"""CPU model of the RC march's directional miss proof (k_rc_level + k_dir_clear, tuning rc_mp;
DESIGN.md §5.6).

A ray of RadianceCascades.fs:60-92 that hits nothing returns (0,0,0,1) however its march ends, so a
sample from which no later sample of the ray can pass the hit test ends the ray unread.  The proof
table holds, per angular bin of directions and per cell of C texels, the distance (in cells) a ray of
any direction of the bin can travel from any point of the cell before it reaches a cell holding a
hit-test texel (box sweep of the cone, as k_dir_clear).  The model marches sampled rays of every level
exactly (distance from an exact EDT of the demo scene, as scripts/sim_gather_lines.py) and reports:

  * hit fraction; samples per ray with the current exit proofs and with the directional proof (the
    per-sample test, which proves most misses at their first sample);
  * the fraction of rays proved before any gather;
and asserts on the sampled rays that no proved ray hits.
Usage: python scripts/dirproof_model.py [size=4096] [cell=64] [bins=64] [N=6] [rayRange=2] [rays=30000]
"""
import math
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from sim_gather_lines import dist_field  # noqa: E402


def clear_table(flag, C, NB, steps=64):
    """[NB, G, G] clear distance in cells (255: none within `steps`), as k_dir_clear"""
    G = flag.shape[0]
    out = np.full((NB, G, G), 255, np.int32)
    for j in range(NB):
        ta, tb = 2 * math.pi * j / NB, 2 * math.pi * (j + 1) / NB
        sag = 1 - math.cos((tb - ta) / 2)
        done = np.zeros((G, G), bool)
        for s in range(steps):
            r0, r1 = s * C, (s + 1) * C
            pts = np.array([[math.cos(t) * r, math.sin(t) * r] for t in (ta, tb) for r in (r0, r1)])
            m = r1 * sag + 1.0
            lo, hi = pts.min(0) - m, pts.max(0) + m + C - 1e-6
            x0, x1 = int(math.floor(lo[0] / C)), int(math.floor(hi[0] / C))
            y0, y1 = int(math.floor(lo[1] / C)), int(math.floor(hi[1] / C))
            hit = np.zeros((G, G), bool)
            for oy in range(y0, y1 + 1):
                for ox in range(x0, x1 + 1):
                    a0, a1 = max(0, -oy), min(G, G - oy)
                    b0, b1 = max(0, -ox), min(G, G - ox)
                    if a0 < a1 and b0 < b1:
                        hit[a0:a1, b0:b1] |= flag[a0 + oy:a1 + oy, b0 + ox:b1 + ox]
            new = hit & ~done
            out[j][new] = s
            done |= hit
            if done.all():
                break
    return out


def main():
    a = [float(x) for x in sys.argv[1:]]
    W = int(a[0]) if a else 4096
    C = int(a[1]) if len(a) > 1 else 64
    NB = int(a[2]) if len(a) > 2 else 64
    N = int(a[3]) if len(a) > 3 else 6
    rr = a[4] if len(a) > 4 else 2.0
    n = int(a[5]) if len(a) > 5 else 30000
    D = dist_field(W, W)
    G = W // C
    flag = (D < 0.001).reshape(G, C, G, C).any(axis=(1, 3))
    tab = clear_table(flag, C, NB)
    C2 = W // 64
    cmv = D.reshape(64, C2, 64, C2).min(axis=(1, 3))
    cm = np.where(cmv < 0.001, 0, np.floor(cmv * 512) / 512)
    rng = np.random.default_rng(0)
    print(f"{W}^2 N={N} rayRange={rr}, cells of {C} texels, {NB} bins, {n} rays per level")
    for L in range(N):
        b = 1 << L
        t0 = (4 ** L - 1) / (4 ** N - 1) * rr
        t1 = (4 ** (L + 1) - 1) / (4 ** N - 1) * rr
        bd = W // b
        cx, cy, ai = rng.integers(0, bd, n), rng.integers(0, bd, n), rng.integers(0, 4 * b * b, n)
        ox, oy = (cx + 0.5) * b / W, (cy + 0.5) * b / W
        th = (ai + 0.5) * 2 * math.pi / (4 * b * b)
        dx, dy = np.cos(th), np.sin(th)
        with np.errstate(divide="ignore", invalid="ignore"):
            Tx = np.where(dx > 0, (1 - ox) / dx, np.where(dx < 0, -ox / dx, np.inf))
            Ty = np.where(dy > 0, (1 - oy) / dy, np.where(dy < 0, -oy / dy, np.inf))
        te = np.minimum(t1, np.minimum(Tx, Ty))
        jb = (th / (2 * math.pi) * NB).astype(int) % NB
        use_dir = b * b >= NB  # one bin per direction block
        t = np.full(n, t0)
        act = np.ones(n, bool)
        hit = np.zeros(n, bool)
        cnt_dir = np.zeros(n)
        cnt_exit = np.zeros(n)
        proved0 = np.zeros(n, bool)
        t_e, act_e = t.copy(), act.copy()
        for it in range(32):
            # directional proof march
            px, py = ox + t * dx, oy + t * dy
            live = act & (t <= t1) & (px >= 0) & (py >= 0) & (px <= 1) & (py <= 1)
            ix, iy = np.clip((px * W).astype(int), 0, W - 1), np.clip((py * W).astype(int), 0, W - 1)
            if use_dir:
                clr = tab[jb, iy // C, ix // C] * C / W
                pr = live & (t + clr >= te)
                if it == 0:
                    proved0 = pr.copy()
                live &= ~pr
            cnt_dir += live
            d = D[iy, ix]
            h = live & (d < 0.001)
            hit |= h
            act = live & ~h
            t = np.where(act, t + d, t)
            # exit-proof march (the current kernel)
            px, py = ox + t_e * dx, oy + t_e * dy
            live = act_e & (t_e <= t1) & (px >= 0) & (py >= 0) & (px <= 1) & (py <= 1)
            ix, iy = np.clip((px * W).astype(int), 0, W - 1), np.clip((py * W).astype(int), 0, W - 1)
            dl = cm[iy // C2, ix // C2]
            live &= ~((dl > 0) & (t_e + dl >= te))
            cnt_exit += live
            d = D[iy, ix]
            act_e = live & ~(d < 0.001)
            t_e = np.where(act_e, t_e + d, t_e)
        assert not (proved0 & hit).any(), "a proved ray hits: the proof is unsound"
        print(f"L{L}: hit {hit.mean():.3f}  samples/ray: exit proofs {cnt_exit.mean():.3f}, "
              f"directional {cnt_dir.mean():.3f}{'' if use_dir else ' (bin wider than a block: off)'}  "
              f"| proved at the first sample {proved0.mean():.3f}")


if __name__ == "__main__":
    main()
