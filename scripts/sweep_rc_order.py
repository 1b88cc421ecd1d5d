#!/usr/bin/env python3
"""Sweep the RC workgroup order (tuning "rc_order_L<n>") per level at the bench workload.

Each candidate (px, py, dg) is set on every level (levels where it does not tile the grid fall
back to tile-major inside the library); per-level HIP-event times are collected over interleaved
rounds and the median per level is printed as one JSON line, with the best candidate per level.
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CANDIDATES = [(0, 0, 0), (1, 1, 16), (1, 1, 64), (2, 2, 16), (2, 2, 64), (4, 4, 4), (4, 4, 16), (4, 4, 64),
              (8, 8, 4), (8, 8, 16), (2, 2, 256), (4, 2, 32), (16, 1, 16), (1, 16, 16), (8, 8, 1), (16, 16, 1)]
FOCUS = [(0, 0, 0), (1, 16, 16), (1, 8, 16), (1, 16, 8), (1, 16, 32), (2, 8, 16), (1, 4, 16), (2, 16, 16),
         (1, 16, 4), (1, 8, 8), (1, 8, 32), (1, 32, 16), (1, 32, 8), (4, 4, 4), (2, 4, 4), (4, 8, 4), (2, 8, 8),
         (1, 8, 4), (2, 2, 8), (1, 4, 64), (1, 2, 64)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--cascades", type=int, default=6)
    ap.add_argument("--ray-range", type=float, default=2.0)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--focus", action="store_true", help="second-stage candidate list")
    a = ap.parse_args()
    global CANDIDATES
    if a.focus:
        CANDIDATES = FOCUS
    from radiancecascade2dglobalillumination_amd import RC2DGI, scenes

    W = H = a.size
    N = a.cascades
    ctx = RC2DGI(W, H, cascade_count=N, ray_range=a.ray_range)
    c, e = scenes.demo(W, H)
    ctx.upload("color", c)
    ctx.upload("emissive", e)
    ctx.set_timing(True)
    ctx.do_rc2dgi()
    ref = ctx.download("color")
    times = {k: [] for k in range(len(CANDIDATES))}
    for _ in range(a.rounds):
        for k, (px, py, dg) in enumerate(CANDIDATES):
            for L in range(N):
                ctx.set_tuning(f"rc_order_L{L}", px | (py << 8) | (dg << 16))
            ctx.do_rc2dgi()
            ctx.sync()
            for _ in range(a.steps):
                ctx.do_rc2dgi()
                times[k].append(ctx.pass_times(levels=N)["levels"])
    ok = bool(np.array_equal(ctx.download("color"), ref))
    med = {k: np.median(np.array(t), axis=0) for k, t in times.items()}
    best = [min(med, key=lambda k: med[k][L]) for L in range(N)]
    print(json.dumps({
        "sweep": "rc_order", "size": W, "N": N, "results_identical": ok,
        "candidates": [list(x) for x in CANDIDATES],
        "levels_ms": {str(CANDIDATES[k]): [round(float(x), 4) for x in m] for k, m in med.items()},
        "best_per_level": [list(CANDIDATES[b]) for b in best],
        "best_ms": [round(float(med[best[L]][L]), 4) for L in range(N)],
        "default_ms": [round(float(x), 4) for x in med[0]]}), flush=True)


if __name__ == "__main__":
    main()
