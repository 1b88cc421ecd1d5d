#!/usr/bin/env python3
"""Per-level RC schedule probe: HIP-event time of one cascade level under candidate (variant, order)
pairs, every other level on the committed schedule, candidates interleaved over rounds in one process.

Usage: python scripts/sched_probe.py [--size 4096] [--cascades 6] [--ray-range 2] [--storage f32]
           [--rounds 3] [--frames 8] [--lib PATH] L:V:O [L:V:O ...]
  L level, V rc_variant, O rc_order code ("c" = the committed order of that level, "v" = the committed
  variant's; "all" = rc2dgi_autotune's 48 order candidates; a comma list of orders or variants expands to
  every pair).  Prints one JSON line per level.
"""
import argparse
import itertools
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def autotune_orders():
    """The order codes of rc2dgi_autotune's candidate list (kOrderCandidates in rc2dgi_capi.cpp)."""
    import re

    src = open(os.path.join(ROOT, "radiancecascade2dglobalillumination_amd", "csrc", "rc2dgi_capi.cpp")).read()
    body = src[src.index("kOrderCandidates[][4] = {"):]
    body = body[:body.index("};")]
    quads = re.findall(r"\{(\d+), (\d+), (\d+), (\d+)\}", body)
    return [int(px) | int(py) << 8 | int(dg) << 16 | int(m) << 24 for px, py, dg, m in quads]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--cascades", type=int, default=6)
    ap.add_argument("--ray-range", type=float, default=2.0)
    ap.add_argument("--storage", default="f32")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--tune", action="append", default=[])
    ap.add_argument("--xcd-chunks", default="", help="comma list of log2 XCD interleave chunks (order code bits 26-30) "
                    "to combine with every order candidate (0 = the contiguous split, 16 + t the Latin-square schedule, "
                    "c = keep the candidate's own)")
    ap.add_argument("--scene", default="demo", help="demo | random:<seed> | dense:<seed> (bench.py's scenes)")
    ap.add_argument("cands", nargs="+")
    a = ap.parse_args()
    import bench
    from radiancecascade2dglobalillumination_amd import RC2DGI, scenes

    W, H, N = a.size, a.height or a.size, a.cascades
    g = RC2DGI(W, H, cascade_count=N, ray_range=a.ray_range, storage=a.storage)
    if a.scene == "demo":
        color, emis = scenes.demo(W, H)
    else:
        kind, seed = a.scene.split(":")
        color, emis = scenes.random_scene(W, H, seed=int(seed), coverage={"random": 0.05, "dense": 0.35}[kind])
    g.upload("color", color)
    g.upload("emissive", emis)
    tun = json.load(open(bench.schedule_path(W, H, N, a.ray_range, a.storage)))
    bench.apply_schedule(g, tun, N)
    for kv in a.tune:
        k, v = kv.split("=")
        g.set_tuning(k, int(v))
    g.set_timing(1)
    per_level = {}
    for c in a.cands:
        L, vs, os_ = c.split(":")
        L = int(L)
        ol = [str(x) for x in autotune_orders()] if os_ == "all" else os_.split(",")
        chunks = [None if x == "c" else int(x) for x in a.xcd_chunks.split(",")] if a.xcd_chunks else [None]
        for v, o, lc in itertools.product(vs.split(","), ol, chunks):
            v = tun["rc_variant"][L] if v == "c" else int(v)
            o = tun["rc_order"][L] if o == "c" else int(o)
            if lc is not None:
                o = (o & ~(31 << 26)) | (lc << 26)
            if (v, o) not in per_level.setdefault(L, []):
                per_level[L].append((v, o))
    times = {(L, v, o): [] for L, cs in per_level.items() for v, o in cs}
    for _ in range(a.rounds):
        for L, cs in per_level.items():
            for v, o in cs:
                g.set_tuning(f"rc_variant_L{L}", v)
                g.set_tuning(f"rc_order_L{L}", o)
                g.do_rc2dgi()
                g.sync()
                for _ in range(a.frames):
                    g.do_rc2dgi()
                    times[(L, v, o)].append(g.pass_times(levels=N)["levels"][L])
            g.set_tuning(f"rc_variant_L{L}", tun["rc_variant"][L])
            g.set_tuning(f"rc_order_L{L}", tun["rc_order"][L])
    for L, cs in per_level.items():
        res = sorted(((round(float(np.median(times[(L, v, o)])), 4), v, o) for v, o in cs))
        print(json.dumps({"level": L, "size": [W, H], "N": N, "committed": [tun["rc_variant"][L], tun["rc_order"][L]],
                          "ms_variant_order": res}), flush=True)
    g.close()


if __name__ == "__main__":
    main()
