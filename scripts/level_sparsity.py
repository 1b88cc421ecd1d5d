#!/usr/bin/env python3
"""How much of each cascade level is 'block-constant': per direction block, the fraction of probes whose
texel equals the block's most frequent value (the value every probe of the block takes when none of its
rays hits and its upper taps are block-constant too).  4096^2 N=6 demo frame (or --scene), committed
schedule.  Prints one JSON line."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--cascades", type=int, default=6)
    ap.add_argument("--scene", default="demo")
    a = ap.parse_args()
    from radiancecascade2dglobalillumination_amd import RC2DGI, scenes
    W, N = a.size, a.cascades
    if a.scene == "demo":
        c, e = scenes.demo(W, W)
    else:
        k, s = a.scene.split(":")
        c, e = scenes.random_scene(W, W, int(s), coverage={"random": 0.05, "dense": 0.35}[k])
    ctx = RC2DGI(W, W, cascade_count=N, ray_range=2.0)
    ctx.set_keep_levels(True)
    ctx.frame(c, e)
    ctx.sync()
    out = {"scene": a.scene, "levels": {}}
    for L in range(N):
        g = ctx.download_level(L)  # [CH, CW, 4] f32
        b = 1 << L
        bd = W // b
        v = g.view(np.uint32).reshape(b, bd, b, bd, 4).transpose(0, 2, 1, 3, 4).reshape(b * b, bd * bd, 4)
        # per block: the most frequent texel (as a 128-bit key)
        key = v[..., 0].astype(np.uint64) << np.uint64(32) | v[..., 1].astype(np.uint64)
        key2 = v[..., 2].astype(np.uint64) << np.uint64(32) | v[..., 3].astype(np.uint64)
        frac = []
        for i in range(b * b):
            kk = np.stack([key[i], key2[i]], 1)
            u, cnt = np.unique(kk, axis=0, return_counts=True)
            frac.append(cnt.max() / kk.shape[0])
        frac = np.array(frac)
        out["levels"][f"L{L}"] = {"mode_fraction_mean": round(float(frac.mean()), 4),
                                  "mode_fraction_min": round(float(frac.min()), 4)}
        print(L, out["levels"][f"L{L}"], file=sys.stderr, flush=True)
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
