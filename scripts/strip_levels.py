#!/usr/bin/env python3
"""Per-level cost of row-strip sharding: the cascade phase of each in-process shard timed on its
own (rc2dgi_do_phase(2) after one group frame, one shard at a time, hipEvents per level), summed over the
shards, against the unsharded frame's levels.  Usage: strip_levels.py [size=8192] [N=8] [rayRange=64] [shards=8]
Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np

    from radiancecascade2dglobalillumination_amd import RC2DGI, scenes
    from radiancecascade2dglobalillumination_amd import rc2dgi as R

    a = sys.argv[1:]
    W = int(a[0]) if a else 8192
    N = int(a[1]) if len(a) > 1 else 8
    rr = float(a[2]) if len(a) > 2 else 64.0
    P = int(a[3]) if len(a) > 3 else 8
    sched = os.path.join(ROOT, "radiancecascade2dglobalillumination_amd", "tuning", f"{W}x{W}_N{N}_rr{rr:g}_f32.json")
    tun = json.load(open(sched)) if os.path.exists(sched) else None
    color, emis = scenes.demo(W, W)

    def make(k=None):
        g = RC2DGI(W, W, cascade_count=N, ray_range=rr)
        g.upload("color", color)
        g.upload("emissive", emis)
        if tun:
            sub = (tun.get("strips") or {}).get(str(P), {}) if k is not None else {}
            for L in range(N):
                g.set_tuning(f"rc_order_L{L}", (sub.get("rc_order") or tun["rc_order"])[L])
                g.set_tuning(f"rc_variant_L{L}", (sub.get("rc_variant") or tun["rc_variant"])[L])
        if k is not None:
            g.set_shard(k, P)
        g.set_timing(True)
        return g

    reps = 5
    whole = make()
    lv_w = np.full(N, 1e9)
    for _ in range(reps):
        whole.do_rc2dgi()
        whole.sync()
        t = whole.pass_times(levels=N)
        lv_w = np.minimum(lv_w, t["levels"])
    whole.close()
    shards = [make(k) for k in range(P)]
    R.do_group(shards)
    for g in shards:
        g.sync()
    per = np.zeros((P, N))
    rc = np.zeros(P)
    for k, g in enumerate(shards):
        best = np.full(N, 1e9)
        for _ in range(reps):
            g.do_phase(2)
            g.sync()
            best = np.minimum(best, g.pass_times(levels=N)["levels"])
        per[k] = best
    for g in shards:
        g.close()
    out = {"config": f"{W}x{W} N={N} rr={rr}", "shards": P, "whole_level_ms": [round(x, 4) for x in lv_w],
           "strip_sum_level_ms": [round(x, 4) for x in per.sum(0)],
           "ratio": [round(x, 3) for x in per.sum(0) / lv_w],
           "per_shard_level_ms": [[round(x, 4) for x in r] for r in per]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
