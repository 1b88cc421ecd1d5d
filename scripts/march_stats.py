#!/usr/bin/env python3
"""Lockstep efficiency of the RC march per level (diagnostic build librc2dgi_stats.so):
samples of live rays / ray slots the lockstep loop executed.  Prints one JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RC2DGI_LIB", os.path.join(ROOT, "build", "diag", "librc2dgi_stats.so"))


def main():
    import numpy as np

    from radiancecascade2dglobalillumination_amd import RC2DGI, scenes
    from radiancecascade2dglobalillumination_amd.rc2dgi import load_library

    W = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    rr = float(sys.argv[3]) if len(sys.argv) > 3 else 2.0
    skip = int(sys.argv[4]) if len(sys.argv) > 4 else 1  # tuning rc_skip (exit proofs)
    scene = sys.argv[5] if len(sys.argv) > 5 else "demo"  # demo | random:<seed> | dense:<seed> (bench.py --scene)
    L = load_library()
    L.rc2dgi_diag_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
    ctx = RC2DGI(W, W, cascade_count=N, ray_range=rr)
    ctx.set_tuning("rc_skip", skip)
    sched = os.path.join(ROOT, "radiancecascade2dglobalillumination_amd", "tuning", f"{W}x{W}_N{N}_rr{rr:g}_f32.json")
    if os.path.exists(sched):  # the committed schedule (tile shapes set the wave composition)
        tun = json.load(open(sched))
        for lv in range(N):
            ctx.set_tuning(f"rc_order_L{lv}", tun["rc_order"][lv])
            ctx.set_tuning(f"rc_variant_L{lv}", tun["rc_variant"][lv])
    if scene == "demo":
        c, e = scenes.demo(W, W)
    else:
        kind, seed = scene.split(":")
        c, e = scenes.random_scene(W, W, int(seed), coverage={"random": 0.05, "dense": 0.35}[kind])
    ctx.upload("color", c)
    ctx.upload("emissive", e)
    buf = np.zeros((16, 16), np.uint64)
    ctx.do_rc2dgi()
    ctx.sync()
    L.rc2dgi_diag_stats(buf.ctypes.data, 1)
    ctx.do_rc2dgi()
    ctx.sync()
    L.rc2dgi_diag_stats(buf.ctypes.data, 1)
    out = {}
    for lv in range(N):
        slots, samples, waves = (int(x) for x in buf.reshape(-1)[3 * lv:3 * lv + 3])  # P.stats[level * 3 + i]
        rays = 4 * W * W
        out[f"L{lv}"] = {"samples_per_ray": round(samples / rays, 3), "slot_iters_per_ray": round(slots / rays, 3),
                         "lockstep_efficiency": round(samples / max(slots, 1), 3),
                         "wave_iterations": round(slots / max(waves * 64 * 4, 1), 2)}
        b = buf.reshape(-1)[64 + 4 * lv:64 + 4 * lv + 4]
        out[f"L{lv}"].update({"rays_sampled": round(int(b[0]) / rays, 4), "probes_sampled": round(int(b[1]) / (W * W), 4),
                              "waves_sampled": round(int(b[2]) / max(waves, 1), 4),
                              "rays_hit_pre_tail": round(int(b[3]) / rays, 4)})
    print(json.dumps({"size": W, "N": N, "ray_range": rr, "rc_skip": skip, "scene": scene, "levels": out}))


if __name__ == "__main__":
    main()
