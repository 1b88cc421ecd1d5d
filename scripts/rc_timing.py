#!/usr/bin/env python3
"""Wave-lifetime split of k_rc_level per level and section (diagnostic build librc2dgi_timing.so,
python -m radiancecascade2dglobalillumination_amd._build timing): mean cycles per wave in
map (workgroup-map scalar load) / table (staging loads issued, proof table loaded and written to LDS) /
barrier / rays (origins, proofs) / march (lockstep)
/ tail (queue, barrier) / stage_write (LDS, barrier) / merge (shading loads, bilinear, store).
Run with the committed bench schedule; extra --tune KEY=VALUE knobs.  Prints one JSON line."""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RC2DGI_LIB", os.path.join(ROOT, "build", "diag", "librc2dgi_timing.so"))
SECTIONS = ["map", "table", "barrier", "rays", "march", "tail", "stage_write", "merge"]


def main():
    import numpy as np

    from radiancecascade2dglobalillumination_amd import RC2DGI, scenes
    from radiancecascade2dglobalillumination_amd.rc2dgi import load_library

    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--height", type=int, default=0, help="screen height (default: --size)")
    ap.add_argument("--cascades", type=int, default=6)
    ap.add_argument("--ray-range", type=float, default=2.0)
    ap.add_argument("--tune", action="append", default=[])
    a = ap.parse_args()
    W, N = a.size, a.cascades
    H = a.height or W
    L = load_library()
    L.rc2dgi_diag_stats.argtypes = [ctypes.c_void_p, ctypes.c_int]
    ctx = RC2DGI(W, H, cascade_count=N, ray_range=a.ray_range)
    sched = os.path.join(ROOT, "radiancecascade2dglobalillumination_amd", "tuning", f"{W}x{H}_N{N}_rr{a.ray_range:g}_f32.json")
    if os.path.exists(sched):
        tun = json.load(open(sched))
        for lv in range(N):
            ctx.set_tuning(f"rc_order_L{lv}", tun["rc_order"][lv])
            ctx.set_tuning(f"rc_variant_L{lv}", tun["rc_variant"][lv])
    for kv in a.tune:
        k, v = kv.split("=")
        ctx.set_tuning(k, int(v))
    c, e = scenes.demo(W, H)
    ctx.upload("color", c)
    ctx.upload("emissive", e)
    buf = np.zeros((16, 16), np.uint64)
    ctx.do_rc2dgi()
    ctx.sync()
    L.rc2dgi_diag_stats(buf.ctypes.data, 1)
    ctx.set_timing(True)
    ctx.do_rc2dgi()
    ctx.sync()
    raw = np.zeros(8 * (1 << 17) * 2, np.uint64)  # the per-workgroup records, before the reset below
    L.rc2dgi_diag_raw.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    L.rc2dgi_diag_raw(raw.ctypes.data, raw.size)
    L.rc2dgi_diag_stats(buf.ctypes.data, 1)
    lv_ms = ctx.pass_times(levels=N)["levels"]
    out = {"config": f"{W}x{H} N={N} rr={a.ray_range}", "tune": a.tune, "levels": {}}
    for lv in range(N):
        waves = int(buf[lv, 15])
        cyc = {s: round(float(buf[lv, i]) / max(waves, 1), 1) for i, s in enumerate(SECTIONS)}
        cyc["total"] = round(sum(cyc.values()), 1)
        out["levels"][f"L{lv}"] = {"ms": round(lv_ms[lv], 4), "waves": waves, "cycles_per_wave": cyc}
        print(f"L{lv} {lv_ms[lv]:.3f} ms waves {waves}: " + " ".join(f"{s} {cyc[s]:.0f}" for s in SECTIONS + ['total']),
              file=sys.stderr)
    # per-workgroup records (start / end on the 100 MHz clock, XCC id): per XCD the busy span and the summed
    # workgroup time, each XCD on its own clock
    for lv in range(min(N, 8)):
        rec = raw[(lv << 17) * 2:((lv + 1) << 17) * 2].reshape(-1, 2)
        rec = rec[rec[:, 1] != 0]
        if not len(rec):
            continue
        xcc = (rec[:, 0] >> np.uint64(60)).astype(int)
        t0 = (rec[:, 0] & np.uint64(0xFFFFFFFFFF)).astype(np.int64)
        t1 = (rec[:, 1] & np.uint64(0xFFFFFFFFFF)).astype(np.int64)
        spans, busy, ramp, tail = [], [], [], []
        for x in range(8):
            m = xcc == x
            if m.any():
                a0, a1 = t0[m], t1[m]
                spans.append(round(float(a1.max() - a0.min()) / 100.0, 1))
                busy.append(round(float((a1 - a0).sum()) / 100.0 / 1000.0, 2))
                # workgroups resident over time (10 ns ticks): the ramp until half the peak, the tail after the
                # last time it was above half the peak
                ev = np.concatenate([np.stack([a0, np.ones_like(a0)], 1), np.stack([a1, -np.ones_like(a1)], 1)])
                ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
                conc = np.cumsum(ev[:, 1])
                half = conc.max() / 2.0
                above = np.nonzero(conc >= half)[0]
                ramp.append(round(float(ev[above[0], 0] - a0.min()) / 100.0, 1))
                tail.append(round(float(a1.max() - ev[min(above[-1] + 1, len(ev) - 1), 0]) / 100.0, 1))
        out["levels"][f"L{lv}"]["xcd_span_us"] = spans
        out["levels"][f"L{lv}"]["xcd_wg_time_ms"] = busy
        out["levels"][f"L{lv}"]["xcd_ramp_us"] = ramp
        out["levels"][f"L{lv}"]["xcd_tail_us"] = tail
        print(f"L{lv} per XCD: span us {spans}  summed workgroup ms {busy}  ramp us {ramp}  tail (below half the "
              f"peak residency) us {tail}", file=sys.stderr)
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
