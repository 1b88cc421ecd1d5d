#!/usr/bin/env python3
"""bench.py -- RC-pass throughput (Mpixel*cascades/s) and full-pipeline fps of the MI355X
DoRC2DGI() at 4096^2, cascadeCount=6 (BASELINE.json metric).

One step = one DoRC2DGI() frame (RC2DGI.cs:267-406: ScreenUV, 12 JFA steps + distance
field, 6 cascade levels, blur + copy-back, merge + copy-back) over a synthetic painted
scene already resident in HBM (the reference's demo scene scaled to 4096^2).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--size 4096] [--cascades 6]

Multi-GPU: one process per GPU (torch.distributed.run), each rank renders its own scene
(the path has no exchange step at this size: replicas, "scaling": "weak"); rank 0 prints
the JSON line with the max-over-ranks time.

value = sum over ranks of CW*CH*N per frame * K / max-over-ranks( sum of the K RC-pass
HIP-event times ) -- t_RC as SURVEY.md §8d defines it: the hipEvent time of the N level
launches, recorded on the stream the kernels run on.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def b_rc(W, H, CW, CH, N, gi_bytes=16):
    """Algorithmic bytes of one RC pass: write G_L, read G_{L+1} once,
    read the distance field once per level (gi_bytes = 8 with RGBA16F cascades, 4 with RGBA8)."""
    return gi_bytes * CW * CH * (2 * N - 1) + 4 * W * H * N


def cpu_baseline(W, H, N, rr, budget_s=12.0):
    """The CPU port of the RC pass (oracle/, OpenMP on this host's cores), timed on a
    bounded sample of the same workload: whole-width row bands of every level."""
    import numpy as np

    import oracle
    from radiancecascade2dglobalillumination_amd import scenes

    p = oracle.Params(W=W, H=H, N=N, ray_range=rr)
    CW, CH, S = oracle.dims(p)
    color, emis = scenes.demo(W, H)
    j = oracle.screen_uv(color)
    mx = max(W, H)
    step = np.float32(1.0)
    for _ in range(S):
        step = np.float32(step * np.float32(0.5))
        j = oracle.jfa_step(j, float(step), float(np.float32(W) / mx), float(np.float32(H) / mx))
    dist = oracle.distance_field(j)
    dirs, sky = oracle.dir_tables(p), oracle.sky_table(p)
    offs, o = [], 0
    for L in range(N):
        offs.append(o)
        o += 4 << (2 * L)
    upper = np.zeros((CH, CW, 4), np.float32)
    upper[..., 3] = 1.0
    out = np.zeros((CH, CW, 4), np.float32)
    rows = 8
    done_px, spent = 0, 0.0
    while True:
        t0 = time.perf_counter()
        for L in range(N - 1, -1, -1):
            r0 = (CH // 2) - rows // 2
            oracle.rc_level(p, L, upper if L < N - 1 else None, color, emis, dist, out,
                            np.ascontiguousarray(dirs[offs[L]:]), sky, r0, r0 + rows)
        dt = time.perf_counter() - t0
        done_px += CW * rows * N
        spent += dt
        if spent >= budget_s or rows >= CH:
            break
        rows = min(CH, int(rows * max(2.0, min(8.0, (budget_s - spent) / max(dt, 1e-3) / 2))))
    return dict(value=round(done_px / spent / 1e6, 3), unit="Mpixel*cascades/s", cores=oracle.num_threads(),
                kind="port",
                sample=f"RC pass of the same {W}x{H} N={N} demo frame, whole-width row bands through all {N} "
                       f"levels ({done_px / (CW * N):.0f} rows/level in total, {spent:.1f} s, CPU restatement "
                       f"oracle/rc2dgi_oracle.c, {platform.processor() or platform.machine()})")


# Random 128-byte line requests one MI355X sustains (scripts/gather_ceiling.hip,
# profiles/r01/gather_ceiling.txt): table resident in every XCD's L2 vs in the Infinity Cache
# (mean of the 16 MB and 32 MB rows).
GATHER_L2_GLINES, GATHER_MALL_GLINES = 260.0, 73.0


def tuning_or_none(ctx, key):
    """A tuning key the library may not know (A/B runs against older builds): its value, or None."""
    from radiancecascade2dglobalillumination_amd import RC2DGIError

    try:
        return ctx.get_tuning(key)
    except RC2DGIError:
        return None


def pmc_key(W, H, N, ray_range, storage, scene, orders, variants, knobs=None):
    """What a committed PMC record was measured on: counters describe one configuration, scene and schedule
    (the march's line requests and instructions follow the scene's occluders and the workgroup orders), so a
    bench line carries them only when all of these match (profiles/rc_level_pmc.json, scripts/pmc_summary.py)."""
    return {"config": f"{W}x{H}_N{N}", "ray_range": float(ray_range), "storage": storage, "scene": scene,
            "rc_order": [int(x) for x in orders] if orders else "default",
            "rc_variant": [int(x) for x in variants], "knobs": dict(sorted((knobs or {}).items()))}


def find_pmc_record(path, key):
    """The record of profiles/rc_level_pmc.json measured on exactly `key` (pmc_key), or None."""
    if not os.path.exists(path):
        return None
    with open(path) as f:
        doc = json.load(f)
    for rec in doc.get("records", []):
        if rec.get("key") == key:
            return rec
    return None


def gather_roofline(rec, N, level_ms):
    """The march-bound levels' L1->L2 line-request rate (PMC l2_requests from the committed profile
    over this run's level times) against the random-gather ceiling blended by their L2 hit rate
    (DESIGN.md §5.2).  The upper half of the levels, where the distance gathers dominate."""
    lv = rec.get("per_level", {})
    top = list(range(N // 2, N))
    req = [lv.get(f"k_rc_level L{L}", {}).get("l2_requests") for L in top]
    hit = [lv.get(f"k_rc_level L{L}", {}).get("l2_hit") for L in top]
    if any(x is None for x in req + hit):
        return None
    t = sum(level_ms[L] for L in top) / 1e3
    h = sum(r * x for r, x in zip(req, hit)) / sum(req)
    achieved = sum(req) / t / 1e9
    ceiling = 1.0 / (h / GATHER_L2_GLINES + (1.0 - h) / GATHER_MALL_GLINES)
    return {"kernel": f"k_rc_level L{top[0]}-L{top[-1]}", "achieved": round(achieved, 1), "peak": round(ceiling, 1),
            "unit": "G line requests/s", "frac": round(achieved / ceiling, 4), "l2_hit": round(h, 4),
            "source": "profiles/rc_level_pmc.json (TCC_HIT+TCC_MISS per launch), profiles/r01/gather_ceiling.txt"}


# VALU issue peak: 256 CUs x 4 SIMD-32s; a plain wave64 VALU instruction takes 2 cycles once two or more
# waves share the SIMD (MI355X_MICROARCH.md "Wave scheduling" and the constants table), at the 2.4 GHz
# peak engine clock.  Packed f32 (v_pk_*), transcendental and 64-bit instructions cost more: each
# level's mean cycles per VALU instruction comes from its kernel's instruction mix
# (scripts/isa_mix.py -> profiles/rc_isa_mix.json; 2.0 when absent).
VALU_CLOCK_GHZ, VALU_SIMDS = 2.4, 256 * 4
VALU_PEAK_GINSTS = VALU_SIMDS * VALU_CLOCK_GHZ / 2.0


def valu_roofline(rec, N, level_ms, mix=None):
    """The RC pass against the VALU issue rate: wave instructions per frame (PMC
    SQ_INSTS_VALU per level launch from the committed profile), priced at each level's mean issue
    cycles per instruction, over this run's level times."""
    lv = rec.get("per_level", {})
    ins = [lv.get(f"k_rc_level L{L}", {}).get("valu_insts") for L in range(N)]
    if any(x is None for x in ins):
        return None
    cyc = [((mix or {}).get("levels", {}).get(f"L{L}", {}).get("valu_cycles_per_inst") or 2.0) for L in range(N)]
    t = sum(level_ms) / 1e3
    busy_s = sum(i * c for i, c in zip(ins, cyc)) / (VALU_SIMDS * VALU_CLOCK_GHZ * 1e9)  # all SIMDs issuing
    achieved = sum(ins) / t / 1e9
    return {"kernel": "k_rc_level (all levels)", "achieved": round(achieved, 1), "peak": round(VALU_PEAK_GINSTS, 1),
            "unit": "G VALU wave-instructions/s (peak: plain 2-cycle instructions)",
            "frac": round(busy_s / t, 4), "floor_ms": round(busy_s * 1e3, 4),
            "cycles_per_inst": [round(c, 3) for c in cyc],
            "per_level_frac": [round(i * c / (VALU_SIMDS * VALU_CLOCK_GHZ * 1e9) / (m / 1e3), 4)
                               for i, c, m in zip(ins, cyc, level_ms)],
            "source": "profiles/rc_level_pmc.json (SQ_INSTS_VALU per launch), profiles/rc_isa_mix.json"}


def input_costs(ctx, W, H, color, emis, reps=5):
    """Per-frame cost of producing the painted inputs (outside the timed frames): painting the
    demo scene on the device (rc2dgi_paint) vs uploading both textures from host
    memory (the reference app's path, PCIe).  Restores the bench's own inputs afterwards."""
    from radiancecascade2dglobalillumination_amd import scenes

    cc, cp, ec, ep = scenes.demo_prims(W, H)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.paint("color", cp, cc)
        ctx.paint("emissive", ep, ec)
    ctx.sync()
    paint_ms = (time.perf_counter() - t0) * 1e3 / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.upload("color", color)
        ctx.upload("emissive", emis)
    ctx.sync()
    upload_ms = (time.perf_counter() - t0) * 1e3 / reps
    return {"device_paint_ms": round(paint_ms, 3), "host_upload_ms": round(upload_ms, 3),
            "note": "both input textures per frame; not part of value"}


def sweep_rc(ctx, N, steps, rounds=3):
    """Per-level HIP-event times of every RC tile variant, interleaved over rounds in one
    process (cdna_hip_programming.md §5.4 rule 24); prints one JSON line."""
    import numpy as np

    nv = ctx.get_tuning("rc_variant_count")
    times = {v: [] for v in range(nv)}
    for _ in range(rounds):
        for v in range(nv):
            ctx.set_tuning("rc_variant", v)
            ctx.do_rc2dgi()
            ctx.sync()
            for _ in range(steps):
                ctx.do_rc2dgi()
                times[v].append(ctx.pass_times(levels=N)["levels"])
    from radiancecascade2dglobalillumination_amd.rc2dgi import load_library

    lib = load_library()
    med = {v: np.median(np.array(t), axis=0).tolist() for v, t in times.items()}
    best = [min(range(nv), key=lambda v: med[v][L]) for L in range(N)]
    print(json.dumps({"sweep": "rc_variant", "levels_ms": {str(v): [round(x, 4) for x in m] for v, m in med.items()},
                      "best_per_level": best, "best_total_ms": round(sum(med[best[L]][L] for L in range(N)), 4),
                      "names": [lib_variant_name(v) for v in range(nv)]}), flush=True)


def schedule_path(W, H, N, ray_range=2.0, storage="f32"):
    """The committed RC schedule (per-level rc_order / rc_variant) for a configuration: picked by
    rc2dgi_autotune on an MI355X (bench.py --autotune --save-tuning), loaded by the bench and by
    the parity tests, so the schedule that is timed is the schedule that is tested."""
    return os.path.join(ROOT, "radiancecascade2dglobalillumination_amd", "tuning",
                        f"{W}x{H}_N{N}_rr{ray_range:g}_{storage}.json")


def lib_variant_name(v):
    names = ["16x16x1", "16x8x2", "16x16x2", "32x8x1", "64x4x1", "8x8x1", "32x8x2", "16x16x1d2", "16x16x1d4",
             "16x8x1d2", "32x8x1d2", "16x8x1d4", "8x8x1d4", "16x16x1u", "16x16x1ut", "16x16x1t",
             "16x16x1up", "16x16x1un", "16x16x1p", "16x16x1n", "32x16x1", "16x32x1", "32x32x1", "32x16x1u",
             "32x32x1u"]
    return names[v] if v < len(names) else str(v)


def bench_batch(a, rank, local, world):
    """configs[4]-style batch: a.batch independent scenes per GPU, one context and stream
    each, all frames in flight together; timed by wall clock (streams overlap)."""
    import torch

    from radiancecascade2dglobalillumination_amd import RC2DGI, scenes
    from radiancecascade2dglobalillumination_amd import dist as rdist

    W, H, N = a.size, a.height or a.size, a.cascades
    items = rdist.shard(a.batch * world, rank, world)
    ctxs = []
    for it in items:
        c, e = scenes.random_scene(W, H, seed=rdist.scene_seed(it))
        g = RC2DGI(W, H, cascade_count=N, ray_range=a.ray_range, device=local)
        g.upload("color", c)
        g.upload("emissive", e)
        ctxs.append(g)
    CW, CH = ctxs[0].cascade_resolution
    if a.batch_streams == 1 and len(ctxs) > 1:  # every scene on one stream: frames back to back
        shared = torch.cuda.Stream(device=local)
        for g in ctxs:
            g.set_stream(shared.cuda_stream)
    committed = schedule_path(W, H, N, a.ray_range)
    if ctxs and not a.no_autotune and not a.autotune and os.path.exists(committed):
        with open(committed) as f:  # the committed schedule of this size (tested by the parity suite)
            tun = json.load(f)
        for g in ctxs:
            apply_schedule(g, tun, N)
    elif ctxs and not a.no_autotune:  # setup: one context picks the schedule, the others reuse it
        ctxs[0].autotune(3)
        for g in ctxs[1:]:
            for L in range(N):
                for k in (f"rc_order_L{L}", f"rc_variant_L{L}"):
                    g.set_tuning(k, ctxs[0].get_tuning(k))
    for _ in range(a.warmup):
        for g in ctxs:
            g.do_rc2dgi()
    for g in ctxs:
        g.sync()
    rdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        for g in ctxs:
            g.do_rc2dgi()
    for g in ctxs:
        g.sync()
    torch.cuda.synchronize()
    rdist.barrier()
    wall = rdist.max_over_ranks([time.perf_counter() - t0], device="cuda")[0]
    units = CW * CH * N * a.steps * len(items) * world
    if rank == 0:
        print(json.dumps({
            "metric": "Mpixel*cascades/s (whole DoRC2DGI frames, batch of independent scenes)",
            "value": round(units / wall / 1e6, 1), "unit": "Mpixel*cascades/s", "n_gpus": world, "pg_world": pg_world(),
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(wall * 1e3 / a.steps, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic random scenes resident in HBM",
            "config": {"workload": f"batch {a.batch} x DoRC2DGI {W}x{H} N={N} per GPU, "
                                   + ("one shared stream" if a.batch_streams == 1 else "one stream each"),
                       "parallelism": f"replicas{world}x{a.batch}"},
            "frames_per_s": round(a.steps * len(items) * world / wall, 2)}), flush=True)
    for g in ctxs:
        g.close()


def apply_schedule(g, tun, N, shards=1):
    """Per-level rc_order / rc_variant of a committed schedule.  A schedule may carry a row-strip
    entry ("strips": {"<shards>": {"rc_variant": [...], "rc_order": [...]}}) for the shard contexts
    of that many strips: a shard computes a band of every block's rows, so the tile height that
    wastes the fewest rows can differ from the whole frame's pick (results are identical either way)."""
    sub = (tun.get("strips") or {}).get(str(shards), {}) if shards > 1 else {}
    for L in range(N):
        g.set_tuning(f"rc_order_L{L}", (sub.get("rc_order") or tun["rc_order"])[L])
        g.set_tuning(f"rc_variant_L{L}", (sub.get("rc_variant") or tun["rc_variant"])[L])
    for k, v in {**tun.get("knobs", {}), **sub.get("knobs", {})}.items():  # optional tuning knobs (rc_skip, ...)
        g.set_tuning(k, int(v))


def bench_strips(a, rank, local, world):
    """SURVEY §8e / BASELINE configs[3]: ONE frame split into row strips, one shard per rank
    (strong scaling).  Ranks exchange their distRT strips over RCCL inside librc2dgi
    (rc2dgi_shard_connect).  With one process and --shards P > 1 the P shards run as
    in-process contexts on the one GPU (rc2dgi_do_group): the rehearsal of the decomposition,
    whose time is the sum of the shards' work (redundant halo rows included)."""
    import numpy as np
    import torch

    from radiancecascade2dglobalillumination_amd import RC2DGI, scenes
    from radiancecascade2dglobalillumination_amd import dist as rdist
    from radiancecascade2dglobalillumination_amd import rc2dgi as R

    W, H, N = a.size, a.height or a.size, a.cascades
    color, emis = scenes.demo(W, H)  # the same scene on every rank: one frame
    virtual = world == 1 and a.shards > 1
    nsh = a.shards if virtual else world

    committed = schedule_path(W, H, N, a.ray_range, a.storage)
    tun = None
    if not a.autotune and not a.no_autotune and os.path.exists(committed):
        with open(committed) as f:
            tun = json.load(f)  # the whole frame's committed schedule carries over to the shards

    def make(k):
        g = RC2DGI(W, H, cascade_count=N, ray_range=a.ray_range, device=local)
        g.upload("color", color)
        g.upload("emissive", emis)
        if tun:
            apply_schedule(g, tun, N, nsh)
        elif not a.no_autotune:
            g.autotune(1)  # on the whole frame; the orders carry over to the shard
        for kv in a.tune:
            key, v = kv.split("=")
            g.set_tuning(key, int(v))
        g.set_shard(k, nsh)
        return g

    free0 = torch.cuda.mem_get_info(local)[0]  # (device bytes the shard contexts hold, measured after the warmup)
    if virtual:
        ctxs = [make(k) for k in range(nsh)]
        run = lambda: R.do_group(ctxs)  # noqa: E731
    else:
        g = make(rank)
        uid = [R.shard_unique_id() if rank == 0 else None]
        if world > 1:
            import torch.distributed as dist

            dist.broadcast_object_list(uid, src=0)
        g.connect(uid[0])
        ctxs = [g]
        run = g.do_rc2dgi
    CW, CH = ctxs[0].cascade_resolution
    for _ in range(a.warmup):
        run()
    for g in ctxs:
        g.sync()
    shard_bytes = (free0 - torch.cuda.mem_get_info(local)[0]) // len(ctxs)
    rdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        run()
    for g in ctxs:
        g.sync()
    torch.cuda.synchronize()
    rdist.barrier()
    wall = rdist.max_over_ranks([time.perf_counter() - t0], device="cuda")[0]
    units = CW * CH * N * a.steps  # one frame per step, whatever the shard count
    cfg_line = {"rc_variant": [ctxs[0].get_tuning(f"rc_variant_L{L}") for L in range(N)],
                "strip_tables": tuning_or_none(ctxs[0], "strip_tables_active"),
                "blur_strip_sized": tuning_or_none(ctxs[0], "blur_strip_sized"),
                "cascade_banded": tuning_or_none(ctxs[0], "cascade_banded")}
    for g in ctxs:
        g.close()
    mem = {"device_bytes_per_shard": int(shard_bytes)}
    if rank == 0 and nsh > 1:  # the same frame as one unsharded context, for the per-shard fraction
        free1 = torch.cuda.mem_get_info(local)[0]
        g = RC2DGI(W, H, cascade_count=N, ray_range=a.ray_range, device=local)
        g.upload("color", color)
        g.upload("emissive", emis)
        if tun:
            apply_schedule(g, tun, N)
        g.do_rc2dgi()
        g.sync()
        whole = free1 - torch.cuda.mem_get_info(local)[0]
        g.close()
        mem.update(device_bytes_one_context=int(whole), shard_memory_frac=round(shard_bytes / whole, 3))
    if rank == 0:
        print(json.dumps({
            "metric": f"Mpixel*cascades/s (whole DoRC2DGI frame, row strips) at {W}x{H}, cascadeCount={N}",
            "value": round(units / wall / 1e6, 1), "unit": "Mpixel*cascades/s", "n_gpus": world, "pg_world": pg_world(),
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(wall * 1e3 / a.steps, 4),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": f"synthetic (reference demo scene painted at {W}x{H}, resident in HBM)",
            "config": {"workload": f"DoRC2DGI {W}x{H} cascadeCount={N} rayRange={a.ray_range}, row strips",
                       "shards": nsh, "parallelism": f"strips{nsh}" + ("-in-process" if virtual else "-rccl"),
                       **cfg_line},
            **mem,
            "frames_per_s": round(a.steps / wall, 2)}), flush=True)


def strips_launch_check(a, rank, world):
    """--mode strips --launch-check: the row-strip exchange of one frame rehearsed over the process
    group without a GPU: every JumpFlood step's transfers of the library's plan (rc2dgi_plan_jfa_exchange) as
    point-to-point messages carrying the global rows they stand for, checked at the receiver against the plan's
    window / block layout, and every row the own strip's taps read (JumpFlood.fs, NEAREST + REPEAT) own or
    delivered; then the distRT strips (all-gather) partition the screen.  Returns a summary dict."""
    import math

    import numpy as np
    import torch
    import torch.distributed as dist

    from radiancecascade2dglobalillumination_amd import rc2dgi as R

    W, H, N = a.size, a.height or a.size, a.cascades
    (y0, y1), = R.plan_rows(W, H, N, 1.5, rank, world, R.PLAN_MERGE)
    S = int(math.log(max(W, H)) / math.log(2))  # RC2DGI.cs:290 (double)
    mx = max(W, H)
    aspx = np.float32(W) / np.float32(mx)  # peekUV.y = v + y * _Aspect.x * _StepSize (JumpFlood.fs:20)
    n_xfers = n_rows = 0
    step = np.float32(0.5)
    for t in range(1, S):
        step = np.float32(step * np.float32(0.5))
        info, xf = R.plan_jfa_exchange(W, H, N, world, t)
        bufs, row0 = R.plan_jfa_window(W, H, N, rank, world, t)

        def glob(buf, local):  # global row of a local row of this shard's buffer `buf` at step t
            base = (y0 - info["m"]) if buf == 0 else row0[bufs.index(buf)]
            return (base + local) % H

        held = set(range(y0, y1))
        reqs, inbox = [], []
        for tag, (src, src_row, rows, dst, dst_buf, dst_row) in enumerate(xf):
            if src == rank:
                g = [(y0 - info["m"] + src_row + k) % H for k in range(rows)]
                assert all(y0 <= r < y1 for r in g), f"step {t}: rank {rank} would send rows it does not own"
                if dst == rank:
                    assert [glob(dst_buf, dst_row + k) for k in range(rows)] == g, f"step {t}: local copy lands wrong"
                    held.update(g)
                else:
                    reqs.append(dist.isend(torch.tensor(g, dtype=torch.int64), dst, tag=tag))
                n_xfers += 1
                n_rows += rows
            elif dst == rank:
                buf = torch.empty(rows, dtype=torch.int64)
                reqs.append(dist.irecv(buf, src, tag=tag))
                inbox.append((buf, dst_buf, dst_row, rows))
        for r in reqs:
            r.wait()
        for buf, dst_buf, dst_row, rows in inbox:
            want = [glob(dst_buf, dst_row + k) for k in range(rows)]
            assert buf.tolist() == want, f"step {t}: rank {rank} received rows {buf.tolist()[:4]} for {want[:4]}"
            held.update(want)
        # the rows of J_{t-1} the own strip's taps read (JumpFlood.fs: NEAREST + REPEAT of v + offset)
        v = (np.arange(y0, y1, dtype=np.float32) + np.float32(0.5)) / np.float32(H)
        need = set()
        for k in (-1, 0, 1):
            x = (v + np.float32(np.float32(np.float32(k) * aspx) * step)).astype(np.float32)
            if H & (H - 1) == 0:
                r = np.floor(x * np.float32(H)).astype(np.int64) % H
            else:
                f = (x - np.floor(x)).astype(np.float32)
                r = np.minimum(np.floor(f * np.float32(H)).astype(np.int64), H - 1)
            need |= set(int(q) for q in r)
        missing = need - held
        assert not missing, f"step {t}: rank {rank} taps rows {sorted(missing)[:4]} nobody delivered"
    strips = [None] * world
    dist.all_gather_object(strips, (y0, y1))  # the distRT exchange: every shard gets every strip
    assert sorted(strips)[0][0] == 0 and sorted(strips)[-1][1] == H
    assert all(p[1] == q[0] for p, q in zip(sorted(strips), sorted(strips)[1:]))
    tot = torch.tensor([float(n_xfers), float(n_rows)])
    dist.all_reduce(tot)
    return {"steps_checked": S - 1, "transfers": int(tot[0]), "rows_exchanged": int(tot[1]),
            "strips": [list(p) for p in strips]}


def spawn_ranks(n):
    """bench.py --gpus N outside torch.distributed.run: run N ranks of this same command line under
    it (one process per GPU, rendezvous on 127.0.0.1) as a child, and return its exit code."""
    import socket
    import subprocess

    with socket.socket() as s:  # a free port for the rendezvous
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def pg_world():
    """World size of the initialised process group (1 without one): what the line's n_gpus is."""
    import torch.distributed as dist

    return dist.get_world_size() if dist.is_initialized() else 1


def finish_pg():
    import torch.distributed as dist

    if dist.is_initialized():
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--cascades", type=int, default=6)
    ap.add_argument("--ray-range", type=float, default=2.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--sweep-rc", action="store_true",
                    help="time every RC tile variant per level (interleaved rounds) instead of the bench line")
    ap.add_argument("--scene", default="demo", help="demo | random:<seed> | dense:<seed> (>= 25 %% occluders)")
    ap.add_argument("--batch", type=int, default=0,
                    help="scenes per GPU, one context each (BASELINE configs[4] batch mode)")
    ap.add_argument("--batch-streams", type=int, default=1,
                    help="batch mode: 0 = one stream per scene (frames overlap), 1 = all scenes on one stream")
    ap.add_argument("--mode", default="replicas", choices=("replicas", "strips"),
                    help="strips: one frame split into row strips over the ranks (BASELINE configs[3])")
    ap.add_argument("--storage", default="f32", choices=("f32", "f16", "rgba8"),
                    help="f16: giRT1/2 as RGBA16F (RC2DGI.cs:105-106, SURVEY 8 f4); rgba8: every render texture "
                         "RGBA8 with GL unorm8 arithmetic, the literal app (SURVEY 8 f3)")
    ap.add_argument("--no-autotune", action="store_true",
                    help="keep the library's default RC schedule (no committed schedule, no autotune)")
    ap.add_argument("--autotune", action="store_true",
                    help="time the RC schedule candidates in setup instead of loading the committed schedule "
                         "(radiancecascade2dglobalillumination_amd/tuning/<W>x<H>_N<N>_rr<rayRange>_<storage>.json)")
    ap.add_argument("--save-tuning", default="", help="write the chosen per-level rc_order / rc_variant (JSON)")
    ap.add_argument("--load-tuning", default="",
                    help="apply per-level rc_order / rc_variant from a --save-tuning file instead of autotuning "
                         "(profiler runs replay the bench's schedule)")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="extra rc2dgi_set_tuning knob applied after the schedule (e.g. rc_skip=0), repeatable")
    ap.add_argument("--shards", type=int, default=1,
                    help="strips on one process: run this many shards as in-process contexts")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="process-group backend (nccl = RCCL on the GPU box; gloo only with --launch-check)")
    ap.add_argument("--launch-check", action="store_true",
                    help="no GPU work: bring up the ranks, print the world size the line would carry")
    a = ap.parse_args()

    # --gpus N is the rank count.  Without a torch.distributed.run environment, spawn it here as a
    # child process -- before anything touches the GPU -- and exit with its code; inside one, a
    # world size other than N is an error, never a silent one-GPU line.
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        return spawn_ranks(a.gpus)
    if env_world is not None and int(env_world) != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={env_world}", file=sys.stderr)
        return 2

    from radiancecascade2dglobalillumination_amd import dist as rdist

    if a.launch_check:
        rank, local, world = rdist.init(a.backend)
        got = rdist.max_over_ranks([float(rank)], device="cpu" if a.backend == "gloo" else "cuda")
        extra = {}
        if a.mode == "strips" and world > 1:
            extra = {"mode": "strips", "config": f"{a.size}x{a.height or a.size} N={a.cascades}",
                     **strips_launch_check(a, rank, world)}
        if rank == 0:
            print(json.dumps({"launch_check": True, "n_gpus": world, "pg_world": pg_world(), "backend": a.backend,
                              "max_rank": int(got[0]), **extra}), flush=True)
        finish_pg()
        return 0

    import numpy as np
    import torch

    from radiancecascade2dglobalillumination_amd import RC2DGI, scenes

    rank, local, world = rdist.init("nccl")
    if a.batch:
        return bench_batch(a, rank, local, world)
    if a.mode == "strips":
        return bench_strips(a, rank, local, world)

    W = a.size
    H = a.height or a.size
    N = a.cascades
    if a.scene == "demo":
        color, emis = scenes.demo(W, H, t=3.0 + 0.25 * rank)  # one independent scene per rank
        scene_desc = f"reference demo scene painted at {W}x{H}"
    else:
        kind, seed = a.scene.split(":")
        cov = {"random": 0.05, "dense": 0.35}[kind]  # dense: >= 25 % of the texels occluders
        color, emis = scenes.random_scene(W, H, seed=int(seed) + rank, coverage=cov)
        scene_desc = f"random scene {kind}:{seed} at {W}x{H}"
    # fraction of occluder texels (ScreenUV.fs: any colour channel above zero)
    coverage = float(np.count_nonzero(np.any(color[..., :3] > 0, axis=-1)) / (W * H))
    ctx = RC2DGI(W, H, cascade_count=N, ray_range=a.ray_range, device=local, storage=a.storage)
    CW, CH = ctx.cascade_resolution
    # inputs resident in HBM before the timed region
    ctx.upload("color", color)
    ctx.upload("emissive", emis)
    committed = schedule_path(W, H, N, a.ray_range, a.storage)
    if not a.load_tuning and not a.autotune and not a.no_autotune and os.path.exists(committed):
        a.load_tuning = committed  # the committed schedule: the one the parity tests check at this size
    def apply_tunes():
        for kv in a.tune:
            k, v = kv.split("=")
            ctx.set_tuning(k, int(v))

    apply_tunes()  # (before an autotune, so it tunes under these knobs)
    if a.load_tuning:
        with open(a.load_tuning) as f:
            tun = json.load(f)
        apply_schedule(ctx, tun, N)
        orders = tun["rc_order"]
    else:
        orders = None if a.no_autotune else ctx.autotune(3)  # setup: schedule choice, results identical
    apply_tunes()  # (and after a schedule, over its knobs)
    variants = [ctx.get_tuning(f"rc_variant_L{L}") for L in range(N)]
    orders = [ctx.get_tuning(f"rc_order_L{L}") for L in range(N)] if orders else None
    if a.save_tuning and rank == 0:
        with open(a.save_tuning, "w") as f:
            json.dump({"config": f"{W}x{H} N={N} rayRange={a.ray_range} {a.storage}",
                       "rc_order": [ctx.get_tuning(f"rc_order_L{L}") for L in range(N)], "rc_variant": variants,
                       **({"knobs": {kv.split("=")[0]: int(kv.split("=")[1]) for kv in a.tune}} if a.tune else {})}, f)
    ctx.set_timing(True)
    if a.sweep_rc:
        sweep_rc(ctx, N, a.steps, rounds=3)
        return
    for _ in range(a.warmup):
        ctx.do_rc2dgi()
    ctx.sync()

    # The timed steps carry events around the passes only (timing mode 2): an event between two
    # levels idles the GPU ~5 us (rocprofv3 trace), which a frame without timing does not.
    ctx.set_timing(2)
    rc_ms, tot_ms, lvl_ms = [], [], np.zeros(N)
    pass_acc = {}
    rdist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ctx.do_rc2dgi()
        t = ctx.pass_times()  # waits for this frame's last event
        rc_ms.append(t["rc"])
        tot_ms.append(t["total"])
        for k, v in t.items():
            pass_acc[k] = pass_acc.get(k, 0.0) + v
    ctx.sync()
    torch.cuda.synchronize()
    rdist.barrier()
    wall = time.perf_counter() - t0
    # per-level breakdown (and the gather / VALU rooflines priced on it): further frames with an
    # event around every level, after the timed region
    ctx.set_timing(True)
    lvl_steps = max(1, min(a.steps, 20))
    for _ in range(lvl_steps):
        ctx.do_rc2dgi()
        lvl_ms += np.array(ctx.pass_times(levels=N)["levels"])
    lvl_ms *= a.steps / lvl_steps  # (as a sum over a.steps frames, like rc_ms)
    t_rc, t_tot, wall = rdist.max_over_ranks([sum(rc_ms), sum(tot_ms), wall], device="cuda")
    units = CW * CH * N * a.steps * world
    value = units / (t_rc / 1e3) / 1e6
    bytes_launch = b_rc(W, H, CW, CH, N, {"f32": 16, "f16": 8, "rgba8": 4}[a.storage]) / N
    avg_launch_s = (t_rc / 1e3) / (a.steps * N)
    achieved = bytes_launch / avg_launch_s / 1e9
    traffic, gather, valu = None, None, None
    knobs = {kv.split("=")[0]: int(kv.split("=")[1]) for kv in a.tune}
    if a.load_tuning:
        knobs = {**tun.get("knobs", {}), **knobs}
    key = pmc_key(W, H, N, a.ray_range, a.storage, a.scene, orders, variants, knobs)
    rec = find_pmc_record(os.path.join(ROOT, "profiles", "rc_level_pmc.json"), key)
    chain = bool(tuning_or_none(ctx, "rc_chain"))
    if rec is not None and not chain:
        traffic = rec.get("hbm_bytes_per_launch")
        gather = gather_roofline(rec, N, lvl_ms / a.steps)
        mixp = os.path.join(ROOT, "profiles", "rc_isa_mix.json")
        mix = json.load(open(mixp)) if os.path.exists(mixp) else None
        if mix is not None and mix.get("key") != {k: key[k] for k in ("config", "rc_variant")}:
            mix = None  # (another schedule's instruction mix: price every instruction at 2 cycles instead)
        valu = valu_roofline(rec, N, lvl_ms / a.steps, mix)
    line = {
        "metric": (f"Mpixel*cascades/s (RC pass) at {W}^2, cascadeCount={N}" if W == H else
                   f"Mpixel*cascades/s (RC pass) at {W}x{H}, cascadeCount={N}"),
        "value": round(value, 1),
        "unit": "Mpixel*cascades/s",
        "n_gpus": world, "pg_world": pg_world(),
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(wall * 1e3 / a.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": {"f32": "f32", "f16": "f32 (RGBA16F cascade storage)",
                  "rgba8": "f32 arithmetic, RGBA8 render textures (8-bit blends / filtering)"}[a.storage],
        "data": f"synthetic ({scene_desc}, resident in HBM)",
        "config": {"workload": f"DoRC2DGI {W}x{H} cascadeCount={N} rayRange={a.ray_range}", "screen": [W, H],
                   "scene": a.scene, "occluder_coverage": round(coverage, 4),
                   "cascade_resolution": [CW, CH], "cascade_count": N, "ray_range": a.ray_range,
                   "parallelism": f"replicas{world}",
                   "rc_order": orders or "default", "rc_variant": variants,
                   "rc_pal": ctx.get_tuning("rc_pal"),
                   "rc_skip": ctx.get_tuning("rc_skip"),
                   "rc_schedule": (os.path.relpath(a.load_tuning, ROOT) if a.load_tuning else
                                   ("default" if a.no_autotune else "autotune in setup"))},
        "pmc_key": key,
        "rc_ms_per_frame": round(t_rc / a.steps, 4),
        "rc_level_ms": [round(x / a.steps, 4) for x in lvl_ms.tolist()],
        "rc_level_timing": (f"{lvl_steps} further frames with an event around every level (timing mode 1)" +
                            ("; cascade chain on: levels N-2..0 run in ONE launch, booked on level N-2 (the lower "
                             "levels' entries are event gaps, not level times)" if chain else "")),
        "full_pipeline_ms": round(t_tot / a.steps, 4),
        "pass_ms": {k: round(v / a.steps, 4) for k, v in pass_acc.items()},
        "full_pipeline_fps": round(1e3 * a.steps / t_tot, 2),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_source": ("profiles/rc_level_pmc.json record of this config, scene and schedule"
                                        if traffic is not None else
                                        "null: no PMC record of this (config, scene, schedule)" +
                                        (" (cascade chain on: no per-level launches)" if chain else "")),
                     "kernel": "k_rc_level", "bytes_per_launch": bytes_launch,
                     "avg_launch_ms": round(avg_launch_s * 1e3, 5)},
    }
    if gather:
        line["gather_roofline"] = gather
    if valu:
        line["valu_roofline"] = valu
    line["inputs"] = input_costs(ctx, W, H, color, emis)
    if rank == 0 and world == 1 and not a.no_cpu_baseline:  # the CPU leg: rank 0 at N=1 only
        line["cpu_baseline"] = cpu_baseline(W, H, N, a.ray_range, a.cpu_budget)
    if rank == 0:
        print(json.dumps(line), flush=True)
    ctx.close()
    finish_pg()
    return 0


if __name__ == "__main__":
    sys.exit(main())
