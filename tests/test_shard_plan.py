"""CPU: row-strip sharding of one frame, checked with the oracle.

The planner (``rc2dgi_plan_rows``, host-only, no device) says which rows each shard computes
for every pass.  Here every shard runs the CPU restatement restricted to exactly those rows
into NaN-poisoned render textures; the one exchange (distRT strips) goes through an in-process
copy or, with two processes, through ``torch.distributed`` over gloo.  Each shard's merged
colorRT / tempRT strip must equal the unsharded frame bit for bit: a missing dependency reads
NaN and shows up as a mismatch.
"""
import ctypes
import os
import socket

import numpy as np
import pytest

import oracle
from radiancecascade2dglobalillumination_amd import rc2dgi as R
from radiancecascade2dglobalillumination_amd import scenes


def _rows(p, rank, world, pass_id):
    return R.plan_rows(p.W, p.H, p.N, p.blur_radius, rank, world, pass_id, p.render_scale)


def _strip(H, rank, world):
    return rank * H // world, (rank + 1) * H // world


CLEAR = np.array([0.0, 0.0, 0.0, 1.0], np.float32)  # ClearBackground(Black)


class Shard:
    """One shard of one frame on the CPU restatement, following the C-ABI plan.  Rows a pass
    writes are first cleared as the reference's ClearAllRTs / per-pass clears leave them; every
    other row stays NaN, so reading a row the plan did not compute poisons the result."""

    def __init__(self, p, color, emis, rank, world):
        self.p, self.rank, self.world = p, rank, world
        self.color = np.ascontiguousarray(color, np.float32)
        self.emis = np.ascontiguousarray(emis, np.float32)
        self.CW, self.CH, self.S = oracle.dims(p)
        self.y0, self.y1 = _strip(p.H, rank, world)

    def phase1(self):
        p, L = self.p, oracle.lib()
        W, H = p.W, p.H
        nan = lambda: np.full((H, W, 4), np.nan, np.float32)  # noqa: E731
        mx = max(W, H)
        aspx, aspy = np.float32(W) / np.float32(mx), np.float32(H) / np.float32(mx)
        j1, j2 = oracle.screen_uv(self.color), nan()  # ScreenUV runs whole on every shard
        j1final, step = True, np.float32(1.0)
        for s in range(self.S):
            step = np.float32(step * np.float32(0.5))
            src, dst = (j1, j2) if j1final else (j2, j1)
            for a, b in _rows(p, self.rank, self.world, R.PLAN_JFA + s):
                if s < 2:  # jumpRT2 / the J0 rows in jumpRT1 are cleared texels before their first step
                    dst[a:b] = CLEAR
                L.orc_set_rows(a, b)
                L.orc_jfa_step(oracle._p(src), oracle._p(dst), W, H, float(step), float(aspx), float(aspy), None)
            j1final = not j1final
        self.dist = nan()
        self.dist[self.y0:self.y1] = CLEAR
        L.orc_set_rows(self.y0, self.y1)
        L.orc_distance_field(oracle._p(j1 if j1final else j2), oracle._p(self.dist), W, H, None)
        L.orc_set_rows(-1, -1)
        return self.dist[self.y0:self.y1].copy()

    def phase2(self):
        p, L = self.p, oracle.lib()
        CW, CH = self.CW, self.CH
        assert not np.isnan(self.dist).any(), "distRT exchange incomplete"
        nanc = lambda: np.full((CH, CW, 4), np.nan, np.float32)  # noqa: E731
        dirs, sky = oracle.dir_tables(p), oracle.sky_table(p)
        gi1, gi2 = nanc(), nanc()
        gi1final, off = False, [0]
        for lv in range(p.N):
            off.append(off[-1] + (4 << (2 * lv)))
        for lv in range(p.N - 1, -1, -1):
            src, dst = (gi1, gi2) if gi1final else (gi2, gi1)
            bdy, bsc = CH >> lv, 1 << lv
            for a, b in _rows(p, self.rank, self.world, R.PLAN_LEVEL + lv):
                for by in range(bsc):
                    dst[by * bdy + a:by * bdy + b] = CLEAR
                    L.orc_rc_level(ctypes.byref(p.c()), lv, None if lv == p.N - 1 else oracle._p(src),
                                   oracle._p(self.color), oracle._p(self.emis), oracle._p(self.dist), oracle._p(dst),
                                   oracle._p(np.ascontiguousarray(dirs[off[lv]:off[lv + 1]])), oracle._p(sky), None,
                                   by * bdy + a, by * bdy + b)
            gi1final = not gi1final
        fin = gi1 if gi1final else gi2
        if p.blur_radius > 0:
            blur = nanc()
            for a, b in _rows(p, self.rank, self.world, R.PLAN_BLUR):
                blur[a:b] = CLEAR
                L.orc_set_rows(a, b)
                L.orc_blur(oracle._p(fin), oracle._p(blur), CW, CH, p.blur_radius, None)
            for a, b in _rows(p, self.rank, self.world, R.PLAN_BLUR):
                L.orc_set_rows(a, b)
                L.orc_blur_copyback(oracle._p(blur), oracle._p(fin), CW, CH, None)
        W, H = p.W, p.H
        temp, out = np.full((H, W, 4), np.nan, np.float32), np.full((H, W, 4), np.nan, np.float32)
        for a, b in _rows(p, self.rank, self.world, R.PLAN_MERGE):
            temp[a:b] = CLEAR
            L.orc_set_rows(a, b)
            L.orc_merge(oracle._p(self.color), oracle._p(fin), oracle._p(temp), oracle._p(out), W, H, CW, CH, None)
        L.orc_set_rows(-1, -1)
        return out[self.y0:self.y1], temp[self.y0:self.y1]


CASES = [
    # W, H, N, rayRange, renderScale, blur, world, scene
    (64, 64, 3, 4.0, 1.0, 1.5, 2, "rand:1"),
    (128, 96, 4, 2.0, 1.0, 1.5, 3, "rand:2"),     # non-square, non-power-of-two rows
    (200, 120, 3, 2.0, 1.0, 2.5, 4, "rand:3"),    # non-power-of-two: float JFA taps
    (160, 128, 3, 8.0, 0.5, 1.37, 3, "rand:4"),   # cascades coarser than the screen
    (96, 64, 2, 2.0, 1.0, 0.0, 5, "rand:5"),      # blur off
    (256, 256, 5, 3.0, 1.0, 1.5, 8, "demo"),
    (333, 200, 4, 2.0, 1.7, 1.5, 3, "rand:6"),    # renderScale > 1
]


def _scene(spec, W, H):
    if spec == "demo":
        return scenes.demo(W, H)
    return scenes.random_scene(W, H, int(spec.split(":")[1]))


@pytest.mark.parametrize("W,H,N,rr,rs,blur,world,scene", CASES)
def test_oracle_strips_reproduce_the_frame(W, H, N, rr, rs, blur, world, scene):
    p = oracle.Params(W=W, H=H, N=N, ray_range=rr, render_scale=rs, blur_radius=blur)
    color, emis = _scene(scene, W, H)
    full = oracle.frame(p, color, emis)
    shards = [Shard(p, color, emis, r, world) for r in range(world)]
    strips = [s.phase1() for s in shards]
    for s in shards:  # the exchange: every distRT strip to every shard
        for q, st in enumerate(strips):
            a, b = _strip(H, q, world)
            s.dist[a:b] = st
    for s in shards:
        out, temp = s.phase2()
        assert np.array_equal(out, full.color_out[s.y0:s.y1]), f"shard {s.rank}: colorRT strip differs"
        assert np.array_equal(temp, full.temp[s.y0:s.y1]), f"shard {s.rank}: tempRT strip differs"


def test_plan_shape():
    """Merge rows partition the screen; unsharded plans are whole passes; JFA rows shrink."""
    W = H = 1024
    for world in (1, 2, 3, 8):
        rows = sorted(iv for r in range(world) for iv in R.plan_rows(W, H, 6, 1.5, r, world, R.PLAN_MERGE))
        assert rows[0][0] == 0 and rows[-1][1] == H
        assert all(a[1] == b[0] for a, b in zip(rows, rows[1:]))
    S = 10
    assert all(R.plan_rows(W, H, 6, 1.5, 0, 1, R.PLAN_JFA + s) == [(0, H)] for s in range(S))
    sizes = [sum(b - a for a, b in R.plan_rows(W, H, 6, 1.5, 3, 8, R.PLAN_JFA + s)) for s in range(S)]
    assert sizes[0] == H and sizes[-1] == H // 8 and sizes == sorted(sizes, reverse=True)
    with pytest.raises(R.RC2DGIError):
        R.plan_rows(W, H, 6, 1.5, 8, 8, R.PLAN_MERGE)


# ---------------------------------------------------------------- two processes over gloo
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


GLOO_CASE = (128, 96, 4, 2.0, 1.0, 1.5, "rand:7")


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from radiancecascade2dglobalillumination_amd import dist as rdist

    rdist.init("gloo")
    W, H, N, rr, rs, blur, scene = GLOO_CASE
    p = oracle.Params(W=W, H=H, N=N, ray_range=rr, render_scale=rs, blur_radius=blur)
    color, emis = _scene(scene, W, H)
    sh = Shard(p, color, emis, rank, world)
    mine = sh.phase1()
    strips = [None] * world
    dist.all_gather_object(strips, mine)  # the distRT exchange
    for r, st in enumerate(strips):
        a, b = _strip(H, r, world)
        sh.dist[a:b] = st
    out, _ = sh.phase2()
    outs = [None] * world
    dist.all_gather_object(outs, out)
    if rank == 0:
        q.put(np.concatenate(outs, 0))
    dist.destroy_process_group()


def test_two_ranks_gloo_strips():
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    got = q.get(timeout=300)
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    W, H, N, rr, rs, blur, scene = GLOO_CASE
    p = oracle.Params(W=W, H=H, N=N, ray_range=rr, render_scale=rs, blur_radius=blur)
    color, emis = _scene(scene, W, H)
    assert np.array_equal(got, oracle.frame(p, color, emis).color_out)
