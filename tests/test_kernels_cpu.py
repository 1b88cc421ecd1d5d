"""CPU checks of numeric identities the HIP kernels rely on (no GPU needed)."""
from fractions import Fraction

import numpy as np


def _round_f32(fr: Fraction) -> np.float32:
    """Correctly rounded (nearest-even) float32 of an exact rational."""
    f = np.float32(float(fr))
    cands = [np.nextafter(f, np.float32(-np.inf)), f, np.nextafter(f, np.float32(np.inf))]

    def key(c):
        return abs(Fraction(float(c)) - fr), int(np.frombuffer(np.float32(c).tobytes(), np.uint32)[0]) & 1

    return np.float32(min(cands, key=key))


def _fma(a, b, c) -> np.float32:
    return _round_f32(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c)))


def test_decode_dist_newton_is_exact_fp32_division():
    """k_rc_level decodes the stored 16-bit distance as x = q*(1/65535); r = fma(-x, 65535, q);
    fma(r, 1/65535, x).  RadianceCascades.fs:30-33 computes float(q) / 65535.0 in fp32.
    Equal for every q (exact fma semantics, as v_fma_f32)."""
    c1 = np.float32(1.0) / np.float32(65535.0)
    qs = np.arange(65536, dtype=np.float32)
    want = qs / np.float32(65535.0)
    x = qs * c1
    easy = x == want
    # x already exact for most q; the correction must keep those and fix the rest
    for q in range(65536):
        r = _fma(-x[q], np.float32(65535.0), qs[q])
        got = _fma(r, c1, x[q])
        assert got == want[q], q
    assert easy.mean() > 0.9


def test_hit_threshold_monotone():
    """distance < 0.001 (RadianceCascades.fs:79) is a threshold on q."""
    d = np.arange(65536, dtype=np.float32) / np.float32(65535.0)
    hits = d < np.float32(0.001)
    k = int(np.argmin(hits))
    assert hits[:k].all() and not hits[k:].any() and k == 66


def test_byte_exit_table_entries_are_lower_bounds():
    """k_dist_cmin's byte entries (CminT, rc2dgi_kernels.h): a cell whose smallest distance d passes
    the hit test stores k = min(255, floor(d * 512)) and k_rc_level reads k * (1/512).  That value
    must never exceed d (the exit proof needs a lower bound), and 0 stays 0 (a hit cell proves
    nothing).  Every q, fp32 arithmetic as on the device."""
    q = np.arange(65536, dtype=np.float32)
    d = q / np.float32(65535.0)
    for scale in (256.0, 512.0, 1024.0):
        sc = np.float32(scale)
        k = np.where(d >= np.float32(0.001), np.minimum(np.floor(d * sc), np.float32(255.0)), np.float32(0.0))
        k = k.astype(np.uint8)
        bound = k.astype(np.float32) * (np.float32(1.0) / sc)
        assert (bound <= d).all()
        assert (bound[d < np.float32(0.001)] == 0).all()
        # the bound is tight to one step below saturation
        ok = (d < np.float32(255.0) / sc) & (d >= np.float32(0.001))
        assert (d[ok] - bound[ok] < np.float32(1.0) / sc).all()


def test_pow2_division_is_reciprocal_multiply():
    """div_res(): for n = 2^k, a / n == a * (1/n) bit for bit (exact scaling)."""
    rng = np.random.default_rng(0)
    a = rng.random(100000, dtype=np.float32) * np.float32(5000)
    for n in (1, 2, 64, 1024, 4096, 8192, 16384):
        nf = np.float32(n)
        assert np.array_equal(a / nf, a * (np.float32(1) / nf))


def _jfa_shader_key(si, sj, i, j, W, H):
    """JumpFlood.fs distance in fp32: texcoord differences, squared, summed (no contraction)."""
    f = np.float32
    u, v = (f(i) + f(0.5)) / f(W), (f(j) + f(0.5)) / f(H)
    px, py = (si.astype(f) + f(0.5)) / f(W), (sj.astype(f) + f(0.5)) / f(H)
    dx, dy = px - u, py - v
    return dx * dx + dy * dy


def test_jfa_integer_key_matches_shader_distance():
    """k_jfa_p2 IKEY (W == H <= 4096): float(dx^2 + dy^2) over integer texel differences, scaled by
    W^-2, equals the shader's fp32 distance for every seed offset, so comparisons agree."""
    W = H = 4096
    rng = np.random.default_rng(7)
    i, j = 1234, 3001
    si = np.concatenate([rng.integers(0, W, 200000), np.arange(W)]).astype(np.int64)
    sj = np.concatenate([rng.integers(0, H, 200000), np.full(W, 4095)]).astype(np.int64)
    want = _jfa_shader_key(si, sj, i, j, W, H)
    n = (si - i) ** 2 + (sj - j) ** 2
    got = n.astype(np.float32) * np.float32(2.0 ** -24)
    assert np.array_equal(got, want)
    # the no-seed value (32768, 32768) keys above the initial minDist (W^2) for every texel
    for ii, jj in ((0, 0), (4095, 4095), (0, 4095)):
        d = np.int64(32768 - ii) ** 2 + np.int64(32768 - jj) ** 2
        assert min(d, 2 ** 31 - 1) >= W * W  # v_dot2_i32_i16 with clamp


def test_jfa_scaled_float_key_matches_shader_distance():
    """k_jfa_p2 fp32 key (power-of-two, non-square or > 4096): ((si-i)*scx)^2 + ((sj-j)*scy)^2
    equals the shader distance times max(W,H)^2 exactly."""
    rng = np.random.default_rng(8)
    for W, H in ((128, 64), (64, 128), (8192, 8192), (16384, 256)):
        mx = max(W, H)
        i, j = W // 3, H // 5
        si, sj = rng.integers(0, W, 100000), rng.integers(0, H, 100000)
        want = _jfa_shader_key(si, sj, i, j, W, H)
        f = np.float32
        dx = (si - i).astype(f) * f(mx // W)
        dy = (sj - j).astype(f) * f(mx // H)
        got = (dx * dx + dy * dy) * f(1.0 / mx) * f(1.0 / mx)
        assert np.array_equal(got, want), (W, H)


def _plan_order(lib, code, tx, ty, ng, tw=16, th=16):
    import ctypes

    n = tx * ty * ng
    tiles, groups = (ctypes.c_int * n)(), (ctypes.c_int * n)()
    assert lib.rc2dgi_plan_order(code, tx, ty, tw, th, ng, tiles, groups, n) == 0
    return list(zip(tiles, groups))


def test_rc_workgroup_order_is_a_bijection():
    """Every (tile, direction group) is visited exactly once for any grid, partial patches
    included (row-strip shards give tile grids the patches do not divide), for the plain and
    the direction-oriented / banded orders (the library's own host map, rc2dgi_plan_order)."""
    import itertools

    from radiancecascade2dglobalillumination_amd import _build, load_library

    _build.build()
    lib = load_library()
    for tx, ty, ng, px, py, dg, ori in itertools.product([1, 3, 5, 16], [1, 2, 5, 7, 16], [1, 4, 16],
                                                         [1, 2, 3, 4, 16], [1, 2, 4, 5], [1, 2, 4, 16], [0, 1, 2]):
        if ng % dg:
            continue
        code = px | py << 8 | dg << 16 | ori << 24
        seen = set(_plan_order(lib, code, tx, ty, ng))
        n = tx * ty * ng
        assert len(seen) == n and all(0 <= t < tx * ty and 0 <= d < ng for t, d in seen), (tx, ty, ng, px, py, dg, ori)


def _plan_wg_map(lib, code, tx, ty, ng, tw=16, th=16):
    import ctypes

    n = tx * ty * ng
    tiles, groups = (ctypes.c_int * n)(), (ctypes.c_int * n)()
    assert lib.rc2dgi_plan_wg_map(code, tx, ty, tw, th, ng, tiles, groups, n) == 0
    return list(zip(tiles, groups))


def test_xcd_interleaved_workgroup_map_is_a_bijection():
    """The device map (rc2dgi_plan_wg_map: the XCD split of the logical order, order code bits 26-30 = lc) visits
    every (tile, direction group) exactly once for any count -- whole rounds of 8 chunks interleaved, the
    remainder split contiguously -- and lc = 0 is the contiguous split (each XCD, dispatch id mod 8, one eighth)."""
    import itertools

    from radiancecascade2dglobalillumination_amd import _build, load_library

    _build.build()
    lib = load_library()
    for tx, ty, ng, lc, base in itertools.product([1, 3, 8, 16], [1, 5, 16], [1, 4, 64], [0, 1, 2, 5, 9, 16, 17, 19],
                                                 [0, 4 | 8 << 8 | 4 << 16, 2 | 2 << 8 | 2 << 16 | 1 << 24]):
        n = tx * ty * ng
        m = _plan_wg_map(lib, base | lc << 26, tx, ty, ng)
        assert len(set(m)) == n and all(0 <= t < tx * ty and 0 <= d < ng for t, d in m), (tx, ty, ng, lc, base)
        lo = _plan_order(lib, base | lc << 26, tx, ty, ng)
        assert sorted(m) == sorted(lo)
    # contiguous split: XCD x (dispatch ids x, x + 8, ...) walks logical workgroups [x n / 8, (x + 1) n / 8)
    tx, ty, ng = 16, 16, 16
    n = tx * ty * ng
    lo = _plan_order(lib, 4 | 8 << 8 | 4 << 16, tx, ty, ng)
    m = _plan_wg_map(lib, 4 | 8 << 8 | 4 << 16, tx, ty, ng)
    assert [m[p] for p in range(3, n, 8)] == lo[3 * n // 8:4 * n // 8]
    # interleaved (lc = 4): XCD 3's k-th chunk of 16 is logical chunk 8 k + 3
    m = _plan_wg_map(lib, 4 | 8 << 8 | 4 << 16 | 4 << 26, tx, ty, ng)
    x3 = [m[p] for p in range(3, n, 8)]
    assert x3 == [lo[(k // 16) * 128 + 3 * 16 + k % 16] for k in range(n // 8)]
    # Latin square (lc = 16 + t): 8 regions of S = 8 << t sub-chunks; XCD x's j-th sub-chunk is sub-chunk j of region
    # (x + j) mod 8, so at each step j the 8 XCDs are in 8 different regions and each XCD visits every region
    for t in (0, 1):
        S = 8 << t
        c = n // (8 * S)
        m = _plan_wg_map(lib, 4 | 8 << 8 | 4 << 16 | (16 + t) << 26, tx, ty, ng)
        for x in range(8):
            xs = [m[p] for p in range(x, n, 8)]
            assert xs == [lo[((x + k // c) % 8) * (n // 8) + (k // c) * c + k % c] for k in range(n // 8)]


def test_oriented_order_lays_patches_along_the_rays():
    """Oriented order: a chunk of direction groups near the x axis walks px-wide patches, one near
    the y axis px-tall patches (RC level with 16 direction groups, 16 x 16 tiles)."""
    from radiancecascade2dglobalillumination_amd import _build, load_library

    _build.build()
    lib = load_library()
    m = _plan_order(lib, 16 | 1 << 8 | 2 << 16 | 1 << 24, 16, 16, 16)  # 16 x 1 patches, chunks of 2 groups
    first = [t for t, _ in m[:16 * 2:2]]  # chunk 0, mean angle 2 pi * 1/16 (22.5 deg): the first patch
    assert first == list(range(16))  # one tile row
    q = 2 * 256  # chunk 1, mean angle 2 pi * 3/16 (67.5 deg)
    second = [t for t, _ in m[q:q + 16 * 2:2]]
    assert second == [16 * i for i in range(16)]  # one tile column


def test_banded_order_follows_the_rays():
    """Banded order: within a chunk of direction groups, consecutive tiles advance along the
    chunk's mean ray direction inside a band across it (here 45 degrees: the diagonal)."""
    import math

    from radiancecascade2dglobalillumination_amd import _build, load_library

    _build.build()
    lib = load_library()
    ng, dg = 8, 1  # chunk 1 of 8: mean angle 2 pi * 1.5 / 8 = 67.5 deg; chunk 0: 22.5 deg
    m = _plan_order(lib, 1 | 1 << 8 | dg << 16 | 2 << 24, 16, 16, ng)
    for ch in (0, 1):
        th = 2 * math.pi * (ch + 0.5) / ng
        seq = [t for t, g in m[ch * 256:(ch + 1) * 256]]
        assert all(g == ch for _, g in m[ch * 256:(ch + 1) * 256])
        us = [((t % 16) + 0.5) * math.cos(th) + ((t // 16) + 0.5) * math.sin(th) for t in seq]
        vs = [math.floor((-((t % 16) + 0.5) * math.sin(th) + ((t // 16) + 0.5) * math.cos(th))) for t in seq]
        # bands in order, positions along the ray increasing inside each band
        assert vs == sorted(vs)
        for a, b, va, vb in zip(us, us[1:], vs, vs[1:]):
            assert va != vb or a <= b


def test_packet_index_magic_divisions():
    """k_rc_level's packet index ix / 14 and ix / 26 as one 24-bit multiply and a shift
    (pack_div14, pack_div26 in csrc/rc2dgi_rc.h), exact for every column of a screen <= 16384."""
    ix = np.arange(16384, dtype=np.int64)
    assert np.array_equal((ix * 37450) >> 19, ix // 14)
    assert np.array_equal((ix * 20165) >> 19, ix // 26)
    assert int(ix[-1] * 20165) < 2 ** 32 and int(ix[-1] * 37450) < 2 ** 32


def _nib_encode(q, W):
    """numpy restatement of k_dist_nib for one row (the device decoder is packet_q<3>)."""
    out = []
    for x0 in range(0, W, 26):
        seg = q[x0:x0 + 26].astype(np.int64)
        cnt = len(seg)
        s0 = int(np.floor(np.float32(seg[-1] - seg[0]) / np.float32(max(cnt - 1, 1)) + np.float32(0.5))) if cnt > 1 else 0
        best = None
        for ds in range(-2, 3):
            sl = min(127, max(-128, s0 + ds))
            r = seg - sl * np.arange(cnt)
            base = min(65535, max(0, (int(r.min()) + int(r.max())) >> 1))
            esc = int(np.count_nonzero(np.abs(r - base) > 7))
            if best is None or esc < best[0]:
                best = (esc, sl, base)
        _, sl, base = best
        r = seg - sl * np.arange(cnt) - base
        nib = np.where(np.abs(r) <= 7, r + 7, 15)
        out.append((base, sl, np.concatenate([nib, np.full(26 - cnt, 15)])))
    return out


def test_nibble_packets_round_trip():
    """Every texel decodes to its q exactly or is flagged as an escape (read from the 16-bit
    field), on a distance-like row (|dq| <= 16 per texel, kinks) and on random rows."""
    rng = np.random.default_rng(5)
    rows = [np.clip(np.cumsum(rng.integers(-16, 17, 4096)) + 30000, 0, 65535),
            np.abs(np.arange(1000) - 377) * 16 + 3,
            rng.integers(0, 65536, 300)]
    for q in rows:
        W = len(q)
        esc = 0
        for k, (base, sl, nib) in enumerate(_nib_encode(q, W)):
            for t in range(min(26, W - 26 * k)):
                if nib[t] == 15:
                    esc += 1
                    continue
                assert base + sl * t + int(nib[t]) - 7 == q[26 * k + t]
        assert esc <= W
    # the smooth row mostly fits
    assert sum(int(np.count_nonzero(n == 15)) for _, _, n in _nib_encode(rows[1], len(rows[1]))) < 60


def _exit_terms(dx, dy, aspx, aspy):
    """rc_exit_terms (csrc/rc2dgi_kernels.h), float32 step by step."""
    f = np.float32
    v = [f(dx) * f(aspy), f(dy) * f(aspx)]
    inv, edge = [], []
    for a in range(2):
        dead = not (v[a] > f(2.0 ** -100) or v[a] < f(-(2.0 ** -100)))
        inv.append(f(np.inf) if dead else f(1.0) / v[a])
        edge.append(f(2.0) if dead else (f(1.0 + 2.0 ** -19) if v[a] > 0 else f(-(2.0 ** -19))))
    return inv + edge


def test_screen_exit_terms_put_the_sample_off_screen():
    """The exit proof of k_rc_level (exit_bound) treats every t >= T as off screen, with
    T = min((ex - ox) * ix, (ey - oy) * iy) from the per-direction terms.  Each coordinate of
    o + (t dir) asp is monotone in t, so that holds iff the position at T itself is off screen
    (outside [0, 1] on some axis) -- checked here in float32 for origins right at the edges,
    directions near the axes, and the aspect ratios of non-square screens."""
    f = np.float32
    rng = np.random.default_rng(7)
    edge_o = [f(0.5 / 16384), f(1 - 0.5 / 16384), f(0.5 / 4096), f(1 - 0.5 / 4096), f(0.5)]
    checked = 0
    for W, H in [(4096, 4096), (1200, 900), (900, 1200), (16384, 128), (333, 16384)]:
        mx = max(W, H)
        aspx, aspy = f(W) / f(mx), f(H) / f(mx)
        angles = np.concatenate([rng.uniform(0, 2 * np.pi, 400),
                                 (np.array([0, np.pi / 2, np.pi, 3 * np.pi / 2]) + rng.normal(0, 1e-6, (50, 4))).ravel()])
        dirs = [(f(np.cos(a)), f(np.sin(a))) for a in angles] + [(f(1), f(0)), (f(0), f(-1)), (f(1e-38), f(1))]
        origins = [(a, b) for a in edge_o for b in edge_o] + [tuple(f(x) for x in rng.uniform(0, 1, 2))
                                                              for _ in range(20)]
        for dx, dy in dirs:
            ix, iy, ex, ey = _exit_terms(dx, dy, aspx, aspy)
            for ox, oy in origins:
                with np.errstate(invalid="ignore", over="ignore"):
                    T = min((ex - ox) * ix, (ey - oy) * iy)
                assert T > 0
                if T == np.inf:
                    continue
                px = ox + (T * dx) * aspy
                py = oy + (T * dy) * aspx
                assert px < 0 or px > 1 or py < 0 or py > 1, (W, H, dx, dy, ox, oy, T, px, py)
                checked += 1
    assert checked > 50000, checked
