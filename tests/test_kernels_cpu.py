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


def test_pow2_division_is_reciprocal_multiply():
    """div_res(): for n = 2^k, a / n == a * (1/n) bit for bit (exact scaling)."""
    rng = np.random.default_rng(0)
    a = rng.random(100000, dtype=np.float32) * np.float32(5000)
    for n in (1, 2, 64, 1024, 4096, 8192, 16384):
        nf = np.float32(n)
        assert np.array_equal(a / nf, a * (np.float32(1) / nf))
