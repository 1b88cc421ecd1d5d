"""CPU checks of numeric identities the HIP kernels rely on (no GPU needed)."""
import numpy as np


def test_decode_dist_double_product_is_exact_fp32_division():
    """k_rc_level decodes the stored 16-bit distance as (float)((double)q * (1.0/65535.0));
    RadianceCascades.fs:30-33 computes float(q) / 65535.0 in fp32.  Equal for every q."""
    q = np.arange(65536, dtype=np.float64)
    want = np.float32(q) / np.float32(65535.0)
    got = (q * (1.0 / 65535.0)).astype(np.float32)
    assert np.array_equal(got, want)


def test_hit_threshold_monotone():
    """distance < 0.001 (RadianceCascades.fs:79) is a threshold on q."""
    d = np.arange(65536, dtype=np.float32) / np.float32(65535.0)
    hits = d < np.float32(0.001)
    k = int(np.argmin(hits))
    assert hits[:k].all() and not hits[k:].any() and k == 66
