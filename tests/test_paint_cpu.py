"""CPU: the scene-painting restatement (oracle/paint_ref.py, raylib 5.5 shapes on GL) against
the llvmpipe fixtures (tests/golden/paint_fixtures.npz, tests/golden/make_paint_golden.py), bit
for bit, and the C-ABI primitive layout."""
import ctypes
import os

import numpy as np
import pytest

from oracle import paint_ref

HERE = os.path.dirname(os.path.abspath(__file__))


def paint_cases():
    d = np.load(os.path.join(HERE, "golden", "paint_fixtures.npz"), allow_pickle=False)
    for n in d["names"]:
        W, H = (int(v) for v in d[n + "__size"])
        clear = d[n + "__clear"]
        prims = [(int(p[0]),) + tuple(float(v) for v in p[1:5]) + tuple(int(v) for v in p[5:9])
                 for p in d[n + "__prims"]]
        yield (str(n), W, H, (None if clear[0] < 0 else tuple(int(v) for v in clear)), prims, d[n + "__image"],
               d[n + "__image_u8"])


@pytest.mark.parametrize("case", list(paint_cases()), ids=lambda c: c[0])
def test_paint_restatement_matches_llvmpipe(case):
    name, W, H, clear, prims, want, _ = case
    base = np.zeros((H, W, 4), np.float32)  # a fresh render texture
    got = paint_ref.paint(W, H, prims, clear, base)
    assert np.array_equal(got, want), f"{name}: {np.count_nonzero(np.any(got != want, axis=-1))} texels differ"


@pytest.mark.parametrize("case", list(paint_cases()), ids=lambda c: c[0])
def test_paint_restatement_rgba8_matches_llvmpipe(case):
    """The same draws into an RGBA8 render texture (the literal app): 8-bit blends."""
    name, W, H, clear, prims, _, want = case
    got = paint_ref.paint(W, H, prims, clear, np.zeros((H, W, 4), np.uint8), rgba8=True)
    assert np.array_equal(got, want), f"{name}: {np.count_nonzero(np.any(got != want, axis=-1))} texels differ"


def test_prim_struct_layout():
    from radiancecascade2dglobalillumination_amd.rc2dgi import Prim

    assert ctypes.sizeof(Prim) == 24 and Prim.r.offset == 20
