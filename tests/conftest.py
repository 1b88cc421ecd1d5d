import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def load_fixture(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def params_of(m: dict):
    import oracle

    return oracle.Params(W=m["W"], H=m["H"], N=m["N"], render_scale=m["render_scale"], ray_range=m["ray_range"],
                         sky_radiance=m["sky_radiance"], sky_color=tuple(m["sky_color"]),
                         sun_color=tuple(m["sun_color"]), sun_angle=m["sun_angle"],
                         reflectivity=m["reflectivity"], blur_radius=m["blur_radius"],
                         gi_f16=bool(m.get("gi_f16", False)), rgba8=bool(m.get("rgba8", False)),
                         linux_merge=bool(m.get("linux_merge", False)))


def rel_err(got: np.ndarray, want: np.ndarray, floor: float = 1e-3) -> np.ndarray:
    """|got - want| / max(|want|, floor): the parity metric."""
    return np.abs(got.astype(np.float64) - want) / np.maximum(np.abs(want.astype(np.float64)), floor)


@pytest.fixture(scope="session")
def golden_manifest():
    return manifest()
