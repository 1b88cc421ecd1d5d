"""CPU: the C-ABI library builds, loads and exports every entry point include/rc2dgi.h
declares; argument validation that happens before any device work."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "rc2dgi.h")


def declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(rc2dgi_\w+)\s*\(", src, re.M)))


@pytest.fixture(scope="module")
def lib():
    from radiancecascade2dglobalillumination_amd import _build, load_library

    _build.build()
    return load_library()


def test_header_declares_the_boundary():
    names = declared()
    for must in ("rc2dgi_create", "rc2dgi_destroy", "rc2dgi_set_uniform", "rc2dgi_set_uniform_i", "rc2dgi_upload",
                 "rc2dgi_do", "rc2dgi_sync", "rc2dgi_download", "rc2dgi_query", "rc2dgi_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol(lib):
    for n in declared():
        assert hasattr(lib, n), f"librc2dgi.so does not export {n}"


def test_abi_version(lib):
    assert lib.rc2dgi_abi_version() == 5


def _cfg(**kw):
    from radiancecascade2dglobalillumination_amd.rc2dgi import _Config

    d = dict(screen_width=64, screen_height=64, cascade_count=2, render_scale=1.0, ray_range=2.0, storage=0, device=0,
             flags=0)
    d.update(kw)
    return _Config(d["screen_width"], d["screen_height"], d["cascade_count"], d["render_scale"], d["ray_range"],
                   d["storage"], d["device"], d["flags"], (ctypes.c_int * 4)())


@pytest.mark.parametrize("kw,code", [
    (dict(screen_width=0), -1), (dict(screen_height=-3), -1), (dict(cascade_count=0), -1),
    (dict(cascade_count=16), -1), (dict(render_scale=0.0), -1), (dict(storage=-1), -1), (dict(storage=7), -1),
    (dict(flags=2), -1), (dict(flags=-1), -1),
])
def test_create_validates_config_before_touching_the_device(lib, kw, code):
    h = ctypes.c_void_p()
    assert lib.rc2dgi_create(ctypes.byref(_cfg(**kw)), ctypes.byref(h)) == code
    assert not h.value


def test_null_arguments_are_errors_not_crashes(lib):
    assert lib.rc2dgi_create(None, None) == -1
    assert lib.rc2dgi_do(None) == -1
    assert lib.rc2dgi_sync(None) == -1
    assert lib.rc2dgi_destroy(None) == -1
    assert lib.rc2dgi_query(None, None, None, None, None) == -1


def test_no_device_is_reported_not_aborted(lib):
    import torch

    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is visible")
    h = ctypes.c_void_p()
    assert lib.rc2dgi_create(ctypes.byref(_cfg()), ctypes.byref(h)) == -3  # RC2DGI_E_HIP


def test_product_does_not_import_the_oracle():
    pkg = os.path.join(ROOT, "radiancecascade2dglobalillumination_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                src = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in src and "from oracle" not in src and "rc2dgi_oracle" not in src, f
