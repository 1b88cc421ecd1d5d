"""oracle -- TEST INFRASTRUCTURE ONLY.

numpy/ctypes front end to the CPU restatement of DoRC2DGI() in
``oracle/rc2dgi_oracle.c`` (reference: RC2DGI.cs:267-406 + shaders/*.fs).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package, and only as the checker or as the reported CPU baseline.  The
product (``radiancecascade2dglobalillumination_amd``) never imports, loads or falls
back to it.

Parity pin: the restatement is checked against fixtures produced by
``oracle/_ref/glref`` -- the reference's own GLSL shaders run on Mesa llvmpipe -- in
``tests/test_oracle_golden.py`` (fixtures: ``tests/golden/``).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle_rc2dgi.so")
GLREF_PATH = os.path.join(HERE, "_ref", "glref")

_f32p = ctypes.POINTER(ctypes.c_float)


class _Cfg(ctypes.Structure):
    _fields_ = [
        ("W", ctypes.c_int), ("H", ctypes.c_int), ("N", ctypes.c_int),
        ("render_scale", ctypes.c_float), ("ray_range", ctypes.c_float),
        ("sky_radiance", ctypes.c_float), ("sky_color", ctypes.c_float * 3),
        ("sun_color", ctypes.c_float * 3), ("sun_angle", ctypes.c_float),
        ("reflectivity", ctypes.c_float), ("blur_radius", ctypes.c_float), ("gi_f16", ctypes.c_int),
        ("rgba8", ctypes.c_int), ("linux_merge", ctypes.c_int),
    ]


class _Overrides(ctypes.Structure):
    _fields_ = [("tc_screen", _f32p), ("tc_cascade", _f32p), ("dir_tables", _f32p), ("sky_table", _f32p)]


class _FrameOut(ctypes.Structure):
    _fields_ = [
        ("jump1", _f32p), ("jump2", _f32p), ("dist", _f32p), ("temp", _f32p), ("color_out", _f32p),
        ("gi1", _f32p), ("gi2", _f32p), ("blur", _f32p), ("gi_levels", ctypes.POINTER(_f32p)),
    ]


def build(force: bool = False) -> None:
    """Compile the restatement (and glref when possible) with oracle/Makefile."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", HERE, LIB_PATH], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_frame.restype = ctypes.c_int
        L.orc_frame.argtypes = [ctypes.POINTER(_Cfg), _f32p, _f32p, ctypes.POINTER(_Overrides),
                                ctypes.POINTER(_FrameOut)]
        L.orc_rc_level.restype = None
        L.orc_rc_level.argtypes = [ctypes.POINTER(_Cfg), ctypes.c_int, _f32p, _f32p, _f32p, _f32p, _f32p,
                                   _f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_int]
        L.orc_rc_level_strided.restype = None
        L.orc_rc_level_strided.argtypes = [ctypes.POINTER(_Cfg), ctypes.c_int, _f32p, _f32p, _f32p, _f32p, _f32p,
                                   _f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_dir_table.argtypes = [ctypes.c_int, ctypes.c_int, _f32p]
        L.orc_sky_table.argtypes = [ctypes.POINTER(_Cfg), _f32p]
        L.orc_dims.argtypes = [ctypes.POINTER(_Cfg), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                               ctypes.POINTER(ctypes.c_int)]
        L.orc_screen_uv.argtypes = [_f32p, _f32p, ctypes.c_int, ctypes.c_int, _f32p]
        L.orc_jfa_step.argtypes = [_f32p, _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                                   ctypes.c_float, _f32p]
        L.orc_distance_field.argtypes = [_f32p, _f32p, ctypes.c_int, ctypes.c_int, _f32p]
        L.orc_blur.argtypes = [_f32p, _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_float, _f32p]
        L.orc_blur_copyback.argtypes = [_f32p, _f32p, ctypes.c_int, ctypes.c_int, _f32p]
        L.orc_merge.argtypes = [_f32p, _f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                _f32p]
        L.orc_merge_ex.argtypes = [_f32p, _f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   _f32p, ctypes.c_int]
        L.orc_set_rows.argtypes = [ctypes.c_int, ctypes.c_int]
        L.orc_set_gi_f16.argtypes = [ctypes.c_int]
        L.orc_set_rgba8.argtypes = [ctypes.c_int]
        L.orc_half_rtz.argtypes = [ctypes.c_float]
        L.orc_half_rtz.restype = ctypes.c_float
        L.orc_num_threads.restype = ctypes.c_int
        L.orc_set_num_threads.argtypes = [ctypes.c_int]
        _lib = L
    return _lib


@dataclass
class Params:
    """Host knobs + uniforms, defaults from RC2DGI.cs:34-41,66-68."""
    W: int = 1200
    H: int = 900
    N: int = 6
    render_scale: float = 1.0
    ray_range: float = 2.0
    sky_radiance: float = 1.0
    sky_color: tuple = (0.5, 0.6, 0.8)
    sun_color: tuple = (1.0, 0.9, 0.6)
    sun_angle: float = 0.3
    reflectivity: float = 0.0
    blur_radius: float = 1.5
    gi_f16: bool = False  # giRT1/2 stored as RGBA16F (RC2DGI.cs:105-106)
    rgba8: bool = False   # every render texture RGBA8 (the literal app): texels k*(1/255)
    linux_merge: bool = False  # Merge.fs not found on Linux (RC2DGI.cs:62): merge adds no GI

    def c(self) -> _Cfg:
        return _Cfg(self.W, self.H, self.N, self.render_scale, self.ray_range, self.sky_radiance,
                    (ctypes.c_float * 3)(*self.sky_color), (ctypes.c_float * 3)(*self.sun_color),
                    self.sun_angle, self.reflectivity, self.blur_radius, int(self.gi_f16),
                    int(self.rgba8), int(self.linux_merge))


INV255 = np.float32(1.0) / np.float32(255.0)


def from_u8(a: np.ndarray) -> np.ndarray:
    """RGBA8 texels -> the floats a unorm8 fetch returns on llvmpipe: k * (1/255) (f32 multiply)."""
    return np.ascontiguousarray(np.asarray(a, np.uint8).astype(np.float32) * INV255)


def to_u8(a: np.ndarray) -> np.ndarray:
    """Floats k * (1/255) (an rgba8-mode frame's render textures) -> the texels k."""
    return np.rint(np.asarray(a, np.float32) * np.float32(255.0)).astype(np.uint8)


def _p(a):
    if a is None:
        return None
    assert a.dtype == np.float32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_f32p)


def dims(p: Params):
    cw, ch, s = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    lib().orc_dims(ctypes.byref(p.c()), ctypes.byref(cw), ctypes.byref(ch), ctypes.byref(s))
    return cw.value, ch.value, s.value


def dir_tables(p: Params) -> np.ndarray:
    """Concatenated (cos, sin) tables for levels 0..N-1 (correctly rounded)."""
    parts = []
    for L in range(p.N):
        t = np.empty((4 << (2 * L), 2), np.float32)
        lib().orc_dir_table(L, p.N, _p(t))
        parts.append(t)
    return np.ascontiguousarray(np.concatenate(parts, 0))


def sky_table(p: Params) -> np.ndarray:
    t = np.empty((4 << (2 * (p.N - 1)), 3), np.float32)
    lib().orc_sky_table(ctypes.byref(p.c()), _p(t))
    return t


@dataclass
class Frame:
    jump1: np.ndarray
    jump2: np.ndarray
    dist: np.ndarray
    gi1: np.ndarray
    gi2: np.ndarray
    blur: np.ndarray
    temp: np.ndarray
    color_out: np.ndarray
    gi_levels: list = field(default_factory=list)
    final_gi: int = 1

    @property
    def gi_final(self):
        return self.gi1 if self.final_gi == 1 else self.gi2


def frame(p: Params, color: np.ndarray, emissive: np.ndarray, tc_screen=None, tc_cascade=None,
          dir_tabs=None, sky_tab=None, keep_levels: bool = False, threads: int | None = None) -> Frame:
    """One ClearAllRTs + DoRC2DGI() frame on the CPU restatement."""
    CW, CH, _ = dims(p)
    W, H = p.W, p.H
    if p.rgba8:  # uint8 texels, or floats quantized the way a float upload to RGBA8 is
        q = lambda a: a if a.dtype == np.uint8 else np.rint(np.clip(a, 0, 1) * 255).astype(np.uint8)  # noqa
        color, emissive = from_u8(q(np.asarray(color))), from_u8(q(np.asarray(emissive)))
    color = np.ascontiguousarray(color, np.float32)
    emissive = np.ascontiguousarray(emissive, np.float32)
    assert color.shape == (H, W, 4) and emissive.shape == (H, W, 4)
    scr = lambda: np.empty((H, W, 4), np.float32)  # noqa: E731
    cas = lambda: np.empty((CH, CW, 4), np.float32)  # noqa: E731
    fr = Frame(scr(), scr(), scr(), cas(), cas(), cas(), scr(), scr())
    levels_arr = None
    if keep_levels:
        fr.gi_levels = [cas() for _ in range(p.N)]
        levels_arr = (_f32p * p.N)(*[_p(a) for a in fr.gi_levels])
    keep = [np.ascontiguousarray(x, np.float32) if x is not None else None
            for x in (tc_screen, tc_cascade, dir_tabs, sky_tab)]
    ov = _Overrides(*[_p(x) for x in keep])
    out = _FrameOut(_p(fr.jump1), _p(fr.jump2), _p(fr.dist), _p(fr.temp), _p(fr.color_out),
                    _p(fr.gi1), _p(fr.gi2), _p(fr.blur), levels_arr)
    if threads:
        lib().orc_set_num_threads(int(threads))
    rc = lib().orc_frame(ctypes.byref(p.c()), _p(color), _p(emissive), ctypes.byref(ov), ctypes.byref(out))
    if rc != 0:
        raise ValueError(f"orc_frame failed ({rc})")
    fr.final_gi = 2 if p.N % 2 == 0 else 1
    return fr


def rc_level(p: Params, level: int, upper, color, emissive, dist, out, dir_table, sky_tab, row0=0, row1=None):
    """One RadianceCascades.fs level over rows [row0, row1) (bench cpu_baseline sample)."""
    _, CH, _ = dims(p)
    lib().orc_rc_level(ctypes.byref(p.c()), level, _p(upper), _p(color), _p(emissive), _p(dist), _p(out),
                       _p(dir_table), _p(sky_tab), None, row0, CH if row1 is None else row1)


def rc_level_rows(p: Params, level: int, upper, color, emissive, dist, out, dir_table, sky_tab, row0=0, row1=None,
                  stride=1):
    """rc_level over the rows row0, row0 + stride, ... < row1, in parallel (parity tests)."""
    _, CH, _ = dims(p)
    lib().orc_rc_level_strided(ctypes.byref(p.c()), level, _p(upper), _p(color), _p(emissive), _p(dist), _p(out),
                               _p(dir_table), _p(sky_tab), None, row0, CH if row1 is None else row1, stride)


def _c(a):
    return np.ascontiguousarray(a, np.float32)


class rgba8_textures:
    """``with oracle.rgba8_textures():`` -- the per-pass functions below treat every render
    texture as RGBA8 (8-bit blends, 8.8 fixed-point LINEAR filtering; texels k*(1/255))."""

    def __enter__(self):
        lib().orc_set_rgba8(1)
        return self

    def __exit__(self, *exc):
        lib().orc_set_rgba8(0)
        return False


def screen_uv(color, tc=None):
    """ScreenUV.fs over a cleared jumpRT1 -> (H, W, 4)."""
    color = _c(color)
    H, W = color.shape[:2]
    out = np.empty((H, W, 4), np.float32)
    lib().orc_screen_uv(_p(color), _p(out), W, H, _p(None if tc is None else _c(tc)))
    return out


def jfa_step(src, step: float, aspx: float, aspy: float, tc=None):
    """One JumpFlood.fs step (the source alpha is 1, so dst is fully overwritten)."""
    src = _c(src)
    H, W = src.shape[:2]
    out = np.zeros((H, W, 4), np.float32)
    out[..., 3] = 1.0
    lib().orc_jfa_step(_p(src), _p(out), W, H, step, aspx, aspy, _p(None if tc is None else _c(tc)))
    return out


def distance_field(jump, tc=None):
    jump = _c(jump)
    H, W = jump.shape[:2]
    out = np.zeros((H, W, 4), np.float32)
    out[..., 3] = 1.0
    lib().orc_distance_field(_p(jump), _p(out), W, H, _p(None if tc is None else _c(tc)))
    return out


def blur(gi, radius: float, tc=None):
    gi = _c(gi)
    CH, CW = gi.shape[:2]
    out = np.empty_like(gi)
    lib().orc_blur(_p(gi), _p(out), CW, CH, radius, _p(None if tc is None else _c(tc)))
    return out


def blur_copyback(blur_img, gi, tc=None):
    """Returns the blended copy of blur_img onto (a copy of) gi."""
    blur_img = _c(blur_img)
    g = _c(gi).copy()
    CH, CW = g.shape[:2]
    lib().orc_blur_copyback(_p(blur_img), _p(g), CW, CH, _p(None if tc is None else _c(tc)))
    return g


def merge(color, gi, tc=None, linux_merge=False):
    color, gi = _c(color), _c(gi)
    H, W = color.shape[:2]
    CH, CW = gi.shape[:2]
    temp = np.empty_like(color)
    out = np.empty_like(color)
    lib().orc_merge_ex(_p(color), _p(gi), _p(temp), _p(out), W, H, CW, CH, _p(None if tc is None else _c(tc)),
                       int(linux_merge))
    return temp, out


def num_threads() -> int:
    return lib().orc_num_threads()


def set_num_threads(n: int) -> None:
    lib().orc_set_num_threads(n)
