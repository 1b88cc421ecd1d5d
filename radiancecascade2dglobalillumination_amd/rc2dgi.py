"""Host-side mirror of the reference's GI path over the librc2dgi C ABI.

The reference drives its per-frame GI from C# (RC2DGI.cs):

* knobs/globals ``cascadeCount``, ``renderScale``, ``rayRange`` (RC2DGI.cs:28-31, 66-68)
  and the GUI-driven uniforms ``sunAngle``, ``sunColor``, ``skyColor``, ``skyRadiance``,
  ``reflectivity``, ``cascadeBlurRadius`` (RC2DGI.cs:33-41);
* ``DoRC2DGI()`` (RC2DGI.cs:267-406) -> :meth:`RC2DGI.do_rc2dgi`;
* ``SetGIShaderValues()`` (RC2DGI.cs:408-433) -> :meth:`RC2DGI.set_shader_value` with the
  reference uniform names (``_RayRange``, ``_SkyColor`` ...);
* the painted ``colorRT``/``emissiveRT`` inputs and the debug views of ``jumpRT2``,
  ``distRT``, ``giRT1``, ``giRT2``, ``tempRT`` (RC2DGI.cs:156-163) ->
  :meth:`RC2DGI.upload` / :meth:`RC2DGI.download`.

Every call goes through ``librc2dgi.so`` (HIP kernels for gfx950).  There is no CPU
fallback: if the library is missing or the GPU call fails, this module raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librc2dgi.so")

# rc2dgi_rt (include/rc2dgi.h)
RT = {"color": 0, "emissive": 1, "jump1": 2, "jump2": 3, "dist": 4, "gi1": 5, "gi2": 6, "temp": 7, "blur": 8,
      "final_gi": 9}
SCREEN_RTS = ("color", "emissive", "jump1", "jump2", "dist", "temp")
FMT_RGBA8, FMT_RGBA32F = 0, 1
STATUS = {0: "OK", -1: "E_ARG", -2: "E_UNIFORM", -3: "E_HIP", -4: "E_OOM", -5: "E_UNSUPPORTED", -6: "E_STATE", -7: "E_DEVICE"}
PASS_NAMES = ("screenuv", "jfa", "rc", "blur", "merge", "total")


class RC2DGIError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"rc2dgi {STATUS.get(code, code)}: {msg}")
        self.code = code


class Prim(ctypes.Structure):
    """rc2dgi_prim: raylib DrawRectangleRec (kind 0) / DrawCircleV (kind 1, w = radius)."""
    _fields_ = [("kind", ctypes.c_int), ("x", ctypes.c_float), ("y", ctypes.c_float), ("w", ctypes.c_float),
                ("h", ctypes.c_float), ("r", ctypes.c_ubyte), ("g", ctypes.c_ubyte), ("b", ctypes.c_ubyte),
                ("a", ctypes.c_ubyte)]


class _Config(ctypes.Structure):
    _fields_ = [("screen_width", ctypes.c_int), ("screen_height", ctypes.c_int), ("cascade_count", ctypes.c_int),
                ("render_scale", ctypes.c_float), ("ray_range", ctypes.c_float), ("storage", ctypes.c_int),
                ("device", ctypes.c_int), ("flags", ctypes.c_int), ("reserved", ctypes.c_int * 4)]


_lib = None


def load_library(path: Optional[str] = None):
    """Load librc2dgi.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("RC2DGI_LIB") or LIB_PATH  # (an empty RC2DGI_LIB: the in-tree build)
    if not os.path.exists(path):
        raise RuntimeError(f"{path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                           "(there is no CPU fallback)")
    # One HIP runtime per process: PyTorch ships its own libamdhip64.so.7.  Loading torch first
    # makes this library bind to that copy instead of pulling a second runtime in later.
    try:
        import torch  # noqa: F401
    except Exception:  # torch is optional for the library itself
        pass
    L = ctypes.CDLL(path)
    vp, ip, fp = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_float)
    sig = {
        "rc2dgi_create": ([ctypes.POINTER(_Config), ctypes.POINTER(vp)], ctypes.c_int),
        "rc2dgi_destroy": ([vp], ctypes.c_int),
        "rc2dgi_set_uniform": ([vp, ctypes.c_char_p, fp, ctypes.c_int], ctypes.c_int),
        "rc2dgi_get_uniform": ([vp, ctypes.c_char_p, fp, ctypes.c_int], ctypes.c_int),
        "rc2dgi_set_uniform_i": ([vp, ctypes.c_char_p, ctypes.c_int], ctypes.c_int),
        "rc2dgi_upload": ([vp, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "rc2dgi_upload_device": ([vp, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "rc2dgi_do": ([vp], ctypes.c_int),
        "rc2dgi_sync": ([vp], ctypes.c_int),
        "rc2dgi_download": ([vp, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "rc2dgi_query": ([vp, ip, ip, ip, ip], ctypes.c_int),
        "rc2dgi_last_error": ([vp], ctypes.c_char_p),
        "rc2dgi_abi_version": ([], ctypes.c_int),
        "rc2dgi_set_stream": ([vp, vp], ctypes.c_int),
        "rc2dgi_set_timing": ([vp, ctypes.c_int], ctypes.c_int),
        "rc2dgi_pass_times": ([vp, fp, ctypes.c_int, fp, ctypes.c_int], ctypes.c_int),
        "rc2dgi_set_direction_table": ([vp, ctypes.c_int, fp, ctypes.c_int], ctypes.c_int),
        "rc2dgi_set_sky_table": ([vp, fp, ctypes.c_int], ctypes.c_int),
        "rc2dgi_set_keep_levels": ([vp, ctypes.c_int], ctypes.c_int),
        "rc2dgi_set_tuning": ([vp, ctypes.c_char_p, ctypes.c_int], ctypes.c_int),
        "rc2dgi_get_tuning": ([vp, ctypes.c_char_p, ip], ctypes.c_int),
        "rc2dgi_download_level": ([vp, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "rc2dgi_autotune": ([vp, ctypes.c_int], ctypes.c_int),
        "rc2dgi_paint": ([vp, ctypes.c_int, ctypes.POINTER(ctypes.c_ubyte), vp, ctypes.c_int], ctypes.c_int),
        "rc2dgi_set_shard": ([vp, ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "rc2dgi_shard_rows": ([vp, ip, ip], ctypes.c_int),
        "rc2dgi_shard_unique_id": ([vp, ctypes.c_int], ctypes.c_int),
        "rc2dgi_shard_connect": ([vp, vp, ctypes.c_int], ctypes.c_int),
        "rc2dgi_do_phase": ([vp, ctypes.c_int], ctypes.c_int),
        "rc2dgi_do_group": ([ctypes.POINTER(vp), ctypes.c_int], ctypes.c_int),
        "rc2dgi_device_buffer": ([vp, ctypes.c_int, ctypes.POINTER(vp), ip], ctypes.c_int),
        "rc2dgi_plan_rows": ([ctypes.POINTER(_Config), ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int, ip,
                              ctypes.c_int], ctypes.c_int),
        "rc2dgi_plan_jfa_exchange": ([ctypes.POINTER(_Config), ctypes.c_int, ctypes.c_int, ip, ip, ctypes.c_int],
                                     ctypes.c_int),
        "rc2dgi_plan_jfa_window": ([ctypes.POINTER(_Config), ctypes.c_int, ctypes.c_int, ctypes.c_int, ip, ip],
                                   ctypes.c_int),
        "rc2dgi_download_table": ([vp, ctypes.c_int, vp, ctypes.c_int], ctypes.c_int),
        "rc2dgi_plan_group_waits": ([ctypes.POINTER(_Config), ctypes.c_int, ctypes.c_int, ctypes.c_int, ip,
                                     ctypes.c_int], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def _fp(a: Optional[np.ndarray]):
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


class RC2DGI:
    """One GI context = the reference's render-texture set + DoRC2DGI() on one GPU."""

    def __init__(self, screen_width: int = 1200, screen_height: int = 900, cascade_count: int = 6,
                 render_scale: float = 1.0, ray_range: float = 2.0, device: int = 0, storage: str = "f32",
                 linux_merge_fallback: bool = False):
        """storage: "f32" (RGBA32F render textures), "f16" (giRT1/2 as RGBA16F, RC2DGI.cs:105-106) or
        "rgba8" (every render texture RGBA8 with GL unorm8 arithmetic -- the literal app).
        linux_merge_fallback: the app on a case-sensitive filesystem, where "shaders/Merge.fs" is not
        found (RC2DGI.cs:62) and the merge pass adds no GI to colorRT."""
        self._L = load_library()
        st = {"f32": 0, "rgba8": 1, "f16": 2}[storage]
        cfg = _Config(screen_width, screen_height, cascade_count, render_scale, ray_range, st, device,
                      1 if linux_merge_fallback else 0, (ctypes.c_int * 4)())
        h = ctypes.c_void_p()
        rc = self._L.rc2dgi_create(ctypes.byref(cfg), ctypes.byref(h))
        if rc != 0:
            raise RC2DGIError(rc, f"rc2dgi_create({screen_width}x{screen_height}, N={cascade_count}) failed")
        self._h = h
        self.screen_width, self.screen_height = screen_width, screen_height
        self.render_scale = render_scale
        self.device = device
        self.storage = storage
        self._N = cascade_count

    # ---------------------------------------------------------------- lifetime
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.rc2dgi_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc: int, what: str) -> None:
        if rc != 0:
            msg = self._L.rc2dgi_last_error(self._h)
            raise RC2DGIError(rc, f"{what}: {msg.decode() if msg else ''}")

    # ---------------------------------------------------------------- sizes
    def query(self):
        cw, ch, s, f = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self._check(self._L.rc2dgi_query(self._h, ctypes.byref(cw), ctypes.byref(ch), ctypes.byref(s),
                                         ctypes.byref(f)), "query")
        return cw.value, ch.value, s.value, f.value

    @property
    def cascade_resolution(self):
        """(CW, CH), RC2DGI.cs:70-77"""
        return self.query()[:2]

    @property
    def jfa_steps(self) -> int:
        return self.query()[2]

    @property
    def final_gi(self) -> int:
        """1 or 2: which giRT holds the final GI (RC2DGI.cs:365)."""
        return self.query()[3]

    # ---------------------------------------------------------------- uniforms
    def set_shader_value(self, name: str, value) -> None:
        """SetShaderValue(GI/blur shader, GetShaderLocation(name), value) for the host-set uniforms."""
        v = np.atleast_1d(np.asarray(value, dtype=np.float32)).ravel().copy()
        self._check(self._L.rc2dgi_set_uniform(self._h, name.encode(), _fp(v), v.size), f"set {name}")

    def get_shader_value(self, name: str):
        n = 3 if name in ("_SkyColor", "_SunColor") else 1
        v = np.zeros(n, np.float32)
        self._check(self._L.rc2dgi_get_uniform(self._h, name.encode(), _fp(v), n), f"get {name}")
        return tuple(float(x) for x in v) if n == 3 else float(v[0])

    @property
    def cascade_count(self) -> int:
        """cascadeCount (RC2DGI.cs:66); setting it reallocates the cascade textures."""
        return self._N

    @cascade_count.setter
    def cascade_count(self, n: int) -> None:
        self._check(self._L.rc2dgi_set_uniform_i(self._h, b"_CascadeCount", int(n)), "set _CascadeCount")
        self._N = int(n)

    ray_range = property(lambda s: s.get_shader_value("_RayRange"),
                         lambda s, v: s.set_shader_value("_RayRange", v))
    sky_radiance = property(lambda s: s.get_shader_value("_SkyRadiance"),
                            lambda s, v: s.set_shader_value("_SkyRadiance", v))
    sky_color = property(lambda s: s.get_shader_value("_SkyColor"),
                         lambda s, v: s.set_shader_value("_SkyColor", v))
    sun_color = property(lambda s: s.get_shader_value("_SunColor"),
                         lambda s, v: s.set_shader_value("_SunColor", v))
    sun_angle = property(lambda s: s.get_shader_value("_SunAngle"),
                         lambda s, v: s.set_shader_value("_SunAngle", v))
    reflectivity = property(lambda s: s.get_shader_value("_Reflectivity"),
                            lambda s, v: s.set_shader_value("_Reflectivity", v))
    cascade_blur_radius = property(lambda s: s.get_shader_value("_BlurRadius"),
                                   lambda s, v: s.set_shader_value("_BlurRadius", v))

    # ---------------------------------------------------------------- tables (parity pinning)
    def set_direction_table(self, level: int, cos_sin: Optional[np.ndarray]) -> None:
        a = None if cos_sin is None else np.ascontiguousarray(cos_sin, np.float32).reshape(-1, 2)
        n = 0 if a is None else a.shape[0]
        self._check(self._L.rc2dgi_set_direction_table(self._h, level, _fp(a), n), "set direction table")

    def set_sky_table(self, rgb: Optional[np.ndarray]) -> None:
        a = None if rgb is None else np.ascontiguousarray(rgb, np.float32).reshape(-1, 3)
        n = 0 if a is None else a.shape[0]
        self._check(self._L.rc2dgi_set_sky_table(self._h, _fp(a), n), "set sky table")

    # ---------------------------------------------------------------- I/O
    def upload(self, which: str, img) -> None:
        """Painted colorRT / emissiveRT (H, W, 4) in GL row order: numpy float32/uint8 (host) or a
        torch tensor on this context's GPU (device-resident, enqueued on the context stream)."""
        w = RT[which]
        if hasattr(img, "data_ptr") and getattr(img, "is_cuda", False):
            t = img
            if tuple(t.shape) != (self.screen_height, self.screen_width, 4):
                raise ValueError(f"expected ({self.screen_height}, {self.screen_width}, 4), got {tuple(t.shape)}")
            if not t.is_contiguous():
                raise ValueError("device tensor must be contiguous")
            fmt = FMT_RGBA32F if str(t.dtype) == "torch.float32" else FMT_RGBA8
            if fmt == FMT_RGBA8 and str(t.dtype) != "torch.uint8":
                raise TypeError("device tensor must be float32 or uint8")
            pitch = self.screen_width * (16 if fmt == FMT_RGBA32F else 4)
            self._check(self._L.rc2dgi_upload_device(self._h, w, ctypes.c_void_p(t.data_ptr()), pitch, fmt),
                        f"upload_device {which}")
            return
        a = np.asarray(img)
        if a.shape != (self.screen_height, self.screen_width, 4):
            raise ValueError(f"expected ({self.screen_height}, {self.screen_width}, 4), got {a.shape}")
        if a.dtype == np.uint8:
            a = np.ascontiguousarray(a)
            fmt, pitch = FMT_RGBA8, self.screen_width * 4
        else:
            a = np.ascontiguousarray(a, np.float32)
            fmt, pitch = FMT_RGBA32F, self.screen_width * 16
        self._check(self._L.rc2dgi_upload(self._h, w, a.ctypes.data_as(ctypes.c_void_p), pitch, fmt),
                    f"upload {which}")

    def paint(self, which: str, prims, clear=None) -> None:
        """BeginTextureMode(colorRT | emissiveRT); ClearBackground(clear); raylib rectangles /
        circles (RenderScene / RedrawSceneToRTs, RC2DGI.cs:224-264, 528-545) -- on the GPU.
        prims: (kind, x, y, w_or_radius, h, r, g, b, a) in raylib screen coordinates."""
        arr = (Prim * max(len(prims), 1))()
        for k, p in enumerate(prims):
            arr[k] = Prim(int(p[0]), float(p[1]), float(p[2]), float(p[3]), float(p[4]),
                          *(int(v) for v in p[5:9]))
        cl = None if clear is None else (ctypes.c_ubyte * 4)(*[int(v) for v in clear])
        self._check(self._L.rc2dgi_paint(self._h, RT[which], cl, arr, len(prims)), f"paint {which}")

    def download(self, which: str, dtype=np.float32) -> np.ndarray:
        w = RT[which]
        cw, ch, _, fin = self.query()
        if which in SCREEN_RTS:
            shape = (self.screen_height, self.screen_width, 4)
        else:
            shape = (ch, cw, 4)
        fmt = FMT_RGBA8 if dtype == np.uint8 else FMT_RGBA32F
        out = np.empty(shape, np.uint8 if fmt == FMT_RGBA8 else np.float32)
        self._check(self._L.rc2dgi_download(self._h, w, out.ctypes.data_as(ctypes.c_void_p),
                                            shape[1] * (4 if fmt == FMT_RGBA8 else 16), fmt), f"download {which}")
        return out

    def set_tuning(self, key: str, value: int) -> None:
        """Performance knobs (results are identical for every value), e.g. rc_variant."""
        self._check(self._L.rc2dgi_set_tuning(self._h, key.encode(), int(value)), f"set_tuning {key}")

    def get_tuning(self, key: str) -> int:
        v = ctypes.c_int()
        self._check(self._L.rc2dgi_get_tuning(self._h, key.encode(), ctypes.byref(v)), f"get_tuning {key}")
        return v.value

    def autotune(self, frames: int = 2) -> list:
        """Pick the fastest RC workgroup order per level on the uploaded scene (results are
        identical for every order); returns the chosen per-level codes."""
        self._check(self._L.rc2dgi_autotune(self._h, int(frames)), "autotune")
        return [self.get_tuning(f"rc_order_L{L}") for L in range(self._N)]

    def set_keep_levels(self, enable: bool = True) -> None:
        """Debug: keep every cascade level G_L as stored by its pass."""
        self._check(self._L.rc2dgi_set_keep_levels(self._h, int(bool(enable))), "set_keep_levels")

    def download_level(self, level: int) -> np.ndarray:
        cw, ch, _, _ = self.query()
        out = np.empty((ch, cw, 4), np.float32)
        self._check(self._L.rc2dgi_download_level(self._h, level, out.ctypes.data_as(ctypes.c_void_p), cw * 16,
                                                  FMT_RGBA32F), f"download_level {level}")
        return out

    TABLES = {"hitc": (0, np.uint8), "cmin": (1, np.uint8), "dclr": (2, np.uint8), "dboxes": (3, np.int32),
              "cellpal": (4, np.float32), "mfield": (5, np.uint16)}

    def download_table(self, name: str) -> np.ndarray:
        """The march's side tables of the last frame (rc2dgi_download_table): hitc / cmin (64, 64), dclr
        (64 bins, 64, 64), dboxes (64 bins, 64 steps, 4), cellpal (64, 64, 16, 4), mfield (H, pitch)."""
        which, dt = self.TABLES[name]
        n = self._L.rc2dgi_download_table(self._h, which, None, 0)
        self._check(n if n < 0 else 0, f"download_table {name}")
        out = np.empty(n // np.dtype(dt).itemsize, dt)
        self._check(min(0, self._L.rc2dgi_download_table(self._h, which, out.ctypes.data_as(ctypes.c_void_p), n)),
                    f"download_table {name}")
        shapes = {"hitc": (64, 64), "cmin": (64, 64), "dclr": (64, 64, 64), "dboxes": (64, 64, 4),
                  "cellpal": (64, 64, 16, 4), "mfield": (self.screen_height, -1)}
        return out.reshape(shapes[name])

    # ---------------------------------------------------------------- the pass chain
    def do_rc2dgi(self) -> None:
        """DoRC2DGI() (RC2DGI.cs:267-406): enqueue the whole pass chain on the context stream."""
        self._check(self._L.rc2dgi_do(self._h), "DoRC2DGI")

    do = do_rc2dgi

    def sync(self) -> None:
        self._check(self._L.rc2dgi_sync(self._h), "sync")

    def set_stream(self, hip_stream: Optional[int]) -> None:
        self._check(self._L.rc2dgi_set_stream(self._h, ctypes.c_void_p(hip_stream or 0)), "set_stream")

    def set_timing(self, enable=True) -> None:
        """True / 1: events around every pass and RC level; 2: around every pass only (no idle gaps
        between the levels); False / 0: off."""
        if isinstance(enable, bool):
            mode = int(enable)
        elif isinstance(enable, (int, np.integer)) and int(enable) in (0, 1, 2):
            mode = int(enable)
        else:
            raise ValueError(f"set_timing: expected a bool or 0, 1, 2, got {enable!r}")
        self._check(self._L.rc2dgi_set_timing(self._h, mode), "set_timing")

    def pass_times(self, levels: int = 0):
        """HIP-event milliseconds of the last frame: dict(screenuv, jfa, rc, blur, merge, total[, levels])."""
        p = np.zeros(len(PASS_NAMES), np.float32)
        lv = np.zeros(max(levels, 1), np.float32)
        self._check(self._L.rc2dgi_pass_times(self._h, _fp(p), p.size, _fp(lv) if levels else None, levels),
                    "pass_times")
        d = {k: float(v) for k, v in zip(PASS_NAMES, p)}
        if levels:
            d["levels"] = [float(x) for x in lv[:levels]]
        return d

    # ---------------------------------------------------------------- row-strip sharding
    def set_shard(self, rank: int, world: int) -> None:
        """Compute screen rows [rank*H/world, (rank+1)*H/world) of the merged colorRT (and what
        they depend on).  world = 1: the whole frame."""
        self._check(self._L.rc2dgi_set_shard(self._h, int(rank), int(world)), "set_shard")

    def shard_rows(self):
        y0, y1 = ctypes.c_int(), ctypes.c_int()
        self._check(self._L.rc2dgi_shard_rows(self._h, ctypes.byref(y0), ctypes.byref(y1)), "shard_rows")
        return y0.value, y1.value

    def connect(self, unique_id: bytes) -> None:
        """RCCL communicator over the shards (one process per GPU); then do_rc2dgi() runs the
        distRT exchange itself."""
        buf = ctypes.create_string_buffer(bytes(unique_id), UNIQUE_ID_BYTES)
        self._check(self._L.rc2dgi_shard_connect(self._h, buf, UNIQUE_ID_BYTES), "shard_connect")

    def do_phase(self, phase: int) -> None:
        """1: ScreenUV + JumpFlood + DistanceField; 2: cascades, blur, merge (exchange distRT between)."""
        self._check(self._L.rc2dgi_do_phase(self._h, int(phase)), f"do_phase {phase}")

    def device_buffer(self, which: str):
        """(device pointer, pitch in bytes) of a render texture's raw storage."""
        p, pitch = ctypes.c_void_p(), ctypes.c_int()
        self._check(self._L.rc2dgi_device_buffer(self._h, RT[which], ctypes.byref(p), ctypes.byref(pitch)),
                    f"device_buffer {which}")
        return p.value, pitch.value

    def frame(self, color, emissive) -> None:
        """Upload the painted scene and run one DoRC2DGI() (the reference's per-frame order,
        RC2DGI.cs:122-132)."""
        self.upload("color", color)
        self.upload("emissive", emissive)
        self.do_rc2dgi()


def abi_version() -> int:
    return load_library().rc2dgi_abi_version()


UNIQUE_ID_BYTES = 128
PLAN_JFA, PLAN_LEVEL, PLAN_BLUR, PLAN_MERGE = 0, 1000, 2000, 2001


def shard_unique_id() -> bytes:
    """RCCL unique id for rc2dgi_shard_connect (create on rank 0, send to the other ranks)."""
    L = load_library()
    buf = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
    rc = L.rc2dgi_shard_unique_id(buf, UNIQUE_ID_BYTES)
    if rc != 0:
        raise RC2DGIError(rc, "rc2dgi_shard_unique_id")
    return buf.raw


def do_group(ctxs: Sequence["RC2DGI"]) -> None:
    """One sharded frame over in-process contexts (context k = shard k of len(ctxs))."""
    L = load_library()
    arr = (ctypes.c_void_p * len(ctxs))(*[c._h.value for c in ctxs])
    rc = L.rc2dgi_do_group(arr, len(ctxs))
    if rc != 0:
        msgs = [c._L.rc2dgi_last_error(c._h) for c in ctxs]
        raise RC2DGIError(rc, "rc2dgi_do_group: " + "; ".join(m.decode() for m in msgs if m))


def plan_rows(W: int, H: int, N: int, blur_radius: float, rank: int, world: int, pass_id: int,
              render_scale: float = 1.0):
    """Host-only planner: [(begin, end), ...] rows shard `rank` of `world` computes for a pass
    (PLAN_JFA + step, PLAN_LEVEL + level, PLAN_BLUR, PLAN_MERGE)."""
    L = load_library()
    cfg = _Config(W, H, N, render_scale, 2.0, 0, 0, 0, (ctypes.c_int * 4)())
    buf = (ctypes.c_int * 64)()
    n = L.rc2dgi_plan_rows(ctypes.byref(cfg), float(blur_radius), rank, world, pass_id, buf, 32)
    if n < 0:
        raise RC2DGIError(n, "rc2dgi_plan_rows")
    if n > 32:
        buf = (ctypes.c_int * (2 * n))()
        n = L.rc2dgi_plan_rows(ctypes.byref(cfg), float(blur_radius), rank, world, pass_id, buf, n)
    return [(buf[2 * k], buf[2 * k + 1]) for k in range(n)]


JFA_INFO = ("m", "hmax", "mg_max", "halo", "sh_minus", "sh_zero", "sh_plus", "mg", "same_block")


def plan_jfa_exchange(W: int, H: int, N: int, world: int, step: int, render_scale: float = 1.0):
    """Host-only JumpFlood exchange plan of row-strip shards for JFA step `step` (>= 1): a dict of
    JFA_INFO and the transfers [(src, src_window_row, rows, dst, dst_buf, dst_row), ...] in the order
    every shard issues them (rc2dgi_plan_jfa_exchange)."""
    L = load_library()
    cfg = _Config(W, H, N, render_scale, 2.0, 0, 0, 0, (ctypes.c_int * 4)())
    info = (ctypes.c_int * 9)()
    n = L.rc2dgi_plan_jfa_exchange(ctypes.byref(cfg), world, step, info, None, 0)
    if n < 0:
        raise RC2DGIError(n, "rc2dgi_plan_jfa_exchange")
    buf = (ctypes.c_int * max(6 * n, 1))()
    L.rc2dgi_plan_jfa_exchange(ctypes.byref(cfg), world, step, info, buf, n)
    return dict(zip(JFA_INFO, list(info))), [tuple(buf[6 * k:6 * k + 6]) for k in range(n)]


def plan_group_waits(W: int, H: int, N: int, world: int, rank: int, step: int, render_scale: float = 1.0):
    """Host-only: the peers shard `rank` of a group frame awaits (their step step-1 done) before JFA step
    `step` (rc2dgi_plan_group_waits): (readers of its J_{step-2}, senders of the J_{step-1} rows it copies)."""
    L = load_library()
    cfg = _Config(W, H, N, render_scale, 2.0, 0, 0, 0, (ctypes.c_int * 4)())
    buf = (ctypes.c_int * max(2 * world, 1))()
    n = L.rc2dgi_plan_group_waits(ctypes.byref(cfg), world, rank, step, buf, 2 * world)
    if n < 0:
        raise RC2DGIError(n, "rc2dgi_plan_group_waits")
    got = list(buf[:n])
    return sorted(q for q in got if q >= 0), sorted(-1 - q for q in got if q < 0)


def plan_jfa_window(W: int, H: int, N: int, rank: int, world: int, step: int, render_scale: float = 1.0):
    """Where shard `rank` reads tap y of JFA step `step`: ([buffer per tap], [global row of each
    buffer's local row 0]) (rc2dgi_plan_jfa_window)."""
    L = load_library()
    cfg = _Config(W, H, N, render_scale, 2.0, 0, 0, 0, (ctypes.c_int * 4)())
    buf, row0 = (ctypes.c_int * 3)(), (ctypes.c_int * 3)()
    rc = L.rc2dgi_plan_jfa_window(ctypes.byref(cfg), rank, world, step, buf, row0)
    if rc < 0:
        raise RC2DGIError(rc, "rc2dgi_plan_jfa_window")
    return list(buf), list(row0)


__all__ = ["RC2DGI", "RC2DGIError", "load_library", "abi_version", "RT", "PASS_NAMES", "shard_unique_id", "do_group",
           "plan_rows", "plan_jfa_exchange", "plan_jfa_window", "PLAN_JFA", "PLAN_LEVEL", "PLAN_BLUR", "PLAN_MERGE"]
