"""MI355X-native DoRC2DGI(): the 2-D radiance-cascades GI pass chain of
Hybrid46/RadianceCascade2DGlobalIllumination as hand-written gfx950 HIP kernels behind
a C ABI (include/rc2dgi.h, librc2dgi.so).

* :class:`RC2DGI` -- host mirror of the reference's DoRC2DGI()/SetGIShaderValues()
  operator interface (rc2dgi.py);
* :mod:`scenes` -- synthetic painted-scene inputs for tests and benchmarks.
"""
from .rc2dgi import RC2DGI, RC2DGIError, abi_version, load_library  # noqa: F401

__all__ = ["RC2DGI", "RC2DGIError", "abi_version", "load_library"]
