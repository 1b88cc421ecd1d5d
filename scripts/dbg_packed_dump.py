"""GPU debug: dump one failing frame of the rolled packed march (variant 17, f32, 512^2 N=6) --
the distance field and every level -- for the CPU-side analysis of which rays go wrong."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np  # noqa: E402

from radiancecascade2dglobalillumination_amd import RC2DGI, scenes  # noqa: E402

W, N = 512, 6
color, emis = scenes.demo(W, W)
ctx = RC2DGI(W, W, cascade_count=N, ray_range=2.0)
ctx.set_keep_levels(True)
ctx.set_tuning("rc_variant", int(os.environ.get("V", "17")))
ctx.upload("color", color)
ctx.upload("emissive", emis)
out = {}
for rep in range(2):
    ctx.do_rc2dgi()
    ctx.sync()
    for L in range(N):
        out[f"r{rep}_L{L}"] = ctx.download_level(L)
out["dist"] = ctx.download("dist")
np.savez_compressed(os.path.join(os.path.dirname(__file__), "..", "gpurun_out", "dbg_packed_dump.npz"), **out)
print("dumped", flush=True)
