"""GPU debug: the packed-field marches (16/17 unrolled, 18/19 rolled) in a fresh
context: per-level mismatches vs the oracle and run-to-run determinism.  The product passes; the
diagnostic build that waits for the escape loads at the branch join instead of right after each
(python -m radiancecascade2dglobalillumination_amd._build escplain -> build/diag/librc2dgi_escplain.so;
extra flags such as -DRC2DGI_DIAG_LDS_PAD=30000 pass through) reproduces the failure.
Run with RC2DGI_LIB=<library>, DBG_CASES=rolled|unrolled, DBG_REPS=<frames>."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np  # noqa: E402

import oracle  # noqa: E402
from radiancecascade2dglobalillumination_amd import RC2DGI, scenes  # noqa: E402

print("lib", os.environ.get("RC2DGI_LIB", "default"), flush=True)
CASES = {"rolled": (("f32", 512, 6, 18), ("f16", 512, 6, 18), ("f32", 512, 6, 19), ("f16", 512, 6, 19),
                    ("f32", 512, 6, 16), ("f32", 512, 6, 17)),
         "unrolled": (("f16", 1024, 6, 17), ("f32", 1024, 6, 17), ("f16", 1024, 6, 16), ("f32", 1024, 6, 16),
                      ("f16", 512, 6, 17), ("f16", 2048, 6, 17))}[os.environ.get("DBG_CASES", "rolled")]
REPS = int(os.environ.get("DBG_REPS", "3"))
for storage, W, N, v in CASES:
    color, emis = scenes.demo(W, W)
    fr = oracle.frame(oracle.Params(W=W, H=W, N=N, ray_range=2.0, gi_f16=storage == "f16"), color, emis,
                      keep_levels=True)
    ctx = RC2DGI(W, W, cascade_count=N, ray_range=2.0, storage=storage)
    ctx.set_keep_levels(True)
    ctx.set_tuning("rc_variant", v)
    ctx.upload("color", color)
    ctx.upload("emissive", emis)
    prev = None
    for rep in range(REPS):
        ctx.do_rc2dgi()
        ctx.sync()
        lv = [ctx.download_level(L) for L in range(N)]
        bad = [int(np.count_nonzero(np.any(lv[L] != fr.gi_levels[L], axis=-1))) for L in range(N)]
        same = None if prev is None else all(np.array_equal(a, b) for a, b in zip(prev, lv))
        print(f"{storage} {W}^2 N{N} v{v} run {rep}: bad texels per level {bad}; same as previous: {same}", flush=True)
        prev = lv
    ctx.close()
