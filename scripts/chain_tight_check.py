#!/usr/bin/env python3
"""rc_chain 3 (timing-only build: RC2DGI_LIB=build/ab/librc2dgi_tight.so from `_build.py exp tight
-DRC2DGI_DIAG_CHAIN_TIGHT`; waits only for the footprint inside the upper blocks) against the level-by-level
launches on one frame pair: does it still reproduce every level (C1 by default)?  Prints differing texel counts."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from radiancecascade2dglobalillumination_amd import RC2DGI, scenes  # noqa: E402

W, H, N = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (1200, 900, 6)))
c, e = scenes.demo(W, H)
g = RC2DGI(W, H, cascade_count=N)
g.set_keep_levels(True)
g.upload("color", c)
g.upload("emissive", e)
out = {}
for on in (0, 3):
    g.set_tuning("rc_chain", on)
    g.set_tuning("poison", 1)
    for f in range(2):
        g.do_rc2dgi()
        g.sync()
    out[on] = {f"G{L}": g.download_level(L) for L in range(N)}
    out[on]["color"] = g.download("color")
    print("rc_chain", on, "timeouts", g.get_tuning("rc_chain_timeouts"))
for k in out[0]:
    a, b = out[0][k], out[3][k]
    print(k, "differing texels", int(np.count_nonzero(np.any(a.view(np.uint32) != b.view(np.uint32), axis=-1))))
g.close()
