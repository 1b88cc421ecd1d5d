#!/usr/bin/env python3
"""Pass times by HIP events (timing mode 2) of the committed bench frame, one line per frame, for a
comparison with the same frames' kernel trace (rocprofv3 --kernel-trace; scripts/frame_gaps.py)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from radiancecascade2dglobalillumination_amd import RC2DGI, scenes  # noqa: E402

W, N = 4096, 6
tun = json.load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                  "radiancecascade2dglobalillumination_amd/tuning/4096x4096_N6_rr2_f32.json")))
color, emis = scenes.demo(W, W)
g = RC2DGI(W, W, cascade_count=N)
g.upload("color", color)
g.upload("emissive", emis)
for L in range(N):
    g.set_tuning(f"rc_order_L{L}", tun["rc_order"][L])
    g.set_tuning(f"rc_variant_L{L}", tun["rc_variant"][L])
g.set_timing(2)
for f in range(8):
    g.do_rc2dgi()
    t = g.pass_times()
    print(f"frame {f}: " + " ".join(f"{k} {v:.4f}" for k, v in t.items()), flush=True)
g.close()
