#!/usr/bin/env python3
"""JumpFlood pass time (HIP events, timing mode 2) of the bench frame for settings of one knob, interleaved.
Usage: jfa_pass.py KEY V1 V2 [--size W] [--rounds R] [--frames F]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from radiancecascade2dglobalillumination_amd import RC2DGI, scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("key")
ap.add_argument("values", nargs="+", type=int)
ap.add_argument("--size", type=int, default=4096)
ap.add_argument("--cascades", type=int, default=6)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--frames", type=int, default=20)
a = ap.parse_args()
color, emis = scenes.demo(a.size, a.size)
g = RC2DGI(a.size, a.size, cascade_count=a.cascades)
g.upload("color", color)
g.upload("emissive", emis)
g.set_timing(2)
for _ in range(3):
    g.do_rc2dgi()
for r in range(a.rounds):
    for v in a.values:
        g.set_tuning(a.key, v)
        g.do_rc2dgi()
        t = []
        for _ in range(a.frames):
            g.do_rc2dgi()
            t.append(g.pass_times())
        jfa = np.median([x["jfa"] for x in t])
        tot = np.median([x["total"] for x in t])
        rc = np.median([x["rc"] for x in t])
        print(f"{a.key}={v} jfa {jfa:.4f} ms  rc {rc:.4f} ms  frame {tot:.4f} ms", flush=True)
g.close()
