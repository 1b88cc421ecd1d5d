#!/usr/bin/env python3
"""Kernels of one whole frame of a rocprofv3 kernel trace with the idle gap before each one
(usage: frame_gaps.py run_kernel_trace.csv [k]: the k-th frame from the end, default 1 = the last;
bench.py's timed frames (timing mode 2) come before its per-level frames).  A frame starts at k_occupancy."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_occupancy" in r["Kernel_Name"]]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 1
lo, hi = (starts[-k - 1], starts[-k]) if len(starts) > k else (starts[-1], len(rows))
prev_end = None
for r in rows[lo:hi]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (st - prev_end) / 1e3 if prev_end is not None else 0.0
    print(f"{r['Kernel_Name'][:72]:72s} gap {gap:7.2f} us  dur {(en - st) / 1e3:8.2f} us")
    prev_end = en if prev_end is None else max(prev_end, en)
