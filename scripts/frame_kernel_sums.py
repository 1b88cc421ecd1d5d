#!/usr/bin/env python3
"""Per-frame GPU time by kernel from a rocprofv3 kernel trace (run_kernel_trace.csv) of bench.py:
the trace holds FRAMES frames (warmup + steps) with the same number of k_occupancy launches each;
the last STEPS frames (the timed ones) are summed, and the GPU-busy time (union of the kernel
intervals) and the span are printed.  Usage: frame_kernel_sums.py FRAMES STEPS TRACE.csv [TRACE2.csv]"""
import csv
import sys


def sums(path, frames, steps):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    occ = [i for i, r in enumerate(rows) if "k_occupancy" in r["Kernel_Name"]]
    per = len(occ) // frames  # occupancy launches per frame (a shard may launch several row intervals)
    first = occ[-steps * per]  # the first occupancy launch of the timed frames
    out = {}
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows[first:])
    busy, (cs, ce) = 0, iv[0]
    for s0, e0 in iv[1:]:
        if s0 > ce:
            busy, cs, ce = busy + ce - cs, s0, e0
        else:
            ce = max(ce, e0)
    busy += ce - cs
    out["(GPU busy, union of kernels)"] = busy / 1e6 / steps
    out["(span, first to last kernel)"] = (max(e for _, e in iv) - iv[0][0]) / 1e6 / steps
    for r in rows[first:]:
        k = r["Kernel_Name"].split("(")[0][:64]
        out[k] = out.get(k, 0.0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 / steps
    return out


def main():
    a = sys.argv[1:]
    frames, steps = int(a[0]), int(a[1])
    u = sums(a[2], frames, steps)
    s = sums(a[3], frames, steps) if len(a) > 3 else {}
    for k in sorted(set(u) | set(s), key=lambda k: -max(u.get(k, 0), s.get(k, 0))):
        print(f"{k:64s} {u.get(k, 0):8.3f} {s.get(k, 0):8.3f}  {s.get(k, 0) - u.get(k, 0):+8.3f}")
    tot = lambda d: sum(v for k, v in d.items() if not k.startswith("("))  # noqa: E731
    print(f"{'kernel sum (ms per frame)':64s} {tot(u):8.3f} {tot(s):8.3f}")


if __name__ == "__main__":
    main()
