#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (scripts/profile_pmc.sh) per kernel and per RC level.

RC-level dispatches are identified by their order inside each frame (levels N-1..0).
FETCH_SIZE / WRITE_SIZE are in KB (rocprofv3); on gfx950 FETCH_SIZE under-reports a wide
coalesced stream by 2x (MI355X_MICROARCH.md §HBM) -- both the raw value and the x2
calibrated value are printed.
Usage: scripts/pmc_summary.py gpurun_out/pmc [--levels 6] [--json out.json [--merge profiles/rc_level_pmc.json]]
The record is keyed on what it was measured on (bench.py's `pmc_key`: config, rayRange, storage, scene, schedule,
knobs), read from the bench line of the first pass's log; --merge replaces the record of the same key in an
existing file and keeps the others (bench.py only uses a record whose key matches its own run).
"""
import argparse
import collections
import csv
import glob
import json
import os


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "g*", "*counter_collection.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                r["_file"] = f
                rows.append(r)
    return rows


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("rc2dgi::", "")
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--levels", type=int, default=6)
    ap.add_argument("--json")
    ap.add_argument("--merge", help="existing records file to merge the new record into")
    ap.add_argument("--all", action="store_true", help="print every collected counter")
    a = ap.parse_args()
    rows = load(a.dir)
    # per (file, dispatch): counters
    disp = collections.defaultdict(dict)
    meta = {}
    for r in rows:
        key = (r["_file"], int(r["Dispatch_Id"]))
        disp[key][r["Counter_Name"]] = disp[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[key] = (short(r["Kernel_Name"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    # RC levels: in each file, rc_level dispatches come in groups of N (levels N-1 .. 0)
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    by_file = collections.defaultdict(list)
    for key in sorted(disp):
        by_file[key[0]].append(key)
    for f, keys in by_file.items():
        rc_seen = 0
        for key in keys:
            name, dur = meta[key]
            if name.startswith("k_rc_level"):
                lvl = a.levels - 1 - (rc_seen % a.levels)
                rc_seen += 1
                name = f"k_rc_level L{lvl}"
            for c, v in disp[key].items():
                per[name][c].append(v)
            per[name]["_dur_ns"].append(dur)
    out = {}
    for name in sorted(per):
        d = per[name]
        avg = {c: sum(v) / len(v) for c, v in d.items()}
        out[name] = avg
        s = f"{name:22s} dur {avg['_dur_ns'] / 1e3:8.1f} us"
        if "FETCH_SIZE" in avg:
            s += f"  FETCH {avg['FETCH_SIZE'] / 1024:8.1f} MB (x2 {2 * avg['FETCH_SIZE'] / 1024:8.1f})"
        if "WRITE_SIZE" in avg:
            s += f"  WRITE {avg['WRITE_SIZE'] / 1024:8.1f} MB"
        if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
            h, m = avg["TCC_HIT_sum"], avg["TCC_MISS_sum"]
            s += f"  L2hit {h / max(h + m, 1):.3f} (req {(h + m) / 1e6:.1f}M)"
        shown = ("SQ_WAVES", "SQ_INSTS_VMEM", "SQ_WAIT_INST_ANY", "SQ_BUSY_CYCLES", "TA_BUSY_avr",
                 "TCP_TOTAL_CACHE_ACCESSES_sum", "TCP_TCC_READ_REQ_sum")
        for c in (sorted(k for k in avg if not k.startswith("_") and k not in ("FETCH_SIZE", "WRITE_SIZE"))
                  if a.all else shown):
            if c in avg:
                s += f"  {c} {avg[c]:.3g}"
        print(s)
    if a.json:
        lv = {k: v for k, v in out.items() if k.startswith("k_rc_level")}
        fetch = [v.get("FETCH_SIZE") for v in lv.values()]
        write = [v.get("WRITE_SIZE") for v in lv.values()]
        key = None
        for lg in sorted(glob.glob(os.path.join(a.dir, "g*.log"))):
            for line in open(lg):
                if line.startswith("{") and '"pmc_key"' in line:
                    key = json.loads(line)["pmc_key"]
            if key:
                break
        if key is None:
            raise SystemExit("no bench line with a pmc_key in the passes' logs")
        rec = {"key": key, "config": key["config"], "kernel": "k_rc_level",
               "note": "HBM bytes per RC-level launch from rocprofv3 PMC (separate passes): "
                       "(2*FETCH_SIZE + WRITE_SIZE)*1024, FETCH doubled per MI355X_MICROARCH.md §HBM",
               "per_level": {k: {"fetch_kb": v.get("FETCH_SIZE"), "write_kb": v.get("WRITE_SIZE"),
                                 "l2_requests": (v["TCC_HIT_sum"] + v["TCC_MISS_sum"]) if "TCC_HIT_sum" in v else None,
                                 "l2_hit": (v["TCC_HIT_sum"] / max(v["TCC_HIT_sum"] + v["TCC_MISS_sum"], 1))
                                 if "TCC_HIT_sum" in v else None,
                                 "valu_insts": v.get("SQ_INSTS_VALU"),
                                 "dur_us": v["_dur_ns"] / 1e3} for k, v in lv.items()}}
        if all(x is not None for x in fetch + write) and lv:
            rec["hbm_bytes_per_launch"] = sum(2 * f * 1024 + w * 1024 for f, w in zip(fetch, write)) / len(lv)
        recs = []
        if a.merge and os.path.exists(a.merge):
            with open(a.merge) as fh:
                recs = [r for r in json.load(fh).get("records", []) if r.get("key") != key]
        with open(a.json, "w") as fh:
            json.dump({"records": recs + [rec]}, fh, indent=1)


if __name__ == "__main__":
    main()
