#!/bin/bash
# PMC of scripts/coalesce_probe: L1 -> L2 requests per gather instruction by sharing pattern
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/coalesce
timeout -k 10 60 ./scripts/coalesce_probe > gpurun_out/coalesce/run.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_BUSY_avr \
  --output-format csv -d gpurun_out/coalesce/pmc -o run -- ./scripts/coalesce_probe > gpurun_out/coalesce/pmc.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
rows = collections.defaultdict(dict)
names = {}
for f in glob.glob("gpurun_out/coalesce/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = int(r["Dispatch_Id"]); names[k] = r["Kernel_Name"].split("(")[0]
        rows[k][r["Counter_Name"]] = rows[k].get(r["Counter_Name"], 0) + float(r["Counter_Value"])
instr = 2048 * 4 * 64
for k in sorted(rows):
    c = rows[k]
    print(f"{names[k][:48]:48s} req/instr {c.get('TCP_TCC_READ_REQ_sum', 0) / instr:6.2f}  "
          f"accesses/instr {c.get('TCP_TOTAL_CACHE_ACCESSES_sum', 0) / instr:6.2f}  TA_BUSY_avr {c.get('TA_BUSY_avr', 0):.0f}")
PY
