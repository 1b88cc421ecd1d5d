#!/bin/bash
# rocprofv3 --kernel-trace --stats of one bench configuration (BENCH_ARGS); summary to gpurun_out/prof_<TAG>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-run}
timeout -k 10 ${PROF_LIMIT:-300} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run \
  -- python3 bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline $BENCH_ARGS > gpurun_out/prof_$TAG.log 2>&1 || exit $?
f=$(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    print(f"{r['Name'][:70]:70s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:9.2f} pct {float(r['Percentage']):6.2f}")
PY
