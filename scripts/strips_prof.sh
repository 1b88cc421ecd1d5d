#!/bin/bash
# Per-kernel time of the C3 frame (8192^2, N=8, rayRange 64) unsharded and as 8 in-process row strips
# (rocprofv3 kernel-trace stats; scripts/frame_kernel_sums.py).  Output: gpurun_out/strips_prof/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/strips_prof; export TMPDIR=/tmp
for m in whole strips8; do
  args="--size 8192 --cascades 8 --ray-range 64 --steps 5 --warmup 2 --no-cpu-baseline"
  [ $m = strips8 ] && args="$args --mode strips --shards 8"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/strips_prof/$m -o run \
    -- python3 bench.py $args > gpurun_out/strips_prof/$m.log 2>&1 || { tail -5 gpurun_out/strips_prof/$m.log; exit 1; }
  tail -1 gpurun_out/strips_prof/$m.log | cut -c1-200
  f=$(find gpurun_out/strips_prof/$m -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:16]:
    print(f"{r['Name'][:72]:72s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:9.2f} tot_ms {float(r['TotalDurationNs'])/1e6:8.2f}")
PY
done
