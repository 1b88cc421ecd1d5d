#!/bin/bash
# Round-end evidence on one GPU:
#   1. bench (no CPU baseline) picks the schedule (autotune) and saves it;
#   2. rocprofv3 --kernel-trace --stats of the bench replaying that schedule;
#   3. PMC FETCH/WRITE/TCC passes of the same -> profiles/rc_level_pmc.json (HBM traffic per launch);
#   4. the final bench line (with cpu_baseline), same schedule, reading the fresh traffic;
#   5. optional batch-mode line (BATCH=<scenes per GPU>).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== tune"
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --save-tuning gpurun_out/tuning.json \
  > gpurun_out/tune.log 2>&1 || exit $?
echo "== rocprofv3 --kernel-trace --stats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
  -- python3 bench.py --no-cpu-baseline --load-tuning gpurun_out/tuning.json > gpurun_out/prof.log 2>&1 || exit $?
tail -1 gpurun_out/prof.log
echo "== pmc"
GROUPS_OVERRIDE="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum" STEPS=5 BENCH_ARGS="--load-tuning gpurun_out/tuning.json" \
  bash scripts/profile_pmc.sh || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc --json gpurun_out/rc_level_pmc.json > gpurun_out/pmc_summary.txt
cut -c1-160 gpurun_out/pmc_summary.txt
cp gpurun_out/rc_level_pmc.json profiles/rc_level_pmc.json
echo "== bench"
timeout -k 10 400 python bench.py --load-tuning gpurun_out/tuning.json > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
if [ -n "$BATCH" ]; then
  echo "== batch"
  timeout -k 10 400 python bench.py --batch $BATCH --steps 5 --warmup 1 > gpurun_out/batch.log 2>&1 || exit $?
  tail -1 gpurun_out/batch.log
fi
