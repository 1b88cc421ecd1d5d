#!/bin/bash
# Round-end evidence on one GPU: bench line (with cpu_baseline), rocprofv3 kernel-trace stats of
# the same command, PMC FETCH/WRITE passes -> profiles/rc_level_pmc.json, batch-mode line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== bench"
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
echo "== rocprofv3 --kernel-trace --stats (same command, no cpu baseline)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
  -- python3 bench.py --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit $?
tail -1 gpurun_out/prof.log
echo "== pmc"
GROUPS_OVERRIDE="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum" STEPS=5 bash scripts/profile_pmc.sh || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc --json gpurun_out/rc_level_pmc.json > gpurun_out/pmc_summary.txt
cat gpurun_out/pmc_summary.txt | cut -c1-160
if [ -n "$BATCH" ]; then
  echo "== batch"
  timeout -k 10 400 python bench.py --batch $BATCH --steps 5 --warmup 1 > gpurun_out/batch.log 2>&1 || exit $?
  tail -1 gpurun_out/batch.log
fi
