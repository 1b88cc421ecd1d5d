#!/bin/bash
# Round-end evidence on one GPU, for the schedule the bench times (the committed per-config
# schedule in radiancecascade2dglobalillumination_amd/tuning/, or TUNE=1: autotune and save it):
#   1. rocprofv3 --kernel-trace --stats of the bench;
#   2. PMC FETCH/WRITE/TCC/SQ_INSTS_VALU passes of the same, per scene -> profiles/rc_level_pmc.json (HBM traffic
#      and VALU wave instructions per launch, one record per config / scene / schedule);
#   3. the final bench line (with cpu_baseline), reading the fresh traffic;
#   4. optional batch-mode line (BATCH=<scenes per GPU>).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
SCHED=""
if [ -n "$TUNE" ]; then
  echo "== tune"
  timeout -k 10 300 python bench.py --autotune --no-cpu-baseline --steps 5 --save-tuning gpurun_out/tuning.json \
    > gpurun_out/tune.log 2>&1 || exit $?
  SCHED="--load-tuning gpurun_out/tuning.json"
fi
echo "== rocprofv3 --kernel-trace --stats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
  -- python3 bench.py --no-cpu-baseline $SCHED > gpurun_out/prof.log 2>&1 || exit $?
tail -1 gpurun_out/prof.log | cut -c1-200
# PMC records per scene (PMC_SCENES, default the demo frame and one random and one dense scene): each keyed on its
# config, scene and schedule, merged into profiles/rc_level_pmc.json (bench.py uses a record only for its own key)
for sc in ${PMC_SCENES:-demo random:1 dense:0}; do
  echo "== pmc $sc"
  rm -rf gpurun_out/pmc
  GROUPS_OVERRIDE="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_INSTS_VALU SQ_WAVES" STEPS=5 BENCH_ARGS="$SCHED --scene $sc" \
    bash scripts/profile_pmc.sh || exit $?
  tag=${sc//:/}
  python3 scripts/pmc_summary.py gpurun_out/pmc --json gpurun_out/rc_level_pmc.json --merge profiles/rc_level_pmc.json \
    > gpurun_out/pmc_summary_$tag.txt || exit $?
  cut -c1-160 gpurun_out/pmc_summary_$tag.txt
  cp gpurun_out/rc_level_pmc.json profiles/rc_level_pmc.json
done
echo "== bench"
timeout -k 10 400 python bench.py $SCHED > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-200
if [ -n "$BATCH" ]; then
  echo "== batch"
  timeout -k 10 400 python bench.py --batch $BATCH --steps 5 --warmup 1 > gpurun_out/batch.log 2>&1 || exit $?
  tail -1 gpurun_out/batch.log | cut -c1-200
fi
