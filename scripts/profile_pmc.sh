#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, --kernel-trace only alongside) on the
# 4096^2 N=6 bench workload.  Output: gpurun_out/pmc/<group>/...counter_collection.csv
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
STEPS=${STEPS:-3}
if [ -n "$LIST" ]; then timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1; fi
i=0
for grp in ${GROUPS_OVERRIDE:-"FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" "TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"}; do
  i=$((i+1))
  echo "== pmc group $i: $grp"
  timeout -k 10 ${PMC_LIMIT:-300} rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/pmc/g$i -o run \
    -- python3 bench.py --steps $STEPS --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/pmc/g$i.log 2>&1
  rc=$?; echo "rc=$rc"; tail -2 gpurun_out/pmc/g$i.log
  [ $rc -eq 0 ] || exit $rc
done
