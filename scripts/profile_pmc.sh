#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, --kernel-trace only alongside) on the
# 4096^2 N=6 bench workload.  Output: gpurun_out/pmc/<group>/...counter_collection.csv
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
STEPS=${STEPS:-3}
if [ -n "$LIST" ]; then timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1; fi
# counter groups separated by ';' (counters inside a group by spaces)
GROUPS_STR=${GROUPS_OVERRIDE:-"FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES;TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"}
IFS=';' read -r -a GRPS <<< "$GROUPS_STR"
# refuse unknown counter names up front (an unknown name made rocprofv3 hang once)
for grp in "${GRPS[@]}"; do for c in $grp; do
  grep -qx "$c" scripts/gfx950_counters.txt || { echo "unknown counter $c"; exit 2; }
done; done
i=0
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  echo "== pmc group $i: $grp"
  timeout -k 10 ${PMC_LIMIT:-180} rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/pmc/g$i -o run \
    -- python3 bench.py --steps $STEPS --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/pmc/g$i.log 2>&1
  rc=$?; echo "rc=$rc"; tail -2 gpurun_out/pmc/g$i.log
  [ $rc -eq 0 ] || exit $rc
done
