#!/bin/bash
# Round-3 exploration on one GPU: the new parity tests, a bench line, then per-variant PMC of the
# L3-L5 march (lines requested, L2 hit rate, latency, instruction counts) for the tile / field
# layouts given in TAGS ("tag:bench args|...").
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  echo "== pytest $TESTS"
  timeout -k 10 ${PYTEST_LIMIT:-900} python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS \
    > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -15 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
if [ -n "$ESC" ]; then
  # the packed-field escape-load forms, one diagnostic library each (wrong texels are
  # reported, not faults)
  for lib in $ESC; do
    echo "== escape form $lib"
    RC2DGI_LIB=$PWD/$lib DBG_REPS=2 timeout -k 10 240 python -u scripts/dbg_packed_rolled.py > gpurun_out/esc_$(basename $lib .so).log 2>&1
    rc=$?; cat gpurun_out/esc_$(basename $lib .so).log | grep -v "^lib"; echo "rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
fi
echo "== bench"
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-400
if [ -n "$TAGS" ]; then
  GROUPS_AB="${GROUPS_AB:-TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum;SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_BUSY_avr}" \
    TAGS="$TAGS" bash scripts/pmc_ab.sh || exit $?
fi
