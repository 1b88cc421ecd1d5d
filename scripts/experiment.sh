#!/bin/bash
# One GPU experiment on one box, parameterised by environment variables; every step is optional and
# they run in this order, the run stopping at the first failure:
#   TESTK       pytest -k expression over the GPU tests (tests/, -m gpu); TESTLIB: a library to test instead
#   LIBS        library builds to A/B, interleaved ROUNDS times (scripts/ab_lib.sh; BENCH_ARGS passed on)
#   CFGS        tuning-knob settings to A/B on the committed schedule (scripts/ab_knobs.sh)
#   PROBE       scripts/sched_probe.py arguments: per-level (variant, order) probe; PROBE_LIB: library to use
#   PROF        a tag: rocprofv3 kernel-trace stats of a bench run (scripts/prof_stats.sh) -> gpurun_out/prof_<tag>
# e.g.  TESTK="variant" PROBE="3:c,20:c 4:c,20:c" gpurun -- bash scripts/experiment.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -n "$TESTK" ]; then
  echo "== test: $TESTK"
  RC2DGI_LIB=${TESTLIB:+$PWD/$TESTLIB} timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest -x -q --timeout 300 \
    --timeout-method thread -m gpu -k "$TESTK" tests > gpurun_out/exp_test.log 2>&1
  rc=$?; tail -3 gpurun_out/exp_test.log; [ $rc -eq 0 ] || exit $rc
fi
#   AB_ARGS     ';'-separated bench argument sets for the LIBS A/B (default: the headline only), e.g.
#               AB_ARGS="; --size 4096 --cascades 8 --ray-range 64"
if [ -n "$LIBS" ]; then
  IFS=';' read -r -a ABS <<< "${AB_ARGS:-}"
  [ ${#ABS[@]} -eq 0 ] && ABS=("")
  for args in "${ABS[@]}"; do
    echo "== A/B libraries: ${args:-headline}"
    BENCH_ARGS="$args" ROUNDS=${ROUNDS:-3} bash scripts/ab_lib.sh || exit $?
  done
fi
if [ -n "$CFGS" ]; then echo "== A/B knobs"; ROUNDS=${ROUNDS:-3} bash scripts/ab_knobs.sh || exit $?; fi
if [ -n "$PROBE" ]; then
  echo "== schedule probe: $PROBE"
  RC2DGI_LIB=${PROBE_LIB:+$PWD/$PROBE_LIB} timeout -k 10 ${PROBE_LIMIT:-400} python -u scripts/sched_probe.py \
    $PROBE_ARGS $PROBE > gpurun_out/exp_probe.json 2> gpurun_out/exp_probe.err || { tail -20 gpurun_out/exp_probe.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/exp_probe.json'):
    d = json.loads(l); print('L%d' % d['level'], 'committed', d['committed'], 'best', d['ms_variant_order'][:6])"
fi
if [ -n "$PROF" ]; then echo "== rocprofv3"; TAG=$PROF bash scripts/prof_stats.sh || exit $?; fi
