#!/bin/bash
# parity of the exit proofs / tail compaction, then RC bench lines over rc_tail settings
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "${TESTS:-exit_proofs or every_rc_variant or packed_fields}" > gpurun_out/t_tail.log 2>&1; rc=$?; tail -3 gpurun_out/t_tail.log; [ $rc -le 1 ] || exit $rc
for cfg in ${CFGS:-"rc_tail=0" "rc_tail=2" "rc_tail=3" "rc_tail=4" "rc_tail=6"}; do
  args=""; for kv in ${cfg//,/ }; do args="$args --tune $kv"; done
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 $BENCH_ARGS $args > gpurun_out/ab.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['rc_ms_per_frame'], d['rc_level_ms'], d['full_pipeline_ms'])"
done
