#!/bin/bash
# rc_nblk: parity, then an interleaved A/B of direction blocks per one-probe workgroup at L3-L5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest -q -x tests/test_gpu_parity.py -k "direction_block or timing" --timeout 120 --timeout-method thread > gpurun_out/nblk_test.log 2>&1
rc=$?; tail -3 gpurun_out/nblk_test.log; [ $rc -eq 0 ] || exit $rc
CFGS="${CFGS:-base rc_nblk_L4=2 rc_nblk_L4=4 rc_nblk_L5=2 rc_nblk_L5=4 rc_nblk_L5=16}" ROUNDS=${ROUNDS:-2} bash scripts/ab_knobs.sh
