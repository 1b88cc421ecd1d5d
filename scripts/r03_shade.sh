#!/bin/bash
# k_shade_cmin: parity (fused vs separate kernels), then an interleaved A/B of the RC pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -m pytest -q -x tests/test_gpu_parity.py -k "shade_cmin" --timeout 300 --timeout-method thread > gpurun_out/shade_test.log 2>&1
rc=$?; tail -2 gpurun_out/shade_test.log; [ $rc -eq 0 ] || exit $rc
CFGS="shade_fused=0 shade_fused=1" ROUNDS=${ROUNDS:-3} bash scripts/ab_knobs.sh
