#!/bin/bash
# Variant 20 (32x16x2 tiles, two waves per direction in the staging): parity of every variant, then A/B at L0-L2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest -q -x tests/test_gpu_parity.py -k "every_rc_variant and f32" --timeout 300 --timeout-method thread > gpurun_out/v20_test.log 2>&1
rc=$?; tail -3 gpurun_out/v20_test.log; [ $rc -eq 0 ] || exit $rc
CFGS="base rc_variant_L0=20 rc_variant_L1=20,rc_variant_L2=20 rc_variant_L0=20,rc_variant_L1=20,rc_variant_L2=20" ROUNDS=${ROUNDS:-3} bash scripts/ab_knobs.sh
