#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp; mkdir -p gpurun_out
echo "== test"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "variant or proof or miss or tail or degenerate" > gpurun_out/t8_test.log 2>&1
rc=$?; tail -2 gpurun_out/t8_test.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B"
ROUNDS=2 TUNES="base:|l4v20:--tune rc_variant_L4=20|l4v21:--tune rc_variant_L4=21|l3v20:--tune rc_variant_L3=20|l5v20:--tune rc_variant_L5=20|l345:--tune rc_variant_L3=20 --tune rc_variant_L4=20 --tune rc_variant_L5=20" bash scripts/ab_tunes.sh
