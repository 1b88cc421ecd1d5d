#!/bin/bash
# delta-coded 3-texel distance words (variants 20/21): parity, then per-level A/B on the committed schedule
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp; mkdir -p gpurun_out
echo "== test"
timeout -k 10 700 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py -k "variant or packed or proof or miss or tail or degenerate" > gpurun_out/tri_test.log 2>&1
rc=$?; tail -2 gpurun_out/tri_test.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B"
ROUNDS=2 TUNES="base:|l4v20:--tune rc_variant_L4=20|l4v21:--tune rc_variant_L4=21|l3v20:--tune rc_variant_L3=20|l5v21:--tune rc_variant_L5=21|l5v20:--tune rc_variant_L5=20|l2v20:--tune rc_variant_L2=20" bash scripts/ab_tunes.sh
