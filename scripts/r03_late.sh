#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp; mkdir -p gpurun_out
echo "== test late"
RC2DGI_LIB=$PWD/build/ab/librc2dgi_late.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "variant or fixture" > gpurun_out/late_test.log 2>&1
rc=$?; tail -2 gpurun_out/late_test.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B"
ROUNDS=3 LIBS="build/ab/librc2dgi_base.so build/ab/librc2dgi_late.so radiancecascade2dglobalillumination_amd/librc2dgi.so" bash scripts/ab_lib.sh || exit $?
echo "== timing late"
RC2DGI_LIB=$PWD/build/diag/librc2dgi_timing_late.so timeout -k 10 120 python scripts/rc_timing.py > gpurun_out/timing_late.json 2> gpurun_out/timing_late.err || exit 1
grep "^L" gpurun_out/timing_late.err
