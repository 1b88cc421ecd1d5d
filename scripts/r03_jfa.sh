#!/bin/bash
# JumpFlood changes: parity tests of every JFA path, A/B against build/ab/librc2dgi_base.so, rocprof of the step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== test"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/jfa_test.log 2>&1
rc=$?; tail -3 gpurun_out/jfa_test.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B"
ROUNDS=${ROUNDS:-2} bash scripts/ab_lib.sh || exit $?
echo "== prof"
TAG=new bash scripts/prof_stats.sh || exit $?
