#!/bin/bash
# one experiment: GPU parity suite (or TESTK subset), then A/B against build/ab/librc2dgi_base.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== test"
if [ -n "$TESTK" ]; then SEL=(-k "$TESTK" tests); else SEL=(-m gpu tests); fi
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "${SEL[@]}" > gpurun_out/ab_test.log 2>&1
rc=$?; tail -3 gpurun_out/ab_test.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B"
ROUNDS=${ROUNDS:-3} bash scripts/ab_lib.sh || exit $?
if [ -n "$PROF" ]; then echo "== prof"; TAG=new bash scripts/prof_stats.sh || exit $?; fi
