#!/bin/bash
# df_side parity test, A/B of df_side, per-kernel rocprof of both, then march stats + stall PMC (round 3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== test"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "df_side" > gpurun_out/side_test.log 2>&1
rc=$?; tail -3 gpurun_out/side_test.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B"
ROUNDS=2 TUNES="base:|noside:--tune df_side=0" bash scripts/ab_tunes.sh || exit $?
echo "== prof"
TAG=side bash scripts/prof_stats.sh || exit $?
TAG=noside BENCH_ARGS="--tune df_side=0" bash scripts/prof_stats.sh || exit $?
bash scripts/r03_diag2.sh
