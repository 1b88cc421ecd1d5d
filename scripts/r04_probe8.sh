#!/bin/bash
# round 4, probe 8: split levels (rc_split) and paired levels 1+0 (rc_pair) -- parity, then A/B on C1
# (1200x900) and the headline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "split_levels or paired_levels" > gpurun_out/r04/split_tests.log 2>&1 || { tail -30 gpurun_out/r04/split_tests.log; exit 1; }
tail -3 gpurun_out/r04/split_tests.log
ROUNDS=2 CFGS="base rc_pair=1 rc_split=56 rc_pair=1,rc_split=56" bash scripts/ab_knobs.sh || exit 1
V12="rc_variant_L1=0,rc_variant_L2=0"
BENCH_ARGS="--size 1200 --height 900" ROUNDS=2 CFGS="base rc_split=56 rc_split=62,$V12 $V12 rc_split=63,$V12,rc_variant_L0=0 rc_split=60,$V12 rc_split=48" bash scripts/ab_knobs.sh || exit 1
