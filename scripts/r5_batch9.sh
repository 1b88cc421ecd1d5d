#!/bin/bash
# Round-5 batch 9: the cascade chain with the top level in the launch (rc_chain 4): parity, C1 timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "cascade_chain" > gpurun_out/b9_tests.log 2>&1 || { tail -30 gpurun_out/b9_tests.log; exit 1; }
tail -1 gpurun_out/b9_tests.log
BENCH_ARGS="--size 1200 --height 900" TUNES="sep:--tune rc_chain=0|ch:--tune rc_chain=1|ch4:--tune rc_chain=4" ROUNDS=4 bash scripts/ab_tunes.sh > gpurun_out/ab_chain_top.txt 2>&1 || { cat gpurun_out/ab_chain_top.txt; exit 1; }
cat gpurun_out/ab_chain_top.txt
echo done
