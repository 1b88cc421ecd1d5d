#!/bin/bash
# Round-5 batch 8: the cascade chain's dependency window -- rc_chain 3 (only the footprint inside the upper blocks,
# no line widening) against 1 at C1: results and time.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
RC2DGI_LIB=$PWD/build/ab/librc2dgi_tight.so timeout -k 10 120 python scripts/chain_tight_check.py > gpurun_out/chain_tight_check.txt 2>&1 || { cat gpurun_out/chain_tight_check.txt; exit 1; }
cat gpurun_out/chain_tight_check.txt
RC2DGI_LIB=$PWD/build/ab/librc2dgi_tight.so BENCH_ARGS="--size 1200 --height 900" TUNES="sep:--tune rc_chain=0|ch:--tune rc_chain=1|tight:--tune rc_chain=3" ROUNDS=3 bash scripts/ab_tunes.sh > gpurun_out/ab_chain_tight.txt 2>&1 || { cat gpurun_out/ab_chain_tight.txt; exit 1; }
cat gpurun_out/ab_chain_tight.txt
echo done
