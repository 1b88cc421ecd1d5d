#!/bin/bash
# Round-5 batch 7: exit / directional proofs at C1 (rc_skip 2, 3; auto leaves them off below 2048), with and
# without the cascade chain.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
BENCH_ARGS="--size 1200 --height 900" TUNES="auto:--tune rc_chain=0|s2:--tune rc_chain=0 --tune rc_skip=2|s3:--tune rc_chain=0 --tune rc_skip=3|ch:--tune rc_chain=1|ch_s2:--tune rc_chain=1 --tune rc_skip=2|ch_s3:--tune rc_chain=1 --tune rc_skip=3" ROUNDS=3 bash scripts/ab_tunes.sh > gpurun_out/ab_c1_proofs.txt 2>&1 || { cat gpurun_out/ab_c1_proofs.txt; exit 1; }
cat gpurun_out/ab_c1_proofs.txt
echo done
