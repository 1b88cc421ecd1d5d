#!/bin/bash
# Round-5 batch 21: L4 march unrolled (variant 13) against rolled (0) under the interleaved order; L5 rolled.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TUNES="base:|l4v13:--tune rc_variant_L4=13|l5v0:--tune rc_variant_L5=0|l3v0:--tune rc_variant_L3=0" ROUNDS=4 bash scripts/ab_tunes.sh > gpurun_out/ab_l4var.txt 2>&1 || { cat gpurun_out/ab_l4var.txt; exit 1; }
cat gpurun_out/ab_l4var.txt
echo done
