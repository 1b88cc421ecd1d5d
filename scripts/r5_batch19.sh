#!/bin/bash
# Round-5 batch 19: the bound-table exit proofs at L1 / L2 (the table's load and barrier cost ~5 k cycles per
# wave there) -- off per level (rc_noproof_L<n>) against on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TUNES="base:|np1:--tune rc_noproof_L1=1|np2:--tune rc_noproof_L2=1|np12:--tune rc_noproof_L1=1 --tune rc_noproof_L2=1|np3:--tune rc_noproof_L3=1" ROUNDS=3 bash scripts/ab_tunes.sh > gpurun_out/ab_noproof.txt 2>&1 || { cat gpurun_out/ab_noproof.txt; exit 1; }
cat gpurun_out/ab_noproof.txt
echo done
