#!/bin/bash
# Round-5 batch 11: headline knob A/B on the final schedule (workgroup-wide proof, exit-proof modes, fused records).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TUNES="base:|wgp0:--tune rc_wgproof=0|skip2:--tune rc_skip=2|skip3:--tune rc_skip=3|nofuse:--tune shade_fused=0" ROUNDS=3 bash scripts/ab_tunes.sh > gpurun_out/ab_knobs_h.txt 2>&1 || { cat gpurun_out/ab_knobs_h.txt; exit 1; }
cat gpurun_out/ab_knobs_h.txt
echo done
