#!/bin/bash
# round 4, probe 7: re-tune C2 (4096^2 N=8 rr64) and C3 (8192^2 N=8 rr64) with the surface palettes on
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04; export TMPDIR=/tmp
timeout -k 10 400 python bench.py --cascades 8 --ray-range 64 --autotune --no-cpu-baseline --steps 10 \
  --save-tuning gpurun_out/r04/4096x4096_N8_rr64_f32.json > gpurun_out/r04/tune_c2.log 2>&1 || { tail -20 gpurun_out/r04/tune_c2.log; exit 1; }
tail -1 gpurun_out/r04/tune_c2.log | cut -c1-700
timeout -k 10 600 python bench.py --size 8192 --cascades 8 --ray-range 64 --autotune --no-cpu-baseline --steps 5 \
  --save-tuning gpurun_out/r04/8192x8192_N8_rr64_f32.json > gpurun_out/r04/tune_c3.log 2>&1 || { tail -20 gpurun_out/r04/tune_c3.log; exit 1; }
tail -1 gpurun_out/r04/tune_c3.log | cut -c1-700
