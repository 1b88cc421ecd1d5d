#!/bin/bash
# round 4, probe 3: C1 kernel trace (where the app-size frame goes), the f16 / rgba8 4096^2 schedules
# (autotune, saved for commit), the C4 batch line at N=8 on a shared stream and on one stream per scene
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r04/c1prof -o c1 -- \
  python bench.py --size 1200 --height 900 --steps 20 --no-cpu-baseline > gpurun_out/r04/c1_bench.log 2>&1 || { tail -20 gpurun_out/r04/c1_bench.log; exit 1; }
tail -1 gpurun_out/r04/c1_bench.log | cut -c1-600
for st in f16 rgba8; do
  timeout -k 10 300 python bench.py --storage $st --autotune --no-cpu-baseline --steps 20 \
    --save-tuning gpurun_out/r04/4096x4096_N6_rr2_$st.json > gpurun_out/r04/tune_$st.log 2>&1 || { tail -20 gpurun_out/r04/tune_$st.log; exit 1; }
  tail -1 gpurun_out/r04/tune_$st.log | cut -c1-400
done
timeout -k 10 300 python bench.py --cascades 8 --autotune --no-cpu-baseline --steps 20 \
  --save-tuning gpurun_out/r04/4096x4096_N8_rr2_f32.json > gpurun_out/r04/tune_n8.log 2>&1 || { tail -20 gpurun_out/r04/tune_n8.log; exit 1; }
tail -1 gpurun_out/r04/tune_n8.log | cut -c1-400
mkdir -p /tmp/t && cp gpurun_out/r04/4096x4096_N8_rr2_f32.json radiancecascade2dglobalillumination_amd/tuning/
for bs in 1 0; do
  timeout -k 10 300 python bench.py --batch 8 --batch-streams $bs --cascades 8 --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/r04/c4_streams$bs.log 2>&1 || { tail -20 gpurun_out/r04/c4_streams$bs.log; exit 1; }
  tail -1 gpurun_out/r04/c4_streams$bs.log
done
