#!/bin/bash
# Pick the committed RC schedules (radiancecascade2dglobalillumination_amd/tuning/) on one MI355X:
# autotune each BASELINE config the bench times and save the picks to gpurun_out/ (copy them over).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --autotune --no-cpu-baseline --steps 20 --save-tuning gpurun_out/4096x4096_N6_rr2_f32.json > gpurun_out/tune_h.log 2>&1 || exit $?
tail -1 gpurun_out/tune_h.log | cut -c1-900
timeout -k 10 300 python bench.py --autotune --no-cpu-baseline --steps 20 --cascades 8 --ray-range 64 --save-tuning gpurun_out/4096x4096_N8_rr64_f32.json > gpurun_out/tune_c2.log 2>&1 || exit $?
tail -1 gpurun_out/tune_c2.log | cut -c1-900
timeout -k 10 300 python bench.py --autotune --no-cpu-baseline --steps 20 --size 1200 --height 900 --save-tuning gpurun_out/1200x900_N6_rr2_f32.json > gpurun_out/tune_c1.log 2>&1 || exit $?
tail -1 gpurun_out/tune_c1.log | cut -c1-900
