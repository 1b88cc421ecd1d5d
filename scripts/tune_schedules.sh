#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --autotune --no-cpu-baseline --steps 20 --save-tuning gpurun_out/t_4096x4096_N6.json > gpurun_out/tune_h.log 2>&1 || exit $?
tail -1 gpurun_out/tune_h.log | cut -c1-900
timeout -k 10 300 python bench.py --autotune --no-cpu-baseline --steps 20 --cascades 8 --ray-range 64 --save-tuning gpurun_out/t_4096x4096_N8.json > gpurun_out/tune_c2.log 2>&1 || exit $?
tail -1 gpurun_out/tune_c2.log | cut -c1-900
timeout -k 10 300 python bench.py --autotune --no-cpu-baseline --steps 20 --size 1200 --height 900 --save-tuning gpurun_out/t_1200x900_N6.json > gpurun_out/tune_c1.log 2>&1 || exit $?
tail -1 gpurun_out/tune_c1.log | cut -c1-900
