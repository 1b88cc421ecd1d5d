#!/bin/bash
# Round-5 batch 12: rows per lane of the small-screen JumpFlood steps (jfa_rt): parity, C1 frame A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "jfa_rows_per_lane" > gpurun_out/b12_tests.log 2>&1 || { tail -30 gpurun_out/b12_tests.log; exit 1; }
tail -1 gpurun_out/b12_tests.log
BENCH_ARGS="--size 1200 --height 900" TUNES="rt1:--tune jfa_rt=1|rt2:--tune jfa_rt=2|rt4:--tune jfa_rt=4" ROUNDS=3 bash scripts/ab_tunes.sh > gpurun_out/ab_jfa_rt.txt 2>&1 || { cat gpurun_out/ab_jfa_rt.txt; exit 1; }
cat gpurun_out/ab_jfa_rt.txt
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b12 -o run -- \
  python bench.py --no-cpu-baseline --steps 10 --warmup 3 --size 1200 --height 900 --tune jfa_rt=2 > gpurun_out/prof_b12.log 2>&1 || exit 1
grep jfa_step gpurun_out/prof_b12/run_kernel_stats.csv | awk -F'",' '{print $2 "  " substr($1,1,60)}'
echo done
