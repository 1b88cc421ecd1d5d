#!/bin/bash
# Round-5 batch 15 (as 14, plus k_dir_clear on the side stream): the split records / palette pass (k_shade_scan + k_shade_cells, tuning shade_split): parity
# (side tables, palettes, every level at 4096^2, two frames for the list parity), kernel times, bench A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "side_tables or surface_palettes or shade_cmin or shade_split or headline_4096" > gpurun_out/b15_tests.log 2>&1 || { tail -30 gpurun_out/b15_tests.log; exit 1; }
tail -1 gpurun_out/b15_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py \
  -k "committed_bench or committed_headline" > gpurun_out/b15_cfgtests.log 2>&1 || { tail -20 gpurun_out/b15_cfgtests.log; exit 1; }
tail -1 gpurun_out/b15_cfgtests.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b15 -o run -- \
  python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/prof_b15.log 2>&1 || exit 1
grep -E "shade" gpurun_out/prof_b15/run_kernel_stats.csv | awk -F'",' '{print $2 "  " substr($1,1,50)}'
TUNES="side:--tune side_overlap=1|split:--tune side_overlap=0|fused:--tune shade_split=0" ROUNDS=4 bash scripts/ab_tunes.sh > gpurun_out/ab_shade_side.txt 2>&1 || { cat gpurun_out/ab_shade_side.txt; exit 1; }
cat gpurun_out/ab_shade_side.txt
echo done
