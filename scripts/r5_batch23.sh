#!/bin/bash
# Round-5 batch 23: k_blur_rows with 16-row tiles (4 rows per thread: 22 KB of LDS, 7 workgroups per CU) against
# 32-row tiles (39 KB, 4 per CU): parity under the A/B build, rocprof time, frame A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
RC2DGI_LIB=$PWD/build/ab/librc2dgi_blur4.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_shard.py -k "blur_path or headline_4096 or linux_merge or shard" > gpurun_out/b23_tests.log 2>&1 || { tail -30 gpurun_out/b23_tests.log; exit 1; }
tail -1 gpurun_out/b23_tests.log
for lib in cur b4; do
  L=$PWD/radiancecascade2dglobalillumination_amd/librc2dgi.so; [ $lib = b4 ] && L=$PWD/build/ab/librc2dgi_blur4.so
  RC2DGI_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b23_$lib -o run -- \
    python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/prof_b23_$lib.log 2>&1 || exit 1
  echo "== $lib"; grep -E "blur" gpurun_out/prof_b23_$lib/run_kernel_stats.csv | awk -F'",' '{print $2 "  " substr($1,1,40)}'
done
LIBS="radiancecascade2dglobalillumination_amd/librc2dgi.so build/ab/librc2dgi_blur4.so" ROUNDS=4 bash scripts/ab_lib.sh > gpurun_out/ab_blur4.txt 2>&1 || exit 1
cat gpurun_out/ab_blur4.txt
echo done
