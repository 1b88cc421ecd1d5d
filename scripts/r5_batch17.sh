#!/bin/bash
# Round-5 batch 17: k_shade_cells with 1024 lanes (record groups of 4 rows) against 512: parity under the A/B
# build, kernel time, bench A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
RC2DGI_LIB=$PWD/build/ab/librc2dgi_cells1024.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "side_tables or surface_palettes or shade_split" > gpurun_out/b17_tests.log 2>&1 || { tail -30 gpurun_out/b17_tests.log; exit 1; }
tail -1 gpurun_out/b17_tests.log
for lib in cur w1024; do
  L=$PWD/radiancecascade2dglobalillumination_amd/librc2dgi.so; [ $lib = w1024 ] && L=$PWD/build/ab/librc2dgi_cells1024.so
  RC2DGI_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b17_$lib -o run -- \
    python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/prof_b17_$lib.log 2>&1 || exit 1
  echo "== $lib"; grep -E "shade" gpurun_out/prof_b17_$lib/run_kernel_stats.csv | awk -F'",' '{print $2 "  " substr($1,1,40)}'
done
LIBS="radiancecascade2dglobalillumination_amd/librc2dgi.so build/ab/librc2dgi_cells1024.so" ROUNDS=4 bash scripts/ab_lib.sh > gpurun_out/ab_cells1024.txt 2>&1 || exit 1
cat gpurun_out/ab_cells1024.txt
echo done
