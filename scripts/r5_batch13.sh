#!/bin/bash
# Round-5 batch 13: k_shade_cmin under a register cap (occupancy: 114 VGPRs = 4 waves per SIMD, 2 workgroups of
# 512 lanes per CU, 8 rounds over the 4096 cells): rocprof kernel time and whole-bench A/B of the capped builds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for lib in cur w6 w8; do
  L=$PWD/radiancecascade2dglobalillumination_amd/librc2dgi.so; [ $lib != cur ] && L=$PWD/build/ab/librc2dgi_shade$lib.so
  RC2DGI_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b13_$lib -o run -- \
    python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/prof_b13_$lib.log 2>&1 || exit 1
  f=$(find gpurun_out/prof_b13_$lib -name '*kernel_stats.csv' | head -1)
  echo "== $lib"; grep -E "shade_cmin" "$f" | awk -F'",' '{print $2}' | cut -c1-60
done
LIBS="radiancecascade2dglobalillumination_amd/librc2dgi.so build/ab/librc2dgi_shadew6.so build/ab/librc2dgi_shadew8.so" ROUNDS=3 bash scripts/ab_lib.sh > gpurun_out/ab_shade_wpe.txt 2>&1 || exit 1
cat gpurun_out/ab_shade_wpe.txt
echo done
