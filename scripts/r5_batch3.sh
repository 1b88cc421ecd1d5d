#!/bin/bash
# Round-5 batch 3: the row-wise hit path of k_shade_cmin (GPU tests, rocprofv3 kernel times against the base
# library), then the XCD-interleave retune of the C2 and C3 schedules.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "side_tables or surface_palettes or shade_cmin or miss_proofs or exit_proofs" > gpurun_out/b3_tests.log 2>&1 || { tail -20 gpurun_out/b3_tests.log; exit 1; }
tail -1 gpurun_out/b3_tests.log
for lib in base new; do
  L=$PWD/radiancecascade2dglobalillumination_amd/librc2dgi.so; [ $lib = base ] && L=$PWD/build/ab/librc2dgi_base.so
  RC2DGI_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b3_$lib -o run -- \
    python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/prof_b3_$lib.log 2>&1 || exit 1
  f=$(find gpurun_out/prof_b3_$lib -name '*kernel_stats.csv' | head -1)
  echo "== $lib"; grep -E "shade_cmin|dir_clear" "$f" | awk -F'",' '{print $2}' | cut -c1-60
done
CONFIGS="c2 c3" LIMIT=400 bash scripts/retune_all.sh > gpurun_out/retune_b.log 2>&1 || { tail -20 gpurun_out/retune_b.log; exit 1; }
tail -20 gpurun_out/retune_b.log
timeout -k 10 120 python scripts/rc_timing.py --size 1200 --height 900 > gpurun_out/timing_c1.json 2> gpurun_out/timing_c1.err || exit 1
grep "per XCD" gpurun_out/timing_c1.err
timeout -k 10 120 python scripts/rc_timing.py > gpurun_out/timing_h.json 2> gpurun_out/timing_h.err || exit 1
grep "per XCD" gpurun_out/timing_h.err
