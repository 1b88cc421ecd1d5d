#!/bin/bash
# Round-5 batch 4: the cascade chain (rc_chain) parity and timing at C1 / the headline; k_shade_cmin v3 (512 lanes,
# one 8-texel run per lane, LDS transpose on the hit path) against the base library; refactor A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/cfg; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "cascade_chain or side_tables or surface_palettes or shade_cmin" > gpurun_out/b4_tests.log 2>&1 || { tail -30 gpurun_out/b4_tests.log; exit 1; }
tail -1 gpurun_out/b4_tests.log
for lib in base new; do
  L=$PWD/radiancecascade2dglobalillumination_amd/librc2dgi.so; [ $lib = base ] && L=$PWD/build/ab/librc2dgi_base.so
  RC2DGI_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b4_$lib -o run -- \
    python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/prof_b4_$lib.log 2>&1 || exit 1
  f=$(find gpurun_out/prof_b4_$lib -name '*kernel_stats.csv' | head -1)
  echo "== $lib"; grep -E "shade_cmin|dir_clear" "$f" | awk -F'",' '{print $2}' | cut -c1-60
done
ROUNDS=3 bash scripts/ab_lib.sh > gpurun_out/ab_b4.txt 2>&1 || exit 1
cat gpurun_out/ab_b4.txt
BENCH_ARGS="--size 1200 --height 900" TUNES="c0:--tune rc_chain=0|c1:--tune rc_chain=1|c2:--tune rc_chain=2" ROUNDS=3 bash scripts/ab_tunes.sh > gpurun_out/ab_chain_c1.txt 2>&1 || exit 1
cat gpurun_out/ab_chain_c1.txt
TUNES="c0:--tune rc_chain=0|c1:--tune rc_chain=1" ROUNDS=2 bash scripts/ab_tunes.sh > gpurun_out/ab_chain_h.txt 2>&1 || exit 1
cat gpurun_out/ab_chain_h.txt
echo done
