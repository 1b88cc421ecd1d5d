#!/bin/bash
# Round-5 batch 5: the cascade chain as k_rc_level<..., CH> (parity, C1 timing), the library A/B against the base
# build (the bit-transposed k_dir_clear; the other kernels' code is unchanged), rocprofv3 kernel times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/cfg; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "cascade_chain or side_tables or surface_palettes or shade_cmin or miss_proofs" > gpurun_out/b5_tests.log 2>&1 || { tail -30 gpurun_out/b5_tests.log; exit 1; }
tail -1 gpurun_out/b5_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py \
  -k "c1_app or committed_bench" > gpurun_out/b5_cfgtests.log 2>&1 || { tail -20 gpurun_out/b5_cfgtests.log; exit 1; }
tail -1 gpurun_out/b5_cfgtests.log
ROUNDS=3 bash scripts/ab_lib.sh > gpurun_out/ab_b5.txt 2>&1 || exit 1
cat gpurun_out/ab_b5.txt
BENCH_ARGS="--size 1200 --height 900" TUNES="c0:--tune rc_chain=0|c1:--tune rc_chain=1|c2:--tune rc_chain=2" ROUNDS=3 bash scripts/ab_tunes.sh > gpurun_out/ab_chain_c1b.txt 2>&1 || exit 1
cat gpurun_out/ab_chain_c1b.txt
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b5 -o run -- \
  python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/prof_b5.log 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b5_c1chain -o run -- \
  python bench.py --no-cpu-baseline --steps 10 --warmup 3 --size 1200 --height 900 --tune rc_chain=1 > gpurun_out/prof_b5_c1chain.log 2>&1 || exit 1
echo done
