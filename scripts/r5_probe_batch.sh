#!/bin/bash
# Round-5 probe batch (one gpurun call): library A/B of the palette dedup change, the 5-step coset knob, the GPU
# tests those touch, per-XCD timing, march stats per scene, an autotune on a random scene, then the headline's
# L3 variants and tail thresholds under the interleaved orders.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
LIBS="build/ab/librc2dgi_base.so radiancecascade2dglobalillumination_amd/librc2dgi.so" ROUNDS=3 bash scripts/ab_lib.sh > gpurun_out/ab_shadepal.txt 2>&1 || exit 1
TUNES="c1:--tune jfa_coset=1|c2:--tune jfa_coset=2" ROUNDS=3 bash scripts/ab_tunes.sh > gpurun_out/ab_coset.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "side_tables or surface_palettes or shade_cmin or jfa_coset" > gpurun_out/shadepal_tests.log 2>&1 || exit 1
timeout -k 10 120 python scripts/rc_timing.py > gpurun_out/timing_xcd2.json 2> gpurun_out/timing_xcd2.err || exit 1
: > gpurun_out/stats_scenes.jsonl
for sc in demo random:1 random:0 dense:0; do
  timeout -k 10 120 python scripts/march_stats.py 4096 6 2 1 $sc >> gpurun_out/stats_scenes.jsonl || exit 1
done
timeout -k 10 300 python bench.py --no-cpu-baseline --autotune --scene random:1 --save-tuning gpurun_out/tune_random1.json \
  > gpurun_out/bench_auto_r1.json 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --scene random:1 > gpurun_out/bench_committed_r1.json 2>&1 || exit 1
timeout -k 10 400 python scripts/sched_probe.py --rounds 3 --frames 5 --xcd-chunks 0,2,3,4,6,8 3:0,6,13,20,23:c,37748994,17039617 \
  > gpurun_out/probe_l3var.jsonl 2> gpurun_out/probe_l3var.err || exit 1
TUNES="base:|t8:--tune rc_tail_L3=8 --tune rc_tail_L4=8 --tune rc_tail_L5=8|t12:--tune rc_tail_L3=12 --tune rc_tail_L4=12 --tune rc_tail_L5=12|l5t0:--tune rc_tail_L5=0" \
  ROUNDS=3 bash scripts/ab_tunes.sh > gpurun_out/ab_tail2.txt 2>&1 || exit 1
echo done
