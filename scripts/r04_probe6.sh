#!/bin/bash
# round 4, probe 6: re-tune with palettes / early upper samples / far vote on: a fresh autotune of the
# headline, tail thresholds at L3-L5, palettes at C2 / C3, C1 autotuned with the miss proofs on
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --autotune --no-cpu-baseline --steps 20 \
  --save-tuning gpurun_out/r04/4096x4096_N6_rr2_f32.json > gpurun_out/r04/tune_h.log 2>&1 || { tail -20 gpurun_out/r04/tune_h.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r04/tune_h.log').read().strip().splitlines()[-1]); print('autotuned', d['rc_ms_per_frame'], d['rc_level_ms'], d['config']['rc_variant'], d['config']['rc_order'])"
CFGS="base rc_tail=6 rc_tail=8 rc_tail=12 rc_tail=16 rc_noproof_L1=1 rc_noproof_L2=1 rc_noproof_L1=1,rc_noproof_L2=1" ROUNDS=2 bash scripts/ab_knobs.sh || exit 1
BENCH_ARGS="--cascades 8 --ray-range 64" CFGS="base rc_pal=0" ROUNDS=2 bash scripts/ab_knobs.sh || exit 1
BENCH_ARGS="--size 8192 --cascades 8 --ray-range 64 --steps 5" CFGS="base rc_pal=0" ROUNDS=1 bash scripts/ab_knobs.sh || exit 1
timeout -k 10 300 python bench.py --size 1200 --height 900 --autotune --no-cpu-baseline --steps 20 \
  --save-tuning gpurun_out/r04/1200x900_N6_rr2_f32.json > gpurun_out/r04/tune_c1.log 2>&1 || { tail -20 gpurun_out/r04/tune_c1.log; exit 1; }
tail -1 gpurun_out/r04/tune_c1.log | cut -c1-700
