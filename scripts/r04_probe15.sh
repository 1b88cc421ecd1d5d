#!/bin/bash
# round 4, probe 15: whole-bench A/B of the probe-14 orders at C1 and C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04; export TMPDIR=/tmp
BENCH_ARGS="--size 1200 --height 900" CFGS="base rc_order_L2=17041416,rc_order_L3=17302020,rc_order_L4=18876424" ROUNDS=3 bash scripts/ab_knobs.sh || exit 1
BENCH_ARGS="--size 8192 --cascades 8 --ray-range 64 --steps 5" CFGS="base rc_order_L3=33687556,rc_order_L4=525320,rc_order_L5=17827848" ROUNDS=2 bash scripts/ab_knobs.sh || exit 1
