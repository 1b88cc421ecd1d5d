#!/bin/bash
# XCD-interleave retune of the committed schedules of the other configurations (scripts/retune_orders.sh per
# configuration; results in gpurun_out/retune_<tag>.jsonl).  CONFIGS selects a subset.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for cfg in ${CONFIGS:-c1 f16 rgba8 c2 c3}; do
  case $cfg in
    c1) BA="--size 1200 --height 900 --cascades 6"; LV="0 1 2 3 4 5" ;;
    f16) BA="--storage f16"; LV="0 1 2 3 4 5" ;;
    rgba8) BA="--storage rgba8"; LV="0 1 2 3 4 5" ;;
    c2) BA="--cascades 8 --ray-range 64"; LV="0 1 2 3 4 5 6 7" ;;
    c3) BA="--size 8192 --cascades 8 --ray-range 64"; LV="0 1 2 3 4 5 6 7" ;;
  esac
  echo "== $cfg"
  TAG=$cfg BENCH_ARGS="$BA" LEVELS="$LV" LIMIT=${LIMIT:-500} bash scripts/retune_orders.sh || exit 1
done
