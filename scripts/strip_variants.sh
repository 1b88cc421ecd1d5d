#!/bin/bash
# C3 as 8 in-process row strips with per-level tile-variant overrides (TUNES="label:--tune k=v ...|...")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp; mkdir -p gpurun_out/sv
IFS='|' read -ra CASES <<< "$TUNES"
for c in "${CASES[@]}"; do
  lab=${c%%:*}; args=${c#*:}
  timeout -k 10 200 python bench.py --mode strips --shards ${SHARDS:-8} --size 8192 --cascades 8 --ray-range 64 \
    --steps 10 --warmup 2 $args > gpurun_out/sv/$lab.log 2>&1 || exit $?
  echo "$lab $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sv/$lab.log)"
done
