#!/bin/bash
# A/B of tuning knobs on one box: bench lines alternating between the knob sets in TUNES
# ("label:--tune k=v --tune k2=v2|label2:..."), ROUNDS times; prints value, RC ms and per-level ms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
IFS='|' read -r -a SETS <<< "${TUNES:-base:}"
for i in $(seq ${ROUNDS:-2}); do
  for s in "${SETS[@]}"; do
    tag=${s%%:*}; args=${s#*:}
    timeout -k 10 120 python bench.py --no-cpu-baseline --steps ${STEPS:-20} $BENCH_ARGS $args > gpurun_out/ab_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/ab_$tag.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_$tag.log').read().strip().splitlines()[-1]); print('$tag'.ljust(14), d['value'], d['rc_ms_per_frame'], d['rc_level_ms'], d['full_pipeline_ms'])"
  done
done
