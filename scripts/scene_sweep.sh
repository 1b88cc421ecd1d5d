#!/bin/bash
# Headline bench (4096^2, N=6, rayRange 2, committed schedule) on the demo frame and on scenes the schedule
# was not tuned on: random:0..3 (5 % occluders) and dense:0..1 (>= 25 %).  One JSON line per scene in
# gpurun_out/scenes.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/scenes.jsonl
for sc in ${SCENES:-demo random:0 random:1 random:2 random:3 dense:0 dense:1}; do
  timeout -k 10 150 python bench.py --no-cpu-baseline --steps ${STEPS:-20} --scene $sc $BENCH_ARGS > gpurun_out/scene.log 2>&1 || { echo "bench $sc failed"; tail -5 gpurun_out/scene.log; exit 1; }
  tail -1 gpurun_out/scene.log >> gpurun_out/scenes.jsonl
  python3 -c "import json; d=json.loads(open('gpurun_out/scene.log').read().strip().splitlines()[-1]); print('$sc'.ljust(10), d['config']['occluder_coverage'], d['value'], d['rc_ms_per_frame'], d['rc_level_ms'], d['full_pipeline_ms'])"
done
