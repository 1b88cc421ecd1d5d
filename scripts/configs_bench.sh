#!/bin/bash
# One bench line per storage mode and BASELINE config (same box), for DESIGN's tables:
# f16 and rgba8 at 4096^2 N=6, C1 1200x900 N=6, C2 4096^2 N=8 rr64, C3 8192^2 N=8 rr64.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/cfg; export TMPDIR=/tmp
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps 10 "$@" > gpurun_out/cfg/$n.log 2>&1 || return $?
  tail -1 gpurun_out/cfg/$n.log > gpurun_out/cfg/$n.json
  python3 -c "import json; d=json.load(open('gpurun_out/cfg/$n.json')); print('$n', d['value'], d['rc_ms_per_frame'], d.get('full_pipeline_ms'))"
}
run f16 --storage f16 && run rgba8 --storage rgba8 && run c1 --size 1200 --height 900 && \
  run c2 --cascades 8 --ray-range 64 && run c3 --size 8192 --cascades 8 --ray-range 64
