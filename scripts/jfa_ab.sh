#!/bin/bash
# JumpFlood kernel A/B at 4096^2 and 8192^2: rocprofv3 kernel stats per tuning (TUNES="label:--tune k=v ...|...")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
IFS='|' read -ra CASES <<< "$TUNES"
for c in "${CASES[@]}"; do
  lab=${c%%:*}; args=${c#*:}
  STEPS=10 TAG=jfa_$lab BENCH_ARGS="$args" bash scripts/prof_stats.sh > /dev/null || exit $?
  echo "== $lab: $(grep -o '"full_pipeline_ms": [0-9.]*' gpurun_out/prof_jfa_$lab.log)"
  python3 scripts/frame_kernel_sums.py 12 10 gpurun_out/prof_jfa_$lab/run_kernel_trace.csv | grep -i -E "jfa|occup"
done
