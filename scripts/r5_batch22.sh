#!/bin/bash
# Round-5 batch 22: six repeats of the default bench line on one box (the spread of the headline number).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/bench_repeats.jsonl
for r in 1 2 3 4 5 6; do
  timeout -k 10 300 python bench.py $( [ $r -gt 1 ] && echo --no-cpu-baseline ) > gpurun_out/bench_rep.log 2>&1 || { tail -5 gpurun_out/bench_rep.log; exit 1; }
  tail -1 gpurun_out/bench_rep.log >> gpurun_out/bench_repeats.jsonl
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_rep.log').read().strip().splitlines()[-1]); print($r, d['value'], d['rc_ms_per_frame'], d['full_pipeline_ms'], d['roofline']['frac'])"
done
echo done
