#!/bin/bash
# A/B of the timing events' flags (RC2DGI_TIMING_EVENT_FLAGS: 0 default, 0x20000000 no system-scope
# fence, 0x40000000 device-scope release) and of the side kernels on a second stream (side_conc),
# interleaved ROUNDS times on one box; then a kernel trace of the last setting (gaps between kernels).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for i in $(seq ${ROUNDS:-2}); do
  for cfg in ${CFGS:-0:0 0x20000000:0 0x40000000:0 0:1 0x20000000:1}; do
    fl=${cfg%%:*}; sc=${cfg##*:}
    RC2DGI_TIMING_EVENT_FLAGS=$fl timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 --tune side_conc=$sc $BENCH_ARGS > gpurun_out/ab.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['rc_ms_per_frame'], d['rc_level_ms'], d['full_pipeline_ms'], d['ms_per_step'])"
  done
done
if [ -n "${TRACE:-}" ]; then
  fl=${TRACE%%:*}; sc=${TRACE##*:}
  RC2DGI_TIMING_EVENT_FLAGS=$fl timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/evprof -o run \
    -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --tune side_conc=$sc > gpurun_out/evprof.log 2>&1 || exit $?
  python3 scripts/frame_gaps.py gpurun_out/evprof/run_kernel_trace.csv
fi
