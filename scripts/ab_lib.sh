#!/bin/bash
# A/B of library builds in one run (same box): bench lines alternating between the current
# librc2dgi.so and build/ab/librc2dgi_base.so (a build of another commit), ROUNDS times.
# LIBS: other builds to cycle through instead (paths, e.g. from `_build.py exp NAME -D...`).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for i in $(seq ${ROUNDS:-2}); do
  for lib in ${LIBS:-build/ab/librc2dgi_base.so radiancecascade2dglobalillumination_amd/librc2dgi.so}; do
    RC2DGI_LIB=$PWD/$lib timeout -k 10 ${AB_LIMIT:-120} python bench.py --no-cpu-baseline --steps 20 $BENCH_ARGS > gpurun_out/ab.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$(basename $lib)', d['value'], d.get('rc_ms_per_frame'), d.get('rc_level_ms'), d.get('full_pipeline_ms'), 'jfa', d.get('pass_ms', {}).get('jfa'), 'step', d['ms_per_step'], 'mem', d.get('device_bytes_per_shard'))"
  done
done
