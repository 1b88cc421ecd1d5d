#!/bin/bash
# A/B of tuning-knob settings on the committed schedule, interleaved ROUNDS times on one box
# (each line: setting, value, RC ms, per-level ms, full frame ms).  CFGS: settings, commas between
# the KEY=VALUE pairs of one setting, "base" for none.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for i in $(seq ${ROUNDS:-3}); do
  for cfg in ${CFGS:-base rc_skip=3}; do
    args=""; [ "$cfg" = base ] || for kv in ${cfg//,/ }; do args="$args --tune $kv"; done
    timeout -k 10 ${AB_LIMIT:-120} python bench.py --no-cpu-baseline --steps 20 $BENCH_ARGS $args > gpurun_out/ab.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$cfg', d['value'], d.get('rc_ms_per_frame'), d.get('rc_level_ms'), d.get('full_pipeline_ms'), 'jfa', d.get('pass_ms', {}).get('jfa'), 'step', d['ms_per_step'], 'mem', d.get('device_bytes_per_shard'))"
  done
done
