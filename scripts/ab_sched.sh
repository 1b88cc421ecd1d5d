#!/bin/bash
# Autotune a schedule for the bench config, then A/B it against the committed one (same box),
# ROUNDS times: the committed file in radiancecascade2dglobalillumination_amd/tuning/ vs gpurun_out/tuning_new.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --autotune --no-cpu-baseline --steps 5 --save-tuning gpurun_out/tuning_new.json \
  > gpurun_out/tune_new.log 2>&1 || exit $?
cat gpurun_out/tuning_new.json; echo
for i in $(seq ${ROUNDS:-3}); do
  for s in "" "--load-tuning gpurun_out/tuning_new.json"; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 $s > gpurun_out/ab.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('${s:-committed}'[-20:], d['value'], d['rc_ms_per_frame'], d['rc_level_ms'])"
  done
done
