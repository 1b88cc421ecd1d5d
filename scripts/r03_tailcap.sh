#!/bin/bash
# What the long march chains cost: timing-only builds with the march capped at 10 / 16 samples per ray
# (WRONG results by design; _build.py diag N) against the product build, committed schedule, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
for v in full:radiancecascade2dglobalillumination_amd/librc2dgi.so cap10:build/diag/librc2dgi_diag10.so cap16:build/diag/librc2dgi_diag16.so; do
  name=${v%%:*}; lib=${v#*:}
  RC2DGI_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/tc_$name.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/tc_$name.log').read().strip().splitlines()[-1]); print('$name', d['rc_ms_per_frame'], d['rc_level_ms'])"
done; done
