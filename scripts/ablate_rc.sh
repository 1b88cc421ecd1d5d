#!/bin/bash
# RC time split by ablation (timing-only diagnostic builds, WRONG results by design):
#   full           librc2dgi.so
#   nomerge        no level-(L+1) staging and merge       (librc2dgi_nomerge.so: _build.py nomerge)
#   nomarch        march capped at 0 iterations           (librc2dgi_diag0.so:   _build.py diag 0)
# each on the bench workload with the committed schedule (TUNING, default radiancecascade2dglobalillumination_amd/tuning/4096x4096_N6_rr2_f32.json).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for v in full:radiancecascade2dglobalillumination_amd/librc2dgi.so nomerge:build/diag/librc2dgi_nomerge.so \
         nomarch:build/diag/librc2dgi_diag0.so; do
  name=${v%%:*}; lib=${v#*:}
  RC2DGI_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 \
    --load-tuning ${TUNING:-radiancecascade2dglobalillumination_amd/tuning/4096x4096_N6_rr2_f32.json} > gpurun_out/ablate_$name.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ablate_$name.log').read().strip().splitlines()[-1]); print('$name', d['rc_level_ms'], d['rc_ms_per_frame'])"
done
