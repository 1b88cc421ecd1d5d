#!/bin/bash
# round 4, probe 4: surface palettes (parity, then A/B on the committed schedule), then probe 3's work
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu \
  -k "surface_palettes or phase_plane" > gpurun_out/r04/t4.log 2>&1 || { tail -30 gpurun_out/r04/t4.log; exit 1; }
tail -2 gpurun_out/r04/t4.log
CFGS="base rc_pal=1" ROUNDS=3 bash scripts/ab_knobs.sh || exit 1
bash scripts/r04_probe3.sh
