#!/bin/bash
# round 4, probe 5: parity of palettes / early upper samples / committed schedules, A/B of the early upper
# samples, C1 with the miss proofs forced on
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 600 \
  --timeout-method thread -m gpu -k "side_tables or surface_palettes or every_rc_variant or miss_proofs or committed_bench or storage_schedule or c1_app" \
  > gpurun_out/r04/t5.log 2>&1 || { tail -30 gpurun_out/r04/t5.log; exit 1; }
tail -2 gpurun_out/r04/t5.log
LIBS="build/ab/librc2dgi_nowin.so build/ab/librc2dgi_noearly.so build/ab/librc2dgi_fv0.so build/ab/librc2dgi_erec.so radiancecascade2dglobalillumination_amd/librc2dgi.so" ROUNDS=3 bash scripts/ab_lib.sh || exit 1
BENCH_ARGS="--size 1200 --height 900" CFGS="base rc_skip=2 rc_skip=3" ROUNDS=2 bash scripts/ab_knobs.sh || exit 1
