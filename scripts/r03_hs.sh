#!/bin/bash
# hit-time shading (row-strip shards' default) + the 8-strip schedule: tests, then C3 strips A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp; mkdir -p gpurun_out
echo "== test"
timeout -k 10 700 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_configs.py -k "hit_time or shard or c3 or group or phase" > gpurun_out/hs_test.log 2>&1
rc=$?; tail -2 gpurun_out/hs_test.log; [ $rc -eq 0 ] || exit $rc
echo "== strips"
TUNES="new:|noh:--tune rc_hitshade=0|l5v3:--tune rc_variant_L5=3|new2:|noh2:--tune rc_hitshade=0|l5v3b:--tune rc_variant_L5=3" bash scripts/strip_variants.sh
echo "== headline unchanged"
ROUNDS=3 bash scripts/ab_lib.sh
