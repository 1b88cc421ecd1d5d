#!/bin/bash
# round 3: parity suite, A/B vs base, the march-free ablation (upper bound of a distance-field tile's saving at
# L0-L2), and the per-level cost of 8 row strips at C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp; mkdir -p gpurun_out
echo "== test"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/mix_test.log 2>&1
rc=$?; tail -2 gpurun_out/mix_test.log; [ $rc -eq 0 ] || exit $rc
echo "== A/B"
ROUNDS=2 bash scripts/ab_lib.sh || exit $?
echo "== march capped at 0 samples (WRONG results by design)"
for i in 1 2; do
  RC2DGI_LIB=$PWD/build/diag/librc2dgi_diag0.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/diag0.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/diag0.log').read().strip().splitlines()[-1]); print('diag0', d['rc_ms_per_frame'], d['rc_level_ms'])"
done
echo "== strip levels"
timeout -k 10 300 python scripts/strip_levels.py 8192 8 64 8 > gpurun_out/strip_levels.json 2> gpurun_out/strip_levels.err || { tail -5 gpurun_out/strip_levels.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/strip_levels.json')); print(d['whole_level_ms']); print(d['strip_sum_level_ms']); print(d['ratio'])"
