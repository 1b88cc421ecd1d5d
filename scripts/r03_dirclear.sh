#!/bin/bash
# k_dir_clear with per-cell ballots: the proof tests and the committed schedules at full size, then the bench
# and the kernel's duration (rocprofv3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest -q -x tests/test_gpu_parity.py tests/test_gpu_configs.py -k "miss_proofs or exit_proofs or degenerate or committed_bench" --timeout 300 --timeout-method thread > gpurun_out/dc_test.log 2>&1
rc=$?; tail -3 gpurun_out/dc_test.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 > gpurun_out/dcb.log 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/dcb.log').read().strip().splitlines()[-1]); print(d['value'], d['rc_ms_per_frame'], d['rc_level_ms'], d['full_pipeline_ms'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dcprof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/dcprof.log 2>&1 || exit $?
grep -i "dir_clear\|shade_cmin" gpurun_out/dcprof/run_kernel_stats.csv | cut -c1-200
