#!/bin/bash
# k_jfa_pair: parity (pairs vs per-step kernels), JFA pass A/B at 4096^2 (and 8192^2 with BIG=1), kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -m pytest -q -x tests/test_gpu_parity.py -k "jfa_pair or jfa_coset" --timeout 300 --timeout-method thread > gpurun_out/pair_test.log 2>&1
rc=$?; tail -3 gpurun_out/pair_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/jfa_pass.py jfa_pair 0 1 || exit $?
if [ -n "$BIG" ]; then timeout -k 10 300 python scripts/jfa_pass.py jfa_pair 0 1 --size 8192 --cascades 8 --rounds 2 --frames 8 || exit $?; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pairprof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/pairprof.log 2>&1 || exit $?
python3 scripts/frame_gaps.py gpurun_out/pairprof/run_kernel_trace.csv | grep jfa
