#!/bin/bash
# k_jfa_p2w: parity (wide vs per-texel taps), JFA pass A/B at 4096^2, kernel trace of the JFA steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -m pytest -q -x tests/test_gpu_parity.py -k "jfa_wide" --timeout 300 --timeout-method thread > gpurun_out/wide_test.log 2>&1
rc=$?; tail -3 gpurun_out/wide_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/jfa_pass.py jfa_wide 0 1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wideprof -o run -- python3 scripts/jfa_pass.py jfa_wide 1 --rounds 1 --frames 5 > gpurun_out/wideprof.log 2>&1 || exit $?
python3 scripts/frame_gaps.py gpurun_out/wideprof/run_kernel_trace.csv | grep jfa
