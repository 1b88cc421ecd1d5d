#!/bin/bash
# GPU-box check: parity tests, then a bench line, then a rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; stop at the first crash / abort / timeout
# (pytest's exit 1 = failed assertions is not a GPU fault and lets the bench run).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
rocm-smi --showproductname > gpurun_out/gpu_info.txt 2>&1
lscpu > gpurun_out/cpu_info.txt 2>&1
echo "== pytest -m gpu"
timeout -k 10 ${PYTEST_LIMIT:-900} python -m pytest tests -q -m gpu ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
ok $rc || exit $rc
echo "== bench"
timeout -k 10 ${BENCH_LIMIT:-400} python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; tail -3 gpurun_out/bench.log; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
if [ -n "${PROFILE:-1}" ] && [ "${PROFILE:-1}" != "0" ]; then
  echo "== rocprofv3 kernel trace"
  timeout -k 10 ${PROF_LIMIT:-400} rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
    -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1
  rc=$?; tail -3 gpurun_out/prof.log; echo "rocprof rc=$rc"
  find gpurun_out/prof -name "*stats*" | head
fi
