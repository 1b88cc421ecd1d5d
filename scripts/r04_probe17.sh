#!/bin/bash
# round 4, probe 17: k_shade_cmin<PAL> in 512-lane workgroups (8 rows per wave: one records round trip per
# wave instead of two) -- parity, A/B against the previous build, rocprofv3 of the kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "palettes or side_tables" > gpurun_out/r04/pal_tests.log 2>&1 || { tail -30 gpurun_out/r04/pal_tests.log; exit 1; }
tail -2 gpurun_out/r04/pal_tests.log
LIBS="build/ab/librc2dgi_base.so radiancecascade2dglobalillumination_amd/librc2dgi.so" ROUNDS=3 bash scripts/ab_lib.sh || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04/palprof -o run -- python3 bench.py --no-cpu-baseline --steps 10 > gpurun_out/r04/palprof.log 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/r04/palprof/run_kernel_stats.csv')):
    if 'shade_cmin' in r['Name']: print(r['Name'][:45], r['Calls'], r['AverageNs'])"
