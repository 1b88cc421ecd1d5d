#!/bin/bash
# C3 (8192^2, N=8, rayRange 64) on one MI355X: the tuned unsharded frame (its schedule saved), then
# the same frame as 2 / 4 / 8 in-process row-strip shards (rc2dgi_do_group, JumpFlood exchange).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/c3; export TMPDIR=/tmp
timeout -k 10 400 python bench.py --no-cpu-baseline --size 8192 --cascades 8 --ray-range 64 --steps 10 --warmup 2 \
  --autotune --save-tuning gpurun_out/c3/8192x8192_N8_rr64_f32.json > gpurun_out/c3/unsharded.log 2>&1 || exit $?
tail -1 gpurun_out/c3/unsharded.log | cut -c1-300
cp gpurun_out/c3/8192x8192_N8_rr64_f32.json radiancecascade2dglobalillumination_amd/tuning/
for P in 2 4 8; do
  timeout -k 10 300 python bench.py --mode strips --shards $P --size 8192 --cascades 8 --ray-range 64 --steps 10 \
    --warmup 2 > gpurun_out/c3/strips$P.log 2>&1 || exit $?
  tail -1 gpurun_out/c3/strips$P.log | cut -c1-300
done
