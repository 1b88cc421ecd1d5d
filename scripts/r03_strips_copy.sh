#!/bin/bash
# C3 in-process row strips: the exchange copies by k_copy16 vs the runtime's copy (RC2DGI_COPY_RUNTIME=1),
# and the ordering events' flags (0 / device-scope release), interleaved; per-kernel stats of one setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/c3; export TMPDIR=/tmp
run() {
  RC2DGI_COPY_RUNTIME=$1 RC2DGI_ORDER_EVENT_FLAGS=$2 timeout -k 10 300 python bench.py --mode strips --shards 8 --size 8192 \
    --cascades 8 --ray-range 64 --steps 10 --warmup 2 > gpurun_out/c3/s8.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/c3/s8.log').read().strip().splitlines()[-1]); print('copy_runtime=$1 flags=$2', d['ms_per_step'])"
}
for i in 1 2 3; do run 1 0; run 0 0; run 1 0x40000000; run 0 0x40000000; done
for cr in 1 0; do
  RC2DGI_COPY_RUNTIME=$cr timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3/prof$cr -o run -- python3 bench.py --mode strips --shards 8 --size 8192 \
      --cascades 8 --ray-range 64 --steps 5 --warmup 1 > gpurun_out/c3/prof$cr.log 2>&1 || exit $?
done
