#!/bin/bash
# Round-5 batch 20: device memory per shard context (8 in-process row strips at C3) against one unsharded context
# (--shards 1: a strips context of the whole frame).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for sh in 1 8; do
  timeout -k 10 300 python bench.py --size 8192 --cascades 8 --ray-range 64 --mode strips --shards $sh --steps 3 --warmup 1 \
    --no-cpu-baseline > gpurun_out/strips_mem$sh.log 2>&1 || { tail -5 gpurun_out/strips_mem$sh.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/strips_mem$sh.log').read().strip().splitlines()[-1]); print($sh, d['ms_per_step'], d['device_bytes_per_shard'] / 2**30, 'GiB per shard')"
done
echo done
