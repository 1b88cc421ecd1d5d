#!/bin/bash
# Round-5 batch 16: the 8-strip C3 rehearsal, current library against the base build (an earlier round-5 commit);
# run again after the side stream became lazy.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2 3; do
  for lib in base cur; do
    L=$PWD/radiancecascade2dglobalillumination_amd/librc2dgi.so; [ $lib = base ] && L=$PWD/build/ab/librc2dgi_base.so
    RC2DGI_LIB=$L timeout -k 10 300 python bench.py --size 8192 --cascades 8 --ray-range 64 --mode strips --shards 8 --steps 5 \
      --warmup 2 --no-cpu-baseline > gpurun_out/strips_$lib.log 2>&1 || { tail -5 gpurun_out/strips_$lib.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/strips_$lib.log').read().strip().splitlines()[-1]); print('$lib'.ljust(6), d['value'], d['ms_per_step'])"
  done
done
echo done
