#!/bin/bash
# round 4, probe 1: parity of the 512/1024-lane one-probe tiles, then per-level schedule probes
# (product build, and the march-capped-at-0 timing build for the non-march cost)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu \
  -k "every_rc_variant" > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -2 gpurun_out/t1.log
V="c,0,13,20,21,22,23,24"
timeout -k 10 400 python -u scripts/sched_probe.py --rounds 3 --frames 6 3:$V:all 4:$V:all 5:$V:all \
  > gpurun_out/p1.json 2> gpurun_out/p1.err || { tail -20 gpurun_out/p1.err; exit 1; }
RC2DGI_LIB=$PWD/build/diag/librc2dgi_diag0.so timeout -k 10 300 python -u scripts/sched_probe.py --rounds 3 --frames 6 \
  0:c:c 1:c:c 2:c:c 3:$V:c 4:$V:c 5:$V:c > gpurun_out/p1_diag0.json 2> gpurun_out/p1_diag0.err || { tail -20 gpurun_out/p1_diag0.err; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/p1.json", "gpurun_out/p1_diag0.json"):
    for l in open(f):
        d = json.loads(l)
        print(f, d["level"], d["committed"], d["ms_variant_order"][:8])
PY
