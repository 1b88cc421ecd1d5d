#!/bin/bash
# round 4, probe 2: phase-plane march samples (parity, then per-level A/B), and the hit-record-load ablation
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu \
  -k "phase_plane or every_rc_variant" > gpurun_out/t2.log 2>&1 || { tail -30 gpurun_out/t2.log; exit 1; }
tail -2 gpurun_out/t2.log
# phase modes per level: each level's time with rc_phase 0 / 1 / 2 (variant and order committed)
for ph in 0 1 2; do
  timeout -k 10 200 python -u scripts/sched_probe.py --rounds 3 --frames 8 --tune rc_phase=$ph 3:c:c 4:c:c 5:c:c \
    > gpurun_out/p2_ph$ph.json 2> gpurun_out/p2_ph$ph.err || { tail -20 gpurun_out/p2_ph$ph.err; exit 1; }
done
RC2DGI_LIB=$PWD/build/ab/librc2dgi_nohit.so timeout -k 10 200 python -u scripts/sched_probe.py --rounds 3 --frames 8 \
  0:c:c 1:c:c 2:c:c 3:c:c 4:c:c 5:c:c > gpurun_out/p2_nohit.json 2> gpurun_out/p2_nohit.err || { tail -20 gpurun_out/p2_nohit.err; exit 1; }
timeout -k 10 200 python -u scripts/sched_probe.py --rounds 3 --frames 8 \
  0:c:c 1:c:c 2:c:c 3:c:c 4:c:c 5:c:c > gpurun_out/p2_base.json 2> gpurun_out/p2_base.err || exit 1
for f in gpurun_out/p2_ph0.json gpurun_out/p2_ph1.json gpurun_out/p2_ph2.json gpurun_out/p2_base.json gpurun_out/p2_nohit.json; do
  python3 -c "import json,sys; print(sys.argv[1], [(json.loads(l)['level'], json.loads(l)['ms_variant_order'][0][0]) for l in open(sys.argv[1])])" $f
done
