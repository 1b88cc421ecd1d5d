#!/bin/bash
# round 4, probe 9: two-probe 512-lane tiles (variants 25 "32x16x2", 26 "64x8x2") at L0-L2 -- parity, then
# per-level schedule probes against the committed 32x8x2 (variant 6) at the headline, C2 and C1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "every_rc_variant and f32" > gpurun_out/r04/v25_tests.log 2>&1 || { tail -30 gpurun_out/r04/v25_tests.log; exit 1; }
tail -2 gpurun_out/r04/v25_tests.log
timeout -k 10 300 python scripts/sched_probe.py --rounds 3 0:6,25,26:c 1:6,25,26:c 2:6,25,26:c \
  > gpurun_out/r04/v25_h.jsonl 2>&1 || { tail -20 gpurun_out/r04/v25_h.jsonl; exit 1; }
cut -c1-400 gpurun_out/r04/v25_h.jsonl
timeout -k 10 300 python scripts/sched_probe.py --rounds 2 0:25,26:all 1:25,26:all 2:25,26:all \
  > gpurun_out/r04/v25_h_orders.jsonl 2>&1 || { tail -20 gpurun_out/r04/v25_h_orders.jsonl; exit 1; }
python3 - <<'PY'
import json
for line in open('gpurun_out/r04/v25_h_orders.jsonl'):
    if line.startswith('{'):
        d = json.loads(line); print(d['level'], d['committed'], d['ms_variant_order'][:4])
PY
