#!/bin/bash
# round 4, probe 10: a wider grid of workgroup orders (px 1-8, py 2-32, dg 4-64, plain and oriented patches:
# 200 codes) for L2-L5 of the headline, committed variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04; export TMPDIR=/tmp
O=$(cat scripts/r04_orders.txt)
for L in 4 3 5 2; do
  timeout -k 10 400 python scripts/sched_probe.py --rounds 2 --frames 4 $L:c:c,$O > gpurun_out/r04/orders_L$L.jsonl 2>&1 || { tail -20 gpurun_out/r04/orders_L$L.jsonl; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/r04/orders_L$L.jsonl'):
    if l.startswith('{'):
        d = json.loads(l); print('L%d' % d['level'], 'committed', d['committed'], 'best', d['ms_variant_order'][:5])"
done
