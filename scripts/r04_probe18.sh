#!/bin/bash
# round 4, probe 18: order grids (patch + band codes) for the f16 and rgba8 headline schedules, L2-L5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04; export TMPDIR=/tmp
O="$(cat scripts/r04_orders.txt),$(cat scripts/r04_orders_bands.txt)"
for st in f16 rgba8; do
  timeout -k 10 500 python scripts/sched_probe.py --storage $st --rounds 2 --frames 3 2:c:c,$O 3:c:c,$O 4:c:c,$O 5:c:c,$O > gpurun_out/r04/orders_$st.jsonl 2>&1 || { tail -20 gpurun_out/r04/orders_$st.jsonl; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/r04/orders_$st.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); c=d['committed']; r=d['ms_variant_order']
        rk=[x for x in r if x[1]==c[0] and x[2]==c[1]]
        print('$st L%d' % d['level'], 'committed', c, rk[0][0] if rk else None, 'best', r[:3])"
done
