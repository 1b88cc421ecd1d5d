#!/bin/bash
# round 4, probe 14: order grids (patch + band codes) for C3 (8192^2 N8 rr64) L3-L6 and C1 (1200x900) L2-L5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04; export TMPDIR=/tmp
O="$(cat scripts/r04_orders.txt),$(cat scripts/r04_orders_bands.txt)"
probe() {  # tag, sched_probe args...
  local t=$1; shift
  timeout -k 10 500 python scripts/sched_probe.py --rounds 2 --frames 3 "$@" > gpurun_out/r04/orders_$t.jsonl 2>&1 || { tail -20 gpurun_out/r04/orders_$t.jsonl; return 1; }
  python3 -c "
import json
for l in open('gpurun_out/r04/orders_$t.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); c=d['committed']; r=d['ms_variant_order']
        rk=[x for x in r if x[1]==c[0] and x[2]==c[1]]
        print('$t L%d' % d['level'], 'committed', c, rk[0][0] if rk else None, 'best', r[:4])"
}
probe c1 --size 1200 --height 900 2:c:c,$O 3:c:c,$O 4:c:c,$O 5:c:c,$O || exit 1
probe c3a --size 8192 --cascades 8 --ray-range 64 4:c:c,$O || exit 1
probe c3b --size 8192 --cascades 8 --ray-range 64 3:c:c,$O 5:c:c,$O || exit 1
