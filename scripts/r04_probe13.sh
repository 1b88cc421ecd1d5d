#!/bin/bash
# round 4, probe 13: C2 orders from probe 12 in a whole-bench A/B; a grid of band orders (mode 2: px 1-4,
# py 1-16, dg 1-64) for the headline's L2-L5 and C2's L3-L5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04; export TMPDIR=/tmp
BENCH_ARGS="--cascades 8 --ray-range 64" CFGS="base rc_order_L3=17047560,rc_order_L4=262664,rc_order_L5=4202504 rc_order_L4=262664" ROUNDS=3 bash scripts/ab_knobs.sh || exit 1
O=$(cat scripts/r04_orders_bands.txt)
probe() {  # tag, sched_probe args...
  local t=$1; shift
  timeout -k 10 400 python scripts/sched_probe.py --rounds 2 --frames 4 "$@" > gpurun_out/r04/orders_$t.jsonl 2>&1 || { tail -20 gpurun_out/r04/orders_$t.jsonl; return 1; }
  python3 -c "
import json
for l in open('gpurun_out/r04/orders_$t.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); c=d['committed']; r=d['ms_variant_order']
        rk=[x for x in r if x[1]==c[0] and x[2]==c[1]]
        print('$t L%d' % d['level'], 'committed', c, rk[0][0] if rk else None, 'best', r[:4])"
}
probe hb 2:c:c,$O 3:c:c,$O 4:c:c,$O 5:c:c,$O || exit 1
probe c2b --cascades 8 --ray-range 64 3:c:c,$O 4:c:c,$O 5:c:c,$O || exit 1
