#!/bin/bash
# round 4, probe 19: the low-level tile shapes (16x8x2, 32x8x1, 32x8x2) for RGBA16F / RGBA8 cascades: per-level
# probes at L0-L2 of the f16 / rgba8 headline schedules (committed order, then every autotune order for 32x8x2)
# (their parity: tests/test_gpu_parity.py -k every_rc_variant, 9 passed on MI355X)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04; export TMPDIR=/tmp
for st in f16 rgba8; do
  timeout -k 10 400 python scripts/sched_probe.py --storage $st --rounds 2 --frames 4 0:c,1,3,6:c 1:c,1,3,6:c \
    2:c,1,3,6:c 0:6:all 1:6:all 2:6:all > gpurun_out/r04/lowtiles_$st.jsonl 2>&1 || { tail -20 gpurun_out/r04/lowtiles_$st.jsonl; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/r04/lowtiles_$st.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); c=d['committed']; r=d['ms_variant_order']
        rk=[x for x in r if x[1]==c[0] and x[2]==c[1]]
        print('$st L%d' % d['level'], 'committed', c, rk[0][0] if rk else None, 'best', r[:3])"
done
