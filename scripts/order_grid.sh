#!/bin/bash
# Workgroup-order grid for some levels of one configuration: every code of scripts/order_codes_patches.txt (200
# patch / oriented-patch codes: px 1-8, py 2-32, dg 4-64) and/or order_codes_bands.txt (168 band codes: px 1-4,
# py 1-16, dg 1-64) against the committed schedule's order, with the committed variant (scripts/sched_probe.py:
# interleaved rounds in one process).  Prints, per level, the committed order's time and the best codes.
#   LEVELS="3 4 5"  CODES=patches|bands|both (default both)  BENCH_ARGS="--size 8192 --cascades 8 ..."  TAG=name
# e.g.  LEVELS="2 3 4 5" BENCH_ARGS="--cascades 8 --ray-range 64" TAG=c2 gpurun -- bash scripts/order_grid.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
case "${CODES:-both}" in
  patches) O=$(cat scripts/order_codes_patches.txt) ;;
  bands) O=$(cat scripts/order_codes_bands.txt) ;;
  *) O="$(cat scripts/order_codes_patches.txt),$(cat scripts/order_codes_bands.txt)" ;;
esac
cands=""
for L in ${LEVELS:-3 4 5}; do cands="$cands $L:c:c,$O"; done
out=gpurun_out/order_grid_${TAG:-run}.jsonl
timeout -k 10 ${LIMIT:-500} python scripts/sched_probe.py --rounds ${ROUNDS:-2} --frames ${FRAMES:-3} $BENCH_ARGS $cands \
  > $out 2>&1 || { tail -20 $out; exit 1; }
python3 - "$out" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith('{'):
        d = json.loads(line); c = d['committed']; r = d['ms_variant_order']
        rk = [x for x in r if x[1] == c[0] and x[2] == c[1]]
        print('L%d' % d['level'], 'committed', c, rk[0][0] if rk else None, 'best', r[:4])
PY
