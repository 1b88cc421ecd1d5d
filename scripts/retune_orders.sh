#!/bin/bash
# Per-level workgroup orders x XCD interleave (order code bits 26-30) for one configuration's committed
# schedule (variants kept): rc2dgi_autotune's order candidates x lc in LCS, one round, then the best REFINE per
# level re-timed over ROUNDS rounds.  BENCH_ARGS selects the configuration (sched_probe.py options),
# LEVELS the levels; prints the refined JSON lines to gpurun_out/retune_<TAG>.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${TAG:-run}
cands=""
for L in $LEVELS; do cands="$cands $L:c:all"; done
timeout -k 10 ${LIMIT:-600} python scripts/sched_probe.py --rounds 1 --frames ${FRAMES:-3} --xcd-chunks ${LCS:-0,2,3,4,5,6,7,8,9} \
  $BENCH_ARGS $cands > gpurun_out/retune_${tag}_grid.jsonl 2> gpurun_out/retune_${tag}.err || { tail -5 gpurun_out/retune_${tag}.err; exit 1; }
ref=$(python3 - gpurun_out/retune_${tag}_grid.jsonl ${REFINE:-8} <<'PY'
import json, sys
parts = []
for l in open(sys.argv[1]):
    d = json.loads(l)
    codes = [x[2] for x in d["ms_variant_order"][:int(sys.argv[2])]]
    parts.append(f"{d['level']}:c:c," + ",".join(str(c) for c in codes))
print(" ".join(parts))
PY
)
timeout -k 10 ${LIMIT:-600} python scripts/sched_probe.py --rounds ${ROUNDS:-4} --frames 5 $BENCH_ARGS $ref \
  > gpurun_out/retune_${tag}.jsonl 2>> gpurun_out/retune_${tag}.err || { tail -5 gpurun_out/retune_${tag}.err; exit 1; }
python3 - gpurun_out/retune_${tag}.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    r = d["ms_variant_order"]
    com = [x[0] for x in r if x[2] == d["committed"][1] and x[1] == d["committed"][0]]
    print(d["level"], "committed", d["committed"], com, "best", r[0])
PY
