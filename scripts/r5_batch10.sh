#!/bin/bash
# Round-5 batch 10: the 8-strip C3 rehearsal under XCD-interleaved orders for the strips entry (the committed
# round-3 orders, the whole frame's round-5 orders, the round-3 orders with lc 2 / 4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/tuning_exp; export TMPDIR=/tmp
python3 - <<'PY'
import json
t = json.load(open('radiancecascade2dglobalillumination_amd/tuning/8192x8192_N8_rr64_f32.json'))
s = t["strips"]["8"]
for name, orders in (("wholeorders", list(t["rc_order"])),
                     ("lc2", [(o & ((1 << 26) - 1)) | (2 << 26) for o in s["rc_order"]]),
                     ("lc4", [(o & ((1 << 26) - 1)) | (4 << 26) for o in s["rc_order"]])):
    v = json.loads(json.dumps(t))
    v["strips"]["8"]["rc_order"] = orders
    json.dump(v, open(f"gpurun_out/tuning_exp/c3_strips_{name}.json", "w"))
PY
for r in 1 2; do
  for t in committed wholeorders lc2 lc4; do
    f=""; [ $t != committed ] && f="--load-tuning gpurun_out/tuning_exp/c3_strips_$t.json"
    timeout -k 10 300 python bench.py --size 8192 --cascades 8 --ray-range 64 --mode strips --shards 8 --steps 5 --warmup 2 \
      --no-cpu-baseline $f > gpurun_out/strips_$t.log 2>&1 || { tail -5 gpurun_out/strips_$t.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/strips_$t.log').read().strip().splitlines()[-1]); print('$t'.ljust(12), d['value'], d['ms_per_step'])"
  done
done
echo done
