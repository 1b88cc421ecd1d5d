#!/usr/bin/env python3
"""Write the best refined order per level of a scripts/retune_orders.sh result into a committed tuning file
(variants kept; a level keeps its committed order unless the refined best beats it by more than MARGIN ms).
Usage: apply_retune.py retune_<tag>.jsonl tuning/<file>.json [margin_ms] [note]"""
import json
import sys

res, path = sys.argv[1], sys.argv[2]
margin = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0005
t = json.load(open(path))
for line in open(res):
    d = json.loads(line)
    lv, (cv, co) = d["level"], d["committed"]
    assert t["rc_variant"][lv] == cv and t["rc_order"][lv] == co, (lv, d["committed"])
    rows = d["ms_variant_order"]
    com = [ms for ms, v, o in rows if v == cv and o == co]
    best = rows[0]
    if best[1] == cv and (not com or best[0] < com[0] - margin):
        print(f"L{lv}: {co} ({com[0] if com else '?'} ms) -> {best[2]} ({best[0]} ms)")
        t["rc_order"][lv] = best[2]
if len(sys.argv) > 4:
    t["note"] = sys.argv[4]
json.dump(t, open(path, "w"))
open(path, "a").write("\n")
