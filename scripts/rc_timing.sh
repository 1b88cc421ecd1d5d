#!/bin/bash
# k_rc_level wave-lifetime sections (diagnostic build build/diag/librc2dgi_timing.so) for the knob sets
# in TUNES ("label:--tune k=v ...|..."); one JSON line each under gpurun_out/timing_<label>.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
IFS='|' read -r -a SETS <<< "${TUNES:-base:}"
for s in "${SETS[@]}"; do
  tag=${s%%:*}; args=${s#*:}
  echo "== $tag"
  timeout -k 10 120 python scripts/rc_timing.py $args > gpurun_out/timing_$tag.json 2> gpurun_out/timing_$tag.err || { tail -5 gpurun_out/timing_$tag.err; exit 1; }
  grep "^L" gpurun_out/timing_$tag.err
done
