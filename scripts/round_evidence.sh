#!/bin/bash
# Round-end evidence on one box, in one call: the GPU suite, the headline bench with its rocprofv3 kernel stats
# and PMC traffic per scene (scripts/round_profile.sh), one line per BASELINE config and storage mode, the C3 strips,
# the C4 batch lines and the scene sweep (scripts/scene_sweep.sh).  Results under gpurun_out/ (copied into
# profiles/r<NN>/final by hand; gpurun_out/rc_level_pmc.json to profiles/).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  echo "== GPU tests"
  timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 600 --timeout-method thread > gpurun_out/gputests.log 2>&1
  rc=$?; tail -3 gpurun_out/gputests.log; [ $rc -eq 0 ] || exit $rc
fi
bash scripts/round_profile.sh || exit $?
echo "== configs"
bash scripts/configs_bench.sh || exit $?
echo "== C3 strips (8 in-process shards)"
timeout -k 10 400 python bench.py --size 8192 --cascades 8 --ray-range 64 --mode strips --shards 8 --steps 5 --warmup 2 \
  > gpurun_out/cfg/c3_strips8.log 2>&1 || exit $?
tail -1 gpurun_out/cfg/c3_strips8.log | cut -c1-300
echo "== C4 batch (8 scenes, N=8)"
for bs in 1 0; do
  timeout -k 10 400 python bench.py --batch 8 --batch-streams $bs --cascades 8 --steps 5 --warmup 2 \
    > gpurun_out/cfg/c4_streams$bs.log 2>&1 || exit $?
  tail -1 gpurun_out/cfg/c4_streams$bs.log | cut -c1-300
done
echo "== scenes"
bash scripts/scene_sweep.sh || exit $?
