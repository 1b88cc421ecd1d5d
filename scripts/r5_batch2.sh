#!/bin/bash
# Round-5 batch 2 (one gpurun call): the 16-byte-lane k_shade_cmin and the bit-transposed k_dir_clear (GPU tests,
# library A/B, rocprofv3 kernel stats), the retuned C1 / f16 / rgba8 schedules (their full-size tests and bench
# lines), the JumpFlood pass with the 4- and 5-step coset kernels, and per-XCD spans of the headline levels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/cfg; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "side_tables or surface_palettes or shade_cmin or miss_proofs or exit_proofs" > gpurun_out/b2_tests.log 2>&1 || { tail -20 gpurun_out/b2_tests.log; exit 1; }
tail -1 gpurun_out/b2_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py \
  -k "c1_app or storage_schedule or committed_headline or committed_bench" > gpurun_out/b2_cfgtests.log 2>&1 || { tail -20 gpurun_out/b2_cfgtests.log; exit 1; }
tail -1 gpurun_out/b2_cfgtests.log
ROUNDS=3 bash scripts/ab_lib.sh > gpurun_out/ab_side.txt 2>&1 || exit 1
cat gpurun_out/ab_side.txt
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b2 -o run -- python bench.py --no-cpu-baseline --steps 10 --warmup 3 \
  > gpurun_out/prof_b2.log 2>&1 || exit 1
for n in f16 rgba8 c1; do
  case $n in f16) a="--storage f16";; rgba8) a="--storage rgba8";; c1) a="--size 1200 --height 900";; esac
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps 10 $a > gpurun_out/cfg/$n.log 2>&1 || exit 1
  tail -1 gpurun_out/cfg/$n.log > gpurun_out/cfg/$n.json
  python3 -c "import json; d=json.load(open('gpurun_out/cfg/$n.json')); print('$n', d['value'], d['rc_ms_per_frame'], d['rc_level_ms'], d.get('full_pipeline_ms'))"
done
timeout -k 10 200 python scripts/jfa_pass.py jfa_coset 1 2 > gpurun_out/jfa_coset_pass.txt 2>&1 || exit 1
cat gpurun_out/jfa_coset_pass.txt
timeout -k 10 120 python scripts/rc_timing.py > gpurun_out/timing_xcd3.json 2> gpurun_out/timing_xcd3.err || exit 1
grep -i xcd gpurun_out/timing_xcd3.err | head -20
echo done
