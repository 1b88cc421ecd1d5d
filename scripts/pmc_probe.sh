#!/bin/bash
# Bottleneck probe for k_rc_level on the bench workload: autotuned schedule, then one rocprofv3
# --pmc pass per counter group (scripts/profile_pmc.sh), summarised per RC level.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --save-tuning gpurun_out/tuning.json \
  > gpurun_out/tune.log 2>&1 || exit $?
tail -1 gpurun_out/tune.log | cut -c1-600
GROUPS_OVERRIDE=${PROBE_GROUPS:-"SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_VMEM_RD;TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum;TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum;TCC_HIT_sum TCC_MISS_sum"} \
  STEPS=3 BENCH_ARGS="--load-tuning gpurun_out/tuning.json" bash scripts/profile_pmc.sh || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc --all > gpurun_out/pmc_probe.txt
cat gpurun_out/pmc_probe.txt | cut -c1-400
