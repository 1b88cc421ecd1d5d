#!/bin/bash
# march statistics + stall PMC of the product build + tail-threshold A/B (round 3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== stats"
timeout -k 10 120 python scripts/march_stats.py > gpurun_out/march_stats.json 2> gpurun_out/march_stats.err || { tail -5 gpurun_out/march_stats.err; exit 1; }
cut -c1-900 gpurun_out/march_stats.json
echo "== pmc"
GROUPS_OVERRIDE="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS;SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM;TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum;TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
  STEPS=3 bash scripts/profile_pmc.sh > gpurun_out/pmc.log 2>&1 || { tail -5 gpurun_out/pmc.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc --all > gpurun_out/pmc_stalls.txt || exit 1
grep "k_rc_level\|k_jfa" gpurun_out/pmc_stalls.txt | cut -c1-160
