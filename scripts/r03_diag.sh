#!/bin/bash
# Round-3 diagnostics of the committed bench schedule: wave-lifetime sections (timing build), march
# statistics (stats build), and stall PMC passes of the product build -> gpurun_out/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== timing"; bash scripts/rc_timing.sh || exit $?
echo "== stats"
timeout -k 10 120 python scripts/march_stats.py > gpurun_out/march_stats.json 2> gpurun_out/march_stats.err || { tail -5 gpurun_out/march_stats.err; exit 1; }
cat gpurun_out/march_stats.json | cut -c1-600
echo "== pmc"
GROUPS_OVERRIDE="${PMC_GROUPS:-SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS;SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM;TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum}" \
  STEPS=3 bash scripts/profile_pmc.sh || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc --all > gpurun_out/pmc_stalls.txt && grep "k_rc_level\|k_jfa" gpurun_out/pmc_stalls.txt | cut -c1-200
