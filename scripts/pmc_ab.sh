#!/bin/bash
# PMC passes of the bench at two tuning settings (A/B): gpurun_out/pmc_<tag>/ + summaries.
# Usage: TAGS="skip0:--tune rc_skip=0|skip1:--tune rc_skip=1" bash scripts/pmc_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
IFS='|' read -r -a SETS <<< "${TAGS:-skip0:--tune rc_skip=0|skip1:--tune rc_skip=1}"
for s in "${SETS[@]}"; do
  tag=${s%%:*}; args=${s#*:}
  rm -rf gpurun_out/pmc
  GROUPS_OVERRIDE="${GROUPS_AB:-TCC_HIT_sum TCC_MISS_sum;SQ_WAVES SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS;TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum}" \
    STEPS=3 BENCH_ARGS="$args" bash scripts/profile_pmc.sh > gpurun_out/pmc_$tag.log 2>&1 || exit $?
  python3 scripts/pmc_summary.py gpurun_out/pmc --all > gpurun_out/pmc_summary_$tag.txt 2>&1
  mv gpurun_out/pmc gpurun_out/pmc_$tag
  echo "== $tag"; cut -c1-220 gpurun_out/pmc_summary_$tag.txt | head -40
done
