#!/bin/bash
# C3 as 8 in-process strips: per-level variant overrides for the shard contexts
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp; mkdir -p gpurun_out
TUNES="base:|l4v13:--tune rc_variant_L4=13|l4v0:--tune rc_variant_L4=0|l34v3:--tune rc_variant_L3=3 --tune rc_variant_L4=3|l4v3:--tune rc_variant_L4=3|l3v3:--tune rc_variant_L3=3|base2:" bash scripts/strip_variants.sh
