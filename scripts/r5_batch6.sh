#!/bin/bash
# Round-5 batch 6: the cascade chain at C1 under workgroup orders that keep the levels' dependency order
# (tile-major 0, and interleaved tile-major lc << 26), against the level-by-level launches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
o0="--tune rc_order_L0=0 --tune rc_order_L1=0 --tune rc_order_L2=0 --tune rc_order_L3=0 --tune rc_order_L4=0"
o3="--tune rc_order_L0=201326592 --tune rc_order_L1=201326592 --tune rc_order_L2=201326592 --tune rc_order_L3=201326592 --tune rc_order_L4=201326592"
o1="--tune rc_order_L0=67108864 --tune rc_order_L1=67108864 --tune rc_order_L2=67108864 --tune rc_order_L3=67108864 --tune rc_order_L4=67108864"
BENCH_ARGS="--size 1200 --height 900" TUNES="sep:|ch:--tune rc_chain=1|ch_o0:--tune rc_chain=1 $o0|ch_o3:--tune rc_chain=1 $o3|ch_o1:--tune rc_chain=1 $o1|sep_o0:$o0" ROUNDS=3 bash scripts/ab_tunes.sh > gpurun_out/ab_chain_orders.txt 2>&1 || { cat gpurun_out/ab_chain_orders.txt; exit 1; }
cat gpurun_out/ab_chain_orders.txt
echo done
