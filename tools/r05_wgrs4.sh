#!/bin/bash
# Row-sweep refinements (tuning build, ISR_WGRAD_GROUP_CFG): 0 = RS, 13 = + DMA one piece per row,
# 14 = 2 rows read ahead, 15 = both; 12 = round-4 form. Timed twice, bitwise vs 12, ablations of 15.
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
mkdir -p $O
TL=$PWD/image_super_resolution_amd/lib/libisr_tuning.so
K=$O/wgrs4_kernel.jsonl
run() { timeout -k 10 120 python -u tools/ab_wgrad_group.py "$@" >> $K 2>> $O/wgrs4_err.txt; }
for r in 1 2; do
  for v in 12 0 13 14 15; do ISR_LIB=$TL ISR_WGRAD_GROUP_CFG=$v run --dump /tmp/wg_$v.pt || exit 1; done
done
for v in 0 13 14 15; do python -u tools/ab_wgrad_group.py --compare /tmp/wg_12.pt /tmp/wg_$v.pt >> $K || exit 1; done
for a in 1 2 3; do ISR_LIB=$TL ISR_WGRAD_GROUP_CFG=15 ISR_WGRAD_ABLATE=$a run || exit 1; echo "{\"ablate\": $a, \"cfg\": 15}" >> $K; done
for sp in 19 20; do ISR_LIB=$TL ISR_WGRAD_GROUP_CFG=15 ISR_WGRAD_GROUP_SPLITS=$sp run || exit 1; echo "{\"splits\": $sp, \"cfg\": 15}" >> $K; done
