#!/bin/bash
# Grouped weight gradients: do co-resident blocks run in phase? Half the blocks start ~half a stage
# late (tuning build, ISR_WGRAD_ABLATE 4 / 8) vs all together (0); row-sweep form (cfg 0).
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
mkdir -p $O
TL=$PWD/image_super_resolution_amd/lib/libisr_tuning.so
K=$O/wgrs7_kernel.jsonl
for r in 1 2; do
  for a in 0 4 8; do
    ISR_LIB=$TL ISR_WGRAD_ABLATE=$a timeout -k 10 120 python -u tools/ab_wgrad_group.py >> $K 2>> $O/wgrs7_err.txt || exit 1
    echo "{\"ablate\": $a}" >> $K
  done
done
