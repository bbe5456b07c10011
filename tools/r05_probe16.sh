#!/bin/bash
# Timing probe: the trunk's growth-chunk MFMAs as two v_mfma_f32_16x16x32_bf16
# each (same FLOPs and operands, outputs wrong; lib/libisr_probe16.so) vs production, whole trunk
# launch, alternating processes.
set -o pipefail
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2 3; do
  timeout -k 10 120 python -u tools/ab_chain.py --configs 1:1:0:0 --rounds 3 >> gpurun_out/r05/probe16_base.txt 2>&1 || exit 1
  ISR_LIB=$PWD/image_super_resolution_amd/lib/libisr_probe16.so timeout -k 10 120 python -u tools/ab_chain.py --configs 1:1:0:0 --rounds 3 >> gpurun_out/r05/probe16_new.txt 2>&1 || exit 1
done
