#!/bin/bash
# Round 6: how much of the Scaler convs' time is their weight refills?  Tuning-library probes 10 / 11
# (V_W0 and the 32x32 8-wave form without weight refills after chunk 0: outputs wrong, timing only)
# against the production variant 0 and variant 9, inside the production forward (bf16).
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r06
export ISR_LIB=$PWD/image_super_resolution_amd/lib/libisr_tuning.so
timeout -k 10 300 python -u tools/ab_scaler.py --variants 0,10,9,11 --rounds 9 --steps 5 > gpurun_out/r06/t17_ab_scaler_wres.txt 2>&1
echo "rc=$?"
