#!/bin/bash
# Round 6: dynamic instruction mix of the fp16 trunk kernel (per dispatch, summed over waves):
# VALU / SALU / SMEM / LDS instructions per MFMA -- the VALU share is one of the give-back levers.
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r06
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES \
  --output-format csv -d gpurun_out/r06/pmc_mix24 -o mix -- python3 tools/time_forward.py --rounds 1 --steps 3 > gpurun_out/r06/t24.txt 2>&1
echo "rc=$?"
