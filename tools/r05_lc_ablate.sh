#!/bin/bash
# Loader / consumer trunk form: where the time goes (tuning build ablations, timing only).
set -o pipefail
mkdir -p gpurun_out/r05
export ISR_LIB=$PWD/image_super_resolution_amd/lib/libisr_tuning.so
ISR_CHAIN_VARIANT=9 timeout -k 10 300 python -u tools/ab_trunk.py --configs 0:0,1:0,8:0,9:0,2:0,6:0,16:0,25:0,31:0 \
    --rounds 3 > gpurun_out/r05/lc_ablate.jsonl 2>&1 &&
ISR_CHAIN_VARIANT=0 timeout -k 10 300 python -u tools/ab_trunk.py --configs 0:0,9:0,16:0 --rounds 3 \
    > gpurun_out/r05/pair_ablate.jsonl 2>&1
