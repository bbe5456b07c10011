#!/bin/bash
# Round 6: the trunk's A/B forms again under sustained load (20 graph replays per round, 9 rounds,
# interleaved): the production form (0) vs the XCD-aware deal (6), non-temporal halo loads (7) /
# output stores (8), four waves per SIMD (5) and the 8-wave form (2) -- memory-path energy is
# what sets the held clock.  Tuning library, bf16 storage.
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r06
ISR_LIB=$PWD/image_super_resolution_amd/lib/libisr_tuning.so timeout -k 10 600 python -u tools/ab_chain.py \
  --configs 1:1:0:0,1:1:0:6,1:1:0:7,1:1:0:8,1:1:0:5,1:1:0:2 --rounds 9 --steps 20 > gpurun_out/r06/t21_ab_chain.txt 2>&1
echo "rc=$?"
