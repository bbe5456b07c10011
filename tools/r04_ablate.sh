#!/bin/bash
# Trunk-kernel ablation matrix (tuning build, timing only): which part of the per-chunk cost
# bounds the pair form.  Bits: 1 no halo DMA, 4 no stores, 8 no weight DMA, 16 no dependency waits.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
TL=$PWD/image_super_resolution_amd/lib/libisr_tuning.so
echo "== ablate"
ISR_LIB=$TL timeout -k 10 300 python -u tools/ab_trunk.py --rounds 3 --reps 5 \
    --configs ${1:-0:0,1:0,8:0,9:0,4:0,16:0,13:0,29:0,0:1,9:1} > $O/ablate.jsonl 2> $O/ablate.err
rc=$?
echo "rc=$rc"
cat $O/ablate.jsonl
tail -5 $O/ablate.err
exit $rc
