#!/bin/bash
# Trunk-kernel ablation matrix (tuning build, timing only): which part of the per-chunk cost
# bounds the pair form (variant 0) and the 32x32-tile form (variant 3).
# Bits: 1 no halo DMA, 4 no stores, 8 no weight DMA, 16 no dependency waits.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
TL=$PWD/image_super_resolution_amd/lib/libisr_tuning.so
CFG=${1:-0:0,1:0,8:0,9:0,4:0,16:0,13:0,29:0,0:1,9:1}
rc=0
for V in 0 3; do
    echo "== ablate variant $V"
    ISR_CHAIN_VARIANT=$V ISR_LIB=$TL timeout -k 10 240 python -u tools/ab_trunk.py --rounds 3 --reps 5 \
        --configs $CFG > $O/ablate_v$V.jsonl 2> $O/ablate_v$V.err
    rc=$?
    echo "rc=$rc"
    cat $O/ablate_v$V.jsonl
    tail -3 $O/ablate_v$V.err
    [ $rc -ne 0 ] && break
done
exit $rc
