#!/bin/bash
# Deep-ring trunk (variant 4) ablations + event counters (tuning build, timing only).
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
TL=$PWD/image_super_resolution_amd/lib/libisr_tuning.so
echo "== ablate variant 4"
ISR_CHAIN_VARIANT=4 ISR_LIB=$TL timeout -k 10 240 python -u tools/ab_trunk.py --rounds 3 --reps 5 \
    --configs ${1:-0:0,1:0,8:0,9:0,4:0,16:0,29:0} > $O/ablate_v4.jsonl 2> $O/ablate_v4.err
rc=$?
echo "rc=$rc"
cat $O/ablate_v4.jsonl
tail -3 $O/ablate_v4.err
exit $rc
