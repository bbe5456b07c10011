#!/bin/bash
# 32x32-tile trunk form (isr_conv_chain_variant 3): bitwise chain tests, then same-box A/B.
set -u
export TMPDIR=/tmp
O=$PWD/gpurun_out/r03
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -3 $O/$name.out; return $rc; }
step 300 t32_tests python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 150 --timeout-method thread &&
step 200 t32_ab python -u tools/ab_chain.py --configs 1:1:0:0,1:1:0:3 --rounds 7
