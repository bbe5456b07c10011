#!/bin/bash
# Training trunk fix check + plain SRGAN step; then the interleaved-refill build (lib/libisr_il.so)
# through the bitwise chain tests and the same-process chain A/B.  Stops at the first failure.
set -u
export TMPDIR=/tmp
O=gpurun_out/r03
mkdir -p $O
IL=$PWD/image_super_resolution_amd/lib/libisr_il.so
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -3 $O/$name.out; return $rc; }
step 300 train_tests python -u -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread &&
step 300 train_plain python -u tools/bench_train.py --steps 5 --warmup 2 &&
step 200 il_chain_tests env ISR_LIB=$IL python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 150 --timeout-method thread &&
step 200 il_ab_chain env ISR_LIB=$IL python -u tools/ab_chain.py --configs 1:1:0:0,1:1:0:2 --rounds 5
