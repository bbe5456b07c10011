#!/bin/bash
# Same-box A/B of trunk builds (production, interleave step 0, interleave step 2) and of the
# training trunk (per-conv vs trunk kernel).  Stops at the first failure.
set -u
export TMPDIR=/tmp
O=gpurun_out/r03
mkdir -p $O
L=$PWD/image_super_resolution_amd/lib
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -3 $O/$name.out; return $rc; }
step 200 il2_chain_tests env ISR_LIB=$L/libisr_il2.so python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 150 --timeout-method thread &&
for r in 1 2; do
  step 120 ab_prod_$r python -u tools/ab_chain.py --configs 1:1:0:0 --rounds 5 &&
  step 120 ab_il_$r env ISR_LIB=$L/libisr_il.so python -u tools/ab_chain.py --configs 1:1:0:0 --rounds 5 &&
  step 120 ab_il2_$r env ISR_LIB=$L/libisr_il2.so python -u tools/ab_chain.py --configs 1:1:0:0 --rounds 5 || exit 1
done &&
step 300 train_chain1 python -u tools/bench_train.py --steps 5 --warmup 2 &&
step 300 train_chain0 env ISR_TRAIN_CHAIN=0 python -u tools/bench_train.py --steps 5 --warmup 2
