#!/bin/bash
# Same-box A/B: production trunk vs refill-before-step-0-reads (lib/libisr_rf.so).
set -u
export TMPDIR=/tmp
O=$PWD/gpurun_out/r03
mkdir -p $O
RF=$PWD/image_super_resolution_amd/lib/libisr_rf.so
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -1 $O/$name.out; return $rc; }
step 200 rf_tests env ISR_LIB=$RF python -u -m pytest tests/test_gpu_chain.py -x -q -k "bitwise" --timeout 150 --timeout-method thread || exit 1
for r in 1 2 3; do
  step 120 abr_prod_$r python -u tools/ab_chain.py --configs 1:1:0:0 --rounds 5 &&
  step 120 abr_rf_$r env ISR_LIB=$RF python -u tools/ab_chain.py --configs 1:1:0:0 --rounds 5 || exit 1
done
