#!/bin/bash
# conv3x3 MFMA priority (lib/libisr_cprio.so) vs production: kernel tests, SRGAN step A/B.
set -u
export TMPDIR=/tmp
O=$PWD/gpurun_out/r03
mkdir -p $O
CP=$PWD/image_super_resolution_amd/lib/libisr_cprio.so
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -1 $O/$name.out | cut -c1-220; return $rc; }
step 300 cp_tests env ISR_LIB=$CP python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_chain.py -x -q --timeout 200 --timeout-method thread || exit 1
for r in 1 2; do
  step 300 cp_new_$r env ISR_LIB=$CP python -u tools/bench_train.py --steps 5 --warmup 2 &&
  step 300 cp_old_$r python -u tools/bench_train.py --steps 5 --warmup 2 || exit 1
done
