#!/bin/bash
# wgrad split-K reduce 16 slices vs 4 (lib/libisr_oldred.so): gradient tests, then the SRGAN
# step alternating processes.
set -u
export TMPDIR=/tmp
O=$PWD/gpurun_out/r03
mkdir -p $O
OLD=$PWD/image_super_resolution_amd/lib/libisr_oldred.so
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -1 $O/$name.out | cut -c1-220; return $rc; }
step 500 red_tests python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_disc.py tests/test_gpu_denoise.py tests/test_gpu_dist_train.py -x -q --timeout 200 --timeout-method thread || exit 1
for r in 1 2; do
  step 300 red_new_$r python -u tools/bench_train.py --steps 5 --warmup 2 &&
  step 300 red_old_$r env ISR_LIB=$OLD python -u tools/bench_train.py --steps 5 --warmup 2 || exit 1
done
