#!/bin/bash
# PixelShuffle epilogue with 16-byte LDS writes: kernel / model tests, then same-box A/B against
# the previous build (abtmp/libisr_prev.so via ISR_LIB): inference bench and cfg3 step, alternating.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -2 $O/$name.out | cut -c1-330; return $rc; }
PT="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
step 500 ep_tests $PT tests/test_gpu_kernels.py tests/test_gpu_disc.py tests/test_gpu_denoise.py tests/test_gpu_parity.py tests/test_gpu_chain.py tests/test_gpu_train.py &&
step 200 ep_new1 python -u bench.py --no-cpu-baseline &&
ISR_LIB=abtmp/libisr_prev.so step 200 ep_old1 python -u bench.py --no-cpu-baseline &&
step 200 ep_new2 python -u bench.py --no-cpu-baseline &&
ISR_LIB=abtmp/libisr_prev.so step 200 ep_old2 python -u bench.py --no-cpu-baseline &&
step 200 ept_new1 python -u tools/bench_train.py --steps 10 --warmup 3 &&
ISR_LIB=abtmp/libisr_prev.so step 200 ept_old1 python -u tools/bench_train.py --steps 10 --warmup 3 &&
step 200 ept_new2 python -u tools/bench_train.py --steps 10 --warmup 3 &&
ISR_LIB=abtmp/libisr_prev.so step 200 ept_old2 python -u tools/bench_train.py --steps 10 --warmup 3
