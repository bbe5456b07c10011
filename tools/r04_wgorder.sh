#!/bin/bash
# Grouped weight gradients, split-major block order (default) vs member-major
# (ISR_WGRAD_GROUP_ORDER=0): kernel tests, then a same-box A/B of the cfg3 step, alternating.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -3 $O/$name.out; return $rc; }
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
step 400 wo_tests $PT tests/test_gpu_kernels.py -k "wgrad" &&
ISR_WGRAD_GROUP_ORDER=1 step 200 wo_on1 python -u tools/bench_train.py --steps 10 --warmup 3 &&
ISR_WGRAD_GROUP_ORDER=0 step 200 wo_off1 python -u tools/bench_train.py --steps 10 --warmup 3 &&
ISR_WGRAD_GROUP_ORDER=1 step 200 wo_on2 python -u tools/bench_train.py --steps 10 --warmup 3 &&
ISR_WGRAD_GROUP_ORDER=0 step 200 wo_off2 python -u tools/bench_train.py --steps 10 --warmup 3 &&
step 400 wo_train $PT tests/test_gpu_train.py tests/test_gpu_train_cfg3.py
