#!/bin/bash
# VGG(hr) queued behind the trunk kernel only (ISR_TRAIN_HR_EARLY=1) vs behind the whole generator
# A/B of the cfg3 step (ISR_TRAIN_HR_EARLY=1 vs 0, both with the D-step overlap), alternating.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -3 $O/$name.out; return $rc; }
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
step 500 he_tests $PT -s tests/test_gpu_train_cfg3.py tests/test_gpu_vgg.py tests/test_gpu_disc.py tests/test_gpu_chain.py tests/test_gpu_train.py &&
ISR_TRAIN_HR_EARLY=1 step 200 he_on1 python -u tools/bench_train.py --steps 10 --warmup 3 &&
ISR_TRAIN_HR_EARLY=0 step 200 he_off1 python -u tools/bench_train.py --steps 10 --warmup 3 &&
ISR_TRAIN_HR_EARLY=1 step 200 he_on2 python -u tools/bench_train.py --steps 10 --warmup 3 &&
ISR_TRAIN_HR_EARLY=0 step 200 he_off2 python -u tools/bench_train.py --steps 10 --warmup 3 &&
step 400 he_dist $PT tests/test_gpu_dist_train.py
