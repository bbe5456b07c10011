#!/bin/bash
# With the D step on its own stream: weight gradients on the side stream (default) vs on the main
# stream (ISR_TRAIN_SIDE=0), and the reduce stream option (ISR_TRAIN_RED_STREAM=1); cfg3 step, same box.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -1 $O/$name.out | cut -c1-200; return $rc; }
step 200 sd_base1 python -u tools/bench_train.py --steps 10 --warmup 3 &&
ISR_TRAIN_SIDE=0 step 200 sd_noside1 python -u tools/bench_train.py --steps 10 --warmup 3 &&
ISR_TRAIN_RED_STREAM=1 step 200 sd_red1 python -u tools/bench_train.py --steps 10 --warmup 3 &&
step 200 sd_base2 python -u tools/bench_train.py --steps 10 --warmup 3 &&
ISR_TRAIN_SIDE=0 step 200 sd_noside2 python -u tools/bench_train.py --steps 10 --warmup 3 &&
ISR_TRAIN_RED_STREAM=1 step 200 sd_red2 python -u tools/bench_train.py --steps 10 --warmup 3
