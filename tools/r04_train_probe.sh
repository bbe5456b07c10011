#!/bin/bash
# Training-step probes (tuning build, timing only): the step with the weight gradients' split-K
# reduce skipped, and with every weight gradient skipped, against the same build unmodified;
# then the per-phase GPU times of the production build.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -2 $O/$name.out; return $rc; }
TL=$PWD/image_super_resolution_amd/lib/libisr_tuning.so
ISR_LIB=$TL step 240 tp_base python -u tools/bench_train.py --steps 10 --warmup 3 &&
ISR_LIB=$TL ISR_WGRAD_NO_REDUCE=1 step 240 tp_nored python -u tools/bench_train.py --steps 10 --warmup 3 &&
ISR_LIB=$TL ISR_WGRAD_SKIP=1 step 240 tp_nowg python -u tools/bench_train.py --steps 10 --warmup 3 &&
ISR_LIB=$TL step 240 tp_base2 python -u tools/bench_train.py --steps 10 --warmup 3 &&
step 300 tp_phases python -u tools/train_phases.py &&
step 300 tp_torchprof python -u tools/bench_train.py --steps 3 --warmup 2 --torch-profile
