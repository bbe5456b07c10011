#!/bin/bash
# Round-4 evidence: per-chunk stamps of the pair form (tuning build) and the cfg3 training step
# without the profiler.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -4 $O/$name.out; return $rc; }
ISR_LIB=$PWD/image_super_resolution_amd/lib/libisr_tuning.so step 240 items_pair python -u tools/trunk_items.py 0 &&
step 300 train_plain python -u tools/bench_train.py --steps 10 --warmup 3 &&
step 300 train_plain2 python -u tools/bench_train.py --steps 10 --warmup 3 &&
bash tools/r04_pmc_ablate.sh
