#!/bin/bash
# Same-box A/B of the SRGAN training step: round-2 code (worktree ab/r02, its own libisr.so)
# against the current tree, alternating processes.
set -u
export TMPDIR=/tmp
O=$PWD/gpurun_out/r03
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -1 $O/$name.out | cut -c1-300; return $rc; }
for r in 1 2; do
  step 300 trainab_r03_$r python -u tools/bench_train.py --steps 5 --warmup 2 &&
  (cd ab/r02 && step 300 trainab_r02_$r python -u tools/bench_train.py --steps 5 --warmup 2) || exit 1
done
