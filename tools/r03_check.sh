#!/bin/bash
# Full GPU suite, bench line, SRGAN step, kernel trace of the bench.  Stops at the first failure.
set -u
export TMPDIR=/tmp
O=$PWD/gpurun_out/r03
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -2 $O/$name.out | cut -c1-400; return $rc; }
step 900 suite python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread &&
step 150 bench python -u bench.py &&
step 300 train python -u tools/bench_train.py --steps 5 --warmup 2
