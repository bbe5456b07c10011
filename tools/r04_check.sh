#!/bin/bash
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -2 $O/$name.out | cut -c1-300; return $rc; }
step 500 ck_tests python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py tests/test_gpu_train.py tests/test_gpu_train_cfg3.py &&
step 300 ck_bench1 python -u bench.py --no-cpu-baseline &&
step 300 ck_bench2 python -u bench.py --no-cpu-baseline
