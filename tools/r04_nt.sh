#!/bin/bash
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -4 $O/$name.out; return $rc; }
step 400 nt_chain python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_chain.py &&
step 300 nt_ab python -u tools/ab_chain.py --configs 1:1:0:0,1:1:0:7,1:1:0:8 --rounds 6
