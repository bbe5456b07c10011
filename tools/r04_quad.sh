#!/bin/bash
# Variant 5 (two 8-wave workgroups per CU, 4 waves per SIMD): chain bitwise tests, then a same-box
# A/B against the production pair form; the f2 loader throughput on the box's host cores.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -4 $O/$name.out; return $rc; }
step 400 quad_chain python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_chain.py &&
step 300 quad_ab python -u tools/ab_chain.py --configs 1:1:0:0,1:1:0:5 --rounds 5 &&
step 300 loader python -u tools/bench_loader.py --workers 2 4 8 16 --images 256 --batches 24 --out $O/loader.json
