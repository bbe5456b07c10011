#!/bin/bash
# Variant 6 (XCD-aware tile deal): chain bitwise tests and a same-box A/B against production;
# then the round-4 evidence script (pair stamps, plain train bench, PMC per-cause ablations).
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -4 $O/$name.out; return $rc; }
step 400 xcd_chain python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_chain.py &&
step 300 xcd_ab python -u tools/ab_chain.py --configs 1:1:0:0,1:1:0:6 --rounds 6 &&
bash tools/r04_items.sh
