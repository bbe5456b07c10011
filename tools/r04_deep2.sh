#!/bin/bash
# Deep-ring trunk iteration: correctness (bench + multi-tile geometries), same-process A/B against
# the pair form, tuning counters + ablations.  Each step time-limited; stops at the first failure.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -4 $O/$name.out; [ $rc -ne 0 ] && tail -5 $O/$name.err; return $rc; }
step 120 deep_bench python -u tools/r04_deep_first.py 16 128 128 16 &&
step 120 deep_multi python -u tools/r04_deep_first.py 4 512 512 1 &&
step 120 deep_ragged python -u tools/r04_deep_first.py 1 540 960 1 &&
step 200 ab_deep python -u tools/ab_chain.py --configs 1:1:0:0,1:1:0:4 --rounds 5 &&
bash tools/r04_ablate4.sh 0:0,9:0,4:0,16:0,29:0
