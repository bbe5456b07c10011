#!/bin/bash
# Trunk-kernel iteration: bitwise chain tests, same-process A/B of the chain variants, per-item
# stamps (tuning build), bench line.  Each step time-limited; stops at the first failure.
set -u
export TMPDIR=/tmp
O=gpurun_out/r03
mkdir -p $O
TAG=${1:-x}
TL=$PWD/image_super_resolution_amd/lib/libisr_tuning.so
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -4 $O/$name.out; return $rc; }
step 200 chain_tests_$TAG python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_video1080.py -x -q --timeout 150 --timeout-method thread &&
step 200 ab_chain_$TAG python -u tools/ab_chain.py --configs 1:1:0:0,1:1:0:2,1:1:0:1 --rounds 5 &&
step 120 items_$TAG env ISR_LIB=$TL python -u tools/trunk_items.py 0 &&
step 150 bench_$TAG python -u bench.py --no-cpu-baseline &&
[ "${2:-}" = "train" ] && step 300 train_prof_$TAG rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_train -o train -- python3 tools/bench_train.py --steps 3 --warmup 2 && cp /tmp/prof_train/train_kernel_stats.csv $O/train_kernel_stats_$TAG.csv
true
