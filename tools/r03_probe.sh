#!/bin/bash
# Round-3 GPU probe: parity tests of the changed paths, bench line, kernel trace, trunk item
# stamps (tuning build), cfg4 multi-rank prediction, training step.  Each step time-limited.
set -u
export TMPDIR=/tmp
O=gpurun_out/r03
mkdir -p $O
TL=$PWD/image_super_resolution_amd/lib/libisr_tuning.so
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -3 $O/$name.out; return $rc; }
step 400 tests python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_train.py tests/test_gpu_dist_train.py tests/test_gpu_disc.py -x -q --timeout 200 --timeout-method thread &&
step 150 bench python -u bench.py &&
step 300 rocprof rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bench -o bench -- python3 bench.py --no-cpu-baseline &&
cp /tmp/prof_bench/bench_kernel_stats.csv $O/bench_kernel_stats.csv &&
step 120 items env ISR_LIB=$TL python -u tools/trunk_items.py 0 &&
step 300 still_bands python -u tools/bench_still.py --reps 2 --shard bands --sim-world 8 &&
step 300 train python -u tools/bench_train.py --steps 5 --warmup 2
