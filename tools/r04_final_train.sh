#!/bin/bash
# Final training evidence with the grouped weight gradients: plain cfg3 step x2, per-phase GPU
# times, and the step under rocprofv3 --kernel-trace --stats.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
T=/tmp/isr_prof_train
mkdir -p $O $T
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -2 $O/$name.out; return $rc; }
step 200 ft_plain1 python -u tools/bench_train.py --steps 10 --warmup 3 &&
step 200 ft_plain2 python -u tools/bench_train.py --steps 10 --warmup 3 &&
step 300 ft_phases python -u tools/train_phases.py &&
step 600 ft_prof rocprofv3 --kernel-trace --stats --output-format csv -d $T -o train -- python3 tools/bench_train.py --steps 3 --warmup 2 &&
cp $T/train_kernel_stats.csv $O/r04_train_kernel_stats_grouped.csv
