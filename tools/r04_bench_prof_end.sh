#!/bin/bash
# The default bench command under rocprofv3 --kernel-trace --stats on the last commit: the trunk
# kernel's average duration next to the bench line's live HIP-event figure.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
T=/tmp/isr_prof_bench_end
mkdir -p $O $T
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $T -o bench -- python3 bench.py --no-cpu-baseline > $O/bench_prof_end.out 2> $O/bench_prof_end.err &&
cp $T/bench_kernel_stats.csv $O/r04_bench_kernel_stats_end.csv && tail -1 $O/bench_prof_end.out | cut -c1-200
