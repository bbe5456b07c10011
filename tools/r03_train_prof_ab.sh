#!/bin/bash
# Same-box kernel traces of the SRGAN step: round-2 worktree vs current tree.
set -u
export TMPDIR=/tmp
O=$PWD/gpurun_out/r03
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pt3 -o t -- python3 tools/bench_train.py --steps 3 --warmup 2 > $O/tp_r03.out 2> $O/tp_r03.err && cp /tmp/pt3/t_kernel_stats.csv $O/tp_r03_stats.csv &&
(cd ab/r02 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pt2 -o t -- python3 tools/bench_train.py --steps 3 --warmup 2 > $O/tp_r02.out 2> $O/tp_r02.err) && cp /tmp/pt2/t_kernel_stats.csv $O/tp_r02_stats.csv && tail -1 $O/tp_r03.out $O/tp_r02.out | cut -c1-200
