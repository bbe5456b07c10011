#!/bin/bash
# End-of-round check with the training-step overlaps: full -m gpu suite, smoke(), the default
# bench line, the cfg3 step x2, and the step under rocprofv3 --kernel-trace --stats.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
T=/tmp/isr_prof_train2
mkdir -p $O $T
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -3 $O/$name.out | cut -c1-400; return $rc; }
step 900 f2_gpu python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread &&
step 200 f2_smoke python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" &&
step 300 f2_bench python -u bench.py &&
step 200 f2_train1 python -u tools/bench_train.py --steps 10 --warmup 3 &&
step 200 f2_train2 python -u tools/bench_train.py --steps 10 --warmup 3 &&
step 600 f2_prof rocprofv3 --kernel-trace --stats --output-format csv -d $T -o train -- python3 tools/bench_train.py --steps 5 --warmup 3 &&
cp $T/train_kernel_stats.csv $O/r04_train_kernel_stats_overlap.csv
