#!/bin/bash
# Full -m gpu suite, smoke(), the default bench line and the cfg3 step (production build).
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -3 $O/$name.out; return $rc; }
step 900 full_gpu python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread &&
step 200 full_smoke python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" &&
step 300 full_bench python -u bench.py &&
step 200 full_train python -u tools/bench_train.py --steps 10 --warmup 3
