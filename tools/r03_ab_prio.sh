#!/bin/bash
# Same-box A/B of trunk builds: production vs s_setprio variants (ab/libisr_p1.so, _p2.so).
set -u
export TMPDIR=/tmp
O=$PWD/gpurun_out/r03
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -1 $O/$name.out; return $rc; }
step 200 prio_tests env ISR_LIB=$PWD/ab/libisr_p1.so python -u -m pytest tests/test_gpu_chain.py -x -q -k "bitwise" --timeout 150 --timeout-method thread || exit 1
for r in 1 2; do
  step 120 abp_prod_$r python -u tools/ab_chain.py --configs 1:1:0:0 --rounds 5 &&
  step 120 abp_p1_$r env ISR_LIB=$PWD/ab/libisr_p1.so python -u tools/ab_chain.py --configs 1:1:0:0 --rounds 5 &&
  step 120 abp_p2_$r env ISR_LIB=$PWD/ab/libisr_p2.so python -u tools/ab_chain.py --configs 1:1:0:0 --rounds 5 || exit 1
done
step 300 video python -u tools/bench_video.py --frames 48
step 200 smoke python -u -c "import __graft_entry__ as g; g.smoke()"
