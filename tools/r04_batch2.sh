#!/bin/bash
# Round-4 batch 2: buffer-resource extents + fold-kernel recompute (chain bitwise, production and
# -DISR_TRUNK_INTERLEAVE=1 builds), the cfg3-shape training test, the block deal (tests + 8-rank
# simulation with the D2H hand-off).  Each step time-limited; stops at the first failure.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -4 $O/$name.out; return $rc; }
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
step 400 b2_chain $PT tests/test_gpu_chain.py &&
ISR_LIB=$PWD/image_super_resolution_amd/lib/libisr_interleave.so step 400 b2_chain_interleave $PT tests/test_gpu_chain.py &&
step 500 b2_cfg3 $PT -s tests/test_gpu_train_cfg3.py &&
step 400 b2_still $PT -s tests/test_gpu_still4k.py -k "bands or blocks" &&
step 300 b2_still_blocks python -u tools/bench_still.py --shard blocks --sim-world 8 --reps 3 --out $O/still_shards_blocks.json &&
step 300 b2_still_bands python -u tools/bench_still.py --shard bands --sim-world 8 --reps 3 --out $O/still_shards_bands.json
