#!/bin/bash
# Training steps on a high-priority stream (ISR_TRAIN_PRIO=1, option since removed: 65 vs 46 ms,
# profiles/r04_train_prio_ab.jsonl): training tests with it on, then a same-box A/B, alternating.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -3 $O/$name.out; return $rc; }
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
python -c "import torch; print('priority_range', torch.cuda.Stream.priority_range())" &&
ISR_TRAIN_PRIO=1 step 500 pr_tests $PT -s tests/test_gpu_train_cfg3.py tests/test_gpu_dist_train.py &&
ISR_TRAIN_PRIO=1 step 200 pr_on1 python -u tools/bench_train.py --steps 10 --warmup 3 &&
ISR_TRAIN_PRIO=0 step 200 pr_off1 python -u tools/bench_train.py --steps 10 --warmup 3 &&
ISR_TRAIN_PRIO=1 step 200 pr_on2 python -u tools/bench_train.py --steps 10 --warmup 3 &&
ISR_TRAIN_PRIO=0 step 200 pr_off2 python -u tools/bench_train.py --steps 10 --warmup 3
