#!/bin/bash
# SRGAN step: the generator's optimiser launches enqueued before the discriminator step
# (ISR_TRAIN_G_FIRST=1) vs after it (0, default), alternating processes; then the cfg3 tests.
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
mkdir -p $O
for r in 1 2 3; do
  for v in 0 1; do
    ISR_TRAIN_G_FIRST=$v timeout -k 10 200 python -u tools/bench_train.py --steps 10 --warmup 3 > $O/gfirst_$v.$r.out 2>> $O/gfirst_err.txt || exit 1
    python3 -c "import json; d=json.loads(open('$O/gfirst_$v.$r.out').read().strip().splitlines()[-1]); print(json.dumps({'g_first': $v, 'round': $r, 'ms_per_step': d['ms_per_step']}))" >> $O/gfirst.jsonl
  done
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train_cfg3.py tests/test_gpu_train.py > $O/gfirst_tests.txt 2>&1 || exit 1
ISR_TRAIN_G_FIRST=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread "tests/test_gpu_dist_train.py::test_two_rank_data_parallel_matches" > $O/gfirst_dist_tests.txt 2>&1
