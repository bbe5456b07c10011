#!/bin/bash
# Production wgrad forms bit-identical to the round-4 forms (new test), then the grouped launch's
# split count in the cfg3 step (tuning build, ISR_WGRAD_GROUP_SPLITS): 40 (default) / 19 / 39.
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
mkdir -p $O
TL=$PWD/image_super_resolution_amd/lib/libisr_tuning.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad" > $O/wgrs5_tests.txt 2>&1 || exit 1
for r in 1 2; do
  for sp in 40 19 39; do
    ISR_LIB=$TL ISR_WGRAD_GROUP_SPLITS=$sp timeout -k 10 200 python -u tools/bench_train.py --steps 10 --warmup 3 > $O/wgrs5_$sp.$r.out 2>> $O/wgrs5_err.txt || exit 1
    python3 -c "import json; d=json.loads(open('$O/wgrs5_$sp.$r.out').read().strip().splitlines()[-1]); print(json.dumps({'splits': $sp, 'round': $r, 'ms_per_step': d['ms_per_step']}))" >> $O/wgrs5_train.jsonl
  done
done
# host floor of the step: the same step at batch 1 / 2 / 4 (GPU work 16x / 8x / 4x smaller)
for b in 1 2 4 16; do
  timeout -k 10 200 python -u tools/bench_train.py --steps 10 --warmup 3 --batch $b > $O/hostfloor_$b.out 2>> $O/wgrs5_err.txt || exit 1
  python3 -c "import json; d=json.loads(open('$O/hostfloor_$b.out').read().strip().splitlines()[-1]); print(json.dumps({'batch': $b, 'ms_per_step': d['ms_per_step']}))" >> $O/hostfloor.jsonl
done
