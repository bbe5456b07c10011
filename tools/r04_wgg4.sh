#!/bin/bash
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
for r in 1 2; do
  for v in 1 4 0; do
    ISR_TRAIN_WG_GROUP=$v timeout -k 10 200 python -u tools/bench_train.py --steps 10 --warmup 3 > $O/wgg4_$v.$r.out 2> $O/wgg4_$v.$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/wgg4_$v.$r.out').read().strip().splitlines()[-1]); print(json.dumps({'wg_group': '$v', 'round': $r, 'ms_per_step': d['ms_per_step']}))"
  done
done
