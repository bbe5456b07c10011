#!/bin/bash
# Tile configuration of the grouped RDB weight gradients (tuning build, ISR_WGRAD_GROUP_CFG).
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
TL=$PWD/image_super_resolution_amd/lib/libisr_tuning.so
for r in 1 2; do
  for v in ${CFGS:-0 5 6 7}; do
    ISR_LIB=$TL ISR_WGRAD_GROUP_CFG=$v timeout -k 10 200 python -u tools/bench_train.py --steps 10 --warmup 3 > $O/wggc_$v.$r.out 2> $O/wggc_$v.$r.err || exit 1
    python3 -c "import json; d=json.loads(open('$O/wggc_$v.$r.out').read().strip().splitlines()[-1]); print(json.dumps({'group_cfg': $v, 'round': $r, 'ms_per_step': d['ms_per_step']}))"
  done
done
