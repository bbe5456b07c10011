#!/bin/bash
# Split-K reduce kernel shapes (tuning build, ISR_WGRAD_RED): the cfg3 step with each, and with no
# reduce at all (the bound), alternating.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
TL=$PWD/image_super_resolution_amd/lib/libisr_tuning.so
for r in 1 2; do
  for v in 0 1 2 3 4 nored; do
    if [ $v = nored ]; then
      ISR_LIB=$TL ISR_WGRAD_NO_REDUCE=1 timeout -k 10 200 python -u tools/bench_train.py --steps 10 --warmup 3 > $O/red_$v.$r.out 2> $O/red_$v.$r.err || exit 1
    else
      ISR_LIB=$TL ISR_WGRAD_RED=$v timeout -k 10 200 python -u tools/bench_train.py --steps 10 --warmup 3 > $O/red_$v.$r.out 2> $O/red_$v.$r.err || exit 1
    fi
    python3 -c "import json; d=json.loads(open('$O/red_$v.$r.out').read().strip().splitlines()[-1]); print(json.dumps({'red': '$v', 'round': $r, 'ms_per_step': d['ms_per_step']}))"
  done
done
