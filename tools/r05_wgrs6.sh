#!/bin/bash
# Loader waves for the grouped weight gradients (tuning build): cfg 16 = row sweep + 2 DMA-only
# waves per block, 17 = + 2 rows read ahead; 0 = row sweep (production), 12 = round-4 form.
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
mkdir -p $O
TL=$PWD/image_super_resolution_amd/lib/libisr_tuning.so
K=$O/wgrs6_kernel.jsonl
run() { timeout -k 10 120 python -u tools/ab_wgrad_group.py "$@" >> $K 2>> $O/wgrs6_err.txt; }
for r in 1 2; do
  for v in 12 0 16 17; do ISR_LIB=$TL ISR_WGRAD_GROUP_CFG=$v run --dump /tmp/wg_$v.pt || exit 1; done
done
for v in 0 16 17; do python -u tools/ab_wgrad_group.py --compare /tmp/wg_12.pt /tmp/wg_$v.pt >> $K || exit 1; done
for r in 1 2; do
  for v in 0 16; do
    ISR_LIB=$TL ISR_WGRAD_GROUP_CFG=$v timeout -k 10 200 python -u tools/bench_train.py --steps 10 --warmup 3 > $O/wgrs6_$v.$r.out 2>> $O/wgrs6_err.txt || exit 1
    python3 -c "import json; d=json.loads(open('$O/wgrs6_$v.$r.out').read().strip().splitlines()[-1]); print(json.dumps({'group_cfg': $v, 'round': $r, 'ms_per_step': d['ms_per_step']}))" >> $O/wgrs6_train.jsonl
  done
done
