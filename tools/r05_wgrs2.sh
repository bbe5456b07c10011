#!/bin/bash
# Row-sweep weight gradients with asm transposing reads (no compiler vmcnt(0) behind the next
# stage's DMA): launch time + bit-identity vs the production tile, then the cfg3 step.
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
mkdir -p $O
TL=$PWD/image_super_resolution_amd/lib/libisr_tuning.so
for v in 0 8 0 8; do
  ISR_LIB=$TL ISR_WGRAD_GROUP_CFG=$v timeout -k 10 120 python -u tools/ab_wgrad_group.py --dump /tmp/wg_$v.pt >> $O/wgrs2_kernel.jsonl 2>> $O/wgrs2_err.txt || exit 1
done
python -u tools/ab_wgrad_group.py --compare /tmp/wg_0.pt /tmp/wg_8.pt >> $O/wgrs2_kernel.jsonl || exit 1
for r in 1 2; do
  for v in 0 8; do
    ISR_LIB=$TL ISR_WGRAD_GROUP_CFG=$v timeout -k 10 200 python -u tools/bench_train.py --steps 10 --warmup 3 > $O/wgrs2_$v.$r.out 2>> $O/wgrs2_err.txt || exit 1
    python3 -c "import json; d=json.loads(open('$O/wgrs2_$v.$r.out').read().strip().splitlines()[-1]); print(json.dumps({'group_cfg': $v, 'round': $r, 'ms_per_step': d['ms_per_step']}))" >> $O/wgrs2_train.jsonl
  done
done
