#!/bin/bash
# Row-sweep weight gradients (WG::RS, tuning build ISR_WGRAD_GROUP_CFG=8/9/10) vs the production
# grouped tile (cfg 0): launch time + bit-identity of dW/db across processes, then the cfg3 step.
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
mkdir -p $O
TL=$PWD/image_super_resolution_amd/lib/libisr_tuning.so
for v in 0 8 9 10; do
  ISR_LIB=$TL ISR_WGRAD_GROUP_CFG=$v timeout -k 10 120 python -u tools/ab_wgrad_group.py --dump /tmp/wg_$v.pt >> $O/wgrs_kernel.jsonl 2>> $O/wgrs_err.txt || exit 1
done
for v in 8 9 10; do
  python -u tools/ab_wgrad_group.py --compare /tmp/wg_0.pt /tmp/wg_$v.pt >> $O/wgrs_kernel.jsonl || exit 1
done
for r in 1 2; do
  for v in 0 8; do
    ISR_LIB=$TL ISR_WGRAD_GROUP_CFG=$v timeout -k 10 200 python -u tools/bench_train.py --steps 10 --warmup 3 > $O/wgrs_$v.$r.out 2>> $O/wgrs_err.txt || exit 1
    python3 -c "import json; d=json.loads(open('$O/wgrs_$v.$r.out').read().strip().splitlines()[-1]); print(json.dumps({'group_cfg': $v, 'round': $r, 'ms_per_step': d['ms_per_step']}))" >> $O/wgrs_train.jsonl
  done
done
