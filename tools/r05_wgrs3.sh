#!/bin/bash
# Weight gradients: the production lib's new forms (row sweep + asm reads for every kernel-row
# form) vs the round-4 forms (tuning build: ISR_WGRAD_AR=0 ISR_WGRAD_GROUP_CFG=12), bitwise and
# timed; grouped-launch ablations (no refill DMA / no MFMA) and split counts; GPU wgrad tests.
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
mkdir -p $O
TL=$PWD/image_super_resolution_amd/lib/libisr_tuning.so
K=$O/wgrs3_kernel.jsonl
run() { timeout -k 10 120 python -u tools/ab_wgrad_group.py "$@" >> $K 2>> $O/wgrs3_err.txt; }
ISR_LIB=$TL ISR_WGRAD_GROUP_CFG=12 run --dump /tmp/wg_old.pt || exit 1
run --dump /tmp/wg_new.pt || exit 1
ISR_LIB=$TL ISR_WGRAD_GROUP_CFG=11 run --dump /tmp/wg_ar.pt || exit 1
python -u tools/ab_wgrad_group.py --compare /tmp/wg_old.pt /tmp/wg_new.pt >> $K || exit 1
python -u tools/ab_wgrad_group.py --compare /tmp/wg_old.pt /tmp/wg_ar.pt >> $K || exit 1
for a in 1 2 3; do ISR_LIB=$TL ISR_WGRAD_ABLATE=$a run || exit 1; echo "{\"ablate\": $a}" >> $K; done
for sp in 19 39 59 78; do ISR_LIB=$TL ISR_WGRAD_GROUP_SPLITS=$sp run || exit 1; echo "{\"splits\": $sp}" >> $K; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad" > $O/wgrs3_tests.txt 2>&1 || exit 1
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then E="ISR_LIB=$TL ISR_WGRAD_AR=0 ISR_WGRAD_GROUP_CFG=12"; else E="ISR_LIB=$TL"; fi
    env $E timeout -k 10 200 python -u tools/bench_train.py --steps 10 --warmup 3 > $O/wgrs3_$v.$r.out 2>> $O/wgrs3_err.txt || exit 1
    python3 -c "import json; d=json.loads(open('$O/wgrs3_$v.$r.out').read().strip().splitlines()[-1]); print(json.dumps({'wgrad': '$v', 'round': $r, 'ms_per_step': d['ms_per_step']}))" >> $O/wgrs3_train.jsonl
  done
done
