#!/bin/bash
# Rehearse bench.py's N>1 path on a 1-GPU box: 2 ranks share cuda:0 over gloo (the driver's
# 8-GPU run uses one rank per GPU over RCCL), including the cfg3 training leg's data-parallel
# step (bucketed gradient all-reduce) and its scaling_eff field.  usage: bash tools/rehearse_multi.sh
set -eu
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29513 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo --no-cpu-baseline \
  --train-steps 3 --train-warmup 1
