#!/bin/bash
# Round 6, fourth GPU call: fp16 inference storage — its kernel tests first, then the chain
# bitwise tests, the cfg4/cfg5 parity tests that bf16 storage failed, the default-mode SRGAN step,
# the DP test over both optimiser orders, and a short bench.
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r06
mkdir -p $O
step() {  # step <seconds> <log> <cmd...>
  local t=$1 log=$2; shift 2
  timeout -k 10 $t "$@" > $O/$log 2>&1
  local rc=$?
  echo "step $log rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
step 300 t4_fp16.txt $PYT -s tests/test_gpu_fp16.py
step 400 t4_chain.txt $PYT tests/test_gpu_chain.py
step 400 t4_video.txt $PYT -s tests/test_gpu_video1080.py tests/test_gpu_video.py
step 700 t4_still4k.txt $PYT -s tests/test_gpu_still4k.py
step 300 t4_cfg3.txt $PYT -s tests/test_gpu_train_cfg3.py -k default_mode
step 600 t4_dist.txt $PYT -s tests/test_gpu_dist_train.py
step 400 t4_bench.txt python -u bench.py --steps 20 --warmup 5
