#!/bin/bash
# Round 6, tenth GPU call (tuning library shipped for this call only): the chain bitwise tests on every
# remaining A/B trunk form, and the Scaler conv-variant A/B inside the production forward (bf16).
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
export ISR_LIB=$PWD/image_super_resolution_amd/lib/libisr_tuning.so
step 500 t10_chain_tuning.txt python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_chain.py -k bitwise
step 300 t10_ab_scaler.txt python -u tools/ab_scaler.py --variants 0,1,2,3,8,9 --rounds 7 --steps 5
