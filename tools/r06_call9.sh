#!/bin/bash
# Round 6, ninth GPU call: the whole -m gpu suite and smoke() on the current tree (fp16 default,
# the deep-ring / loader-consumer trunk forms removed), then the chain tests on the tuning library.
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
step 900 t9_suite.txt python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/
step 300 t9_smoke.txt python -u -c "import __graft_entry__ as g; g.smoke()"
ISR_LIB=$PWD/image_super_resolution_amd/lib/libisr_tuning.so step 400 t9_chain_tuning.txt python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_chain.py -k bitwise
ISR_LIB=$PWD/image_super_resolution_amd/lib/libisr_tuning.so step 300 t9_ab_scaler.txt python -u tools/ab_scaler.py --variants 0,1,2,3,8,9 --rounds 7 --steps 5
