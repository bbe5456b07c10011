#!/bin/bash
# Round 6, fifth GPU call: bf16 vs fp16 storage A/B on one box (plain timing, then the rocprofv3
# per-kernel split), the default-mode SRGAN step with its autocast yardstick, then the whole -m gpu
# suite with the fp16 default and the tightened uint8 bars.
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
step 300 ab_storage.txt python -u tools/ab_storage.py --rounds 9 --steps 10
step 300 ab_storage_prof.txt rocprofv3 --kernel-trace --stats -d $O/prof_storage -o ab -- python3 tools/ab_storage.py --rounds 3 --steps 5
step 300 t5_cfg3.txt $PYT -s tests/test_gpu_train_cfg3.py -k default_mode
step 1100 t5_suite.txt python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/
