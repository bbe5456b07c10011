#!/bin/bash
# Round 6, seventh GPU call: the storage A/B again with the plan holding its weights (the previous
# bf16 arm ran on freed weights), its effective-clock PMC pass, the fp16 tests incl. the lifetime
# test, and the default-mode SRGAN step with the autocast yardstick.
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
step 300 ab7_trained.txt python -u tools/ab_storage.py --rounds 9 --steps 10
step 120 ab7_clock.txt rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_clock7 -o clk -- python3 tools/ab_storage.py --rounds 2 --steps 3
step 300 t7_fp16.txt $PYT -s tests/test_gpu_fp16.py
step 300 t7_cfg3.txt $PYT -s tests/test_gpu_train_cfg3.py -k default_mode
