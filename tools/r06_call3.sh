#!/bin/bash
# Round 6, third GPU call: the re-targeted parity tests after the first run's findings, and the
# enqueue-order diagnostic over 2 steps with and without the round-5 guard path.
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
step 300 t_kernels3.txt $PYT tests/test_gpu_kernels.py -k "wgrad"
step 300 t_cfg3_3.txt $PYT -s tests/test_gpu_train_cfg3.py -k default_mode
step 400 t_video3.txt $PYT -s tests/test_gpu_video1080.py tests/test_gpu_video.py
step 700 t_still4k3.txt $PYT -s tests/test_gpu_still4k.py
step 420 diag_dp_s2.txt python -u tools/diag_dp_order.py --steps 2 --out $O/diag_dp_order_s2.txt
step 420 diag_dp_s2_r5.txt python -u tools/diag_dp_order.py --steps 2 --round5-guard --out $O/diag_dp_order_s2_r5guard.txt
