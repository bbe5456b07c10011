#!/bin/bash
# Round 6, second GPU call: the enqueue-order diagnostic (fixed), the re-targeted parity tests
# (trained weights at cfg4 / cfg5, default-mode SRGAN step, wgrad asm-read forms), the dist test
# and the 2-rank rehearsal of bench.py's N-rank fields.  Stops at the first GPU-level failure.
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
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
step 420 diag_dp_order2.txt python -u tools/diag_dp_order.py --steps 1 --out $O/diag_dp_order_s1.txt
step 300 t_kernels.txt $PYT tests/test_gpu_kernels.py -k "wgrad"
step 600 t_still4k.txt $PYT -s tests/test_gpu_still4k.py
step 300 t_video.txt $PYT -s tests/test_gpu_video1080.py tests/test_gpu_video.py
step 300 t_cfg3.txt $PYT -s tests/test_gpu_train_cfg3.py -k default_mode
step 400 t_dist.txt $PYT -s tests/test_gpu_dist_train.py
step 400 rehearse.txt bash tools/rehearse_multi.sh
