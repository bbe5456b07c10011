#!/bin/bash
# Round 6, first GPU call: the world-2 enqueue-order diagnostic, the uint8 outlier locations and
# the x2 trained weights for cfg5 parity.  A step that ends by signal / fault / timeout ends the
# call; an ordinary Python error (rc 1) lets the next independent step run.
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
step 420 diag_dp_order.txt python -u tools/diag_dp_order.py --steps 1 --out $O/diag_dp_order_s1.txt
step 240 u8_outliers.txt python -u tests/diag_u8_outliers.py --out $O/u8_outliers.json
step 720 train_x2.txt python -u tools/train_weights.py --scale 2 --shape 256 --epochs 12 --steps 500 --out $O/trained_resnet_x2.safetensors
