#!/bin/bash
# Round 6, sixth GPU call: bf16 vs fp16 storage on the bench workload (trained x4 weights, held-out
# tiles) and on the synthetic weights, then one PMC pass for the effective clock of each form
# (GRBM_GUI_ACTIVE / 8 / kernel time, MI355X_MICROARCH.md 'DVFS give-back').
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
step 300 ab_storage_trained.txt python -u tools/ab_storage.py --rounds 9 --steps 10
step 300 ab_storage_synth.txt python -u tools/ab_storage.py --rounds 5 --steps 10 --weights synth
step 120 ab_storage_clock.txt rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_clock -o clk -- python3 tools/ab_storage.py --rounds 2 --steps 3
