#!/bin/bash
# Round 6: (1) the chain bitwise tests on the tuning library after the variant-1 2 GiB guard;
# (2) per-dispatch cycles and clock of the training step's kernels (cfg3, tools/bench_train.py).
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r06
ISR_LIB=$PWD/image_super_resolution_amd/lib/libisr_tuning.so timeout -k 10 500 python -u -m pytest -v --timeout 300 \
  --timeout-method thread tests/test_gpu_chain.py -k bitwise > gpurun_out/r06/t20_chain_tuning.txt 2>&1
rc=$?; echo "chain tuning rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES --output-format csv -d gpurun_out/r06/pmc_train20 -o tr -- \
  python3 tools/bench_train.py --steps 3 --warmup 2 > gpurun_out/r06/t20_train.json 2> gpurun_out/r06/t20_train.err
echo "train pmc rc=$?"
