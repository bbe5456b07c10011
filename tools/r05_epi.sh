#!/bin/bash
# Epilogue shortcuts (fmax LeakyReLU, uniform full-tile validity): bitwise on both trunk forms, then
# the whole forward in alternating processes against the previous trunk.hip (lib/libisr_base.so).
set -o pipefail
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=tests/test_gpu_chain.py::test_chain_bitwise_equals_per_conv_launches
ISR_TEST_CHAIN_VARIANTS=0,9 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    "$T[2-36-52-2]" "$T[16-128-128-16]" "$T[1-540-960-1]" "$T[10-768-768-1]" > gpurun_out/r05/epi_tests.txt 2>&1 || exit 1
for i in 1 2 3; do
  ISR_LIB=$PWD/image_super_resolution_amd/lib/libisr_base.so timeout -k 10 120 python -u tools/ab_chain.py --configs 1:1:0:0 --rounds 3 >> gpurun_out/r05/epi_ab_base.txt 2>&1 || exit 1
  timeout -k 10 120 python -u tools/ab_chain.py --configs 1:1:0:0,1:1:0:9 --rounds 3 >> gpurun_out/r05/epi_ab_new.txt 2>&1 || exit 1
done
