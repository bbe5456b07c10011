#!/bin/bash
# Loader / consumer trunk form (isr_conv_chain variant 9): bitwise vs per-conv on the small chain
# geometries first, then the whole-forward A/B against the pair form (variant 0).
set -o pipefail
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=tests/test_gpu_chain.py::test_chain_bitwise_equals_per_conv_launches
ISR_TEST_CHAIN_VARIANTS=9 timeout -k 10 240 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    "$T[2-36-52-2]" "$T[1-128-128-1]" "$T[16-128-128-16]" > gpurun_out/r05/lc_tests.txt 2>&1 &&
timeout -k 10 240 python -u tools/ab_chain.py --configs 1:1:0:0,1:1:0:9 --rounds 5 > gpurun_out/r05/lc_ab.txt 2>&1
