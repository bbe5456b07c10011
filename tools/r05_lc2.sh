#!/bin/bash
# Loader / consumer trunk form v2 (cross-chunk step-0 prefetch, deferred publish): bitwise vs
# per-conv, whole-forward A/B against the pair form, tuning-build ablations.
set -o pipefail
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=tests/test_gpu_chain.py::test_chain_bitwise_equals_per_conv_launches
ISR_TEST_CHAIN_VARIANTS=9 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    "$T[2-36-52-2]" "$T[1-128-128-1]" "$T[16-128-128-16]" "$T[1-540-960-1]" "$T[4-512-512-1]" \
    > gpurun_out/r05/lc2_tests.txt 2>&1 &&
timeout -k 10 240 python -u tools/ab_chain.py --configs 1:1:0:0,1:1:0:9 --rounds 5 > gpurun_out/r05/lc2_ab.txt 2>&1 &&
ISR_LIB=$PWD/image_super_resolution_amd/lib/libisr_tuning.so ISR_CHAIN_VARIANT=9 timeout -k 10 300 \
    python -u tools/ab_trunk.py --configs 0:0,9:0,2:0,6:0,25:0,31:0 --rounds 3 > gpurun_out/r05/lc2_ablate.jsonl 2>&1
