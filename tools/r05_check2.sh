#!/bin/bash
# Round-5 GPU check, second half: the test files after test_gpu_train_cfg3.py, smoke(), the default
# bench line and the 2-rank gloo rehearsal.
set -o pipefail
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_trained.py tests/test_gpu_vgg.py tests/test_gpu_video.py \
    tests/test_gpu_video1080.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05/tests2.txt 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05/smoke.txt 2>&1 &&
timeout -k 10 420 python -u bench.py > gpurun_out/r05/bench.json 2> gpurun_out/r05/bench_err.txt &&
timeout -k 10 420 bash tools/rehearse_multi.sh > gpurun_out/r05/rehearse.txt 2>&1
