#!/bin/bash
# Round-6 measurements with fp16 inference storage: the committed profiles (tools/make_profiles.sh r06:
# rocprofv3 kernel stats of bench.py, PMC passes -> profiles/r06_pmc_traffic.json, the bench line
# after them, the cfg3 step under rocprofv3), then cfg5 video (1080p -> 4K at batch 1 and 2) and the
# cfg4 still as one block on one GPU.
set -o pipefail
mkdir -p gpurun_out/r06
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/make_profiles.sh r06 > gpurun_out/r06/make_profiles.txt 2>&1 || exit 1
for b in 1 2; do
  timeout -k 10 240 python -u tools/bench_video.py --frames 24 --batch $b >> gpurun_out/r06/video_bench.jsonl 2>> gpurun_out/r06/video_err.txt || exit 1
done
timeout -k 10 300 python -u tools/bench_still.py --shard blocks > gpurun_out/r06/still_blocks.json 2> gpurun_out/r06/still_err.txt
timeout -k 10 300 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_train_cfg3.py -k default_mode > gpurun_out/r06/t8_cfg3.txt 2>&1
echo "cfg3 default-mode test rc=$?"
