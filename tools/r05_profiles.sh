#!/bin/bash
# Round-5 measurements: the committed profiles (tools/make_profiles.sh r05: rocprofv3 kernel stats of
# bench.py, PMC passes -> profiles/r05_pmc_traffic.json, the bench line after them, the cfg3 step
# under rocprofv3), then cfg5 video (1080p -> 4K at batch 1, 2, 4) and the cfg4 still (whole image
# as ONE block on one GPU, now on the trunk kernel; the 8-rank block deal simulated).
set -o pipefail
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/make_profiles.sh r05 > gpurun_out/r05/make_profiles.txt 2>&1 || exit 1
for b in 1 2 4; do
  timeout -k 10 240 python -u tools/bench_video.py --frames 24 --batch $b >> gpurun_out/r05/video_bench.jsonl 2>> gpurun_out/r05/video_err.txt || exit 1
done
timeout -k 10 300 python -u tools/bench_still.py --shard blocks > gpurun_out/r05/still_blocks.json 2> gpurun_out/r05/still_err.txt &&
timeout -k 10 300 python -u tools/bench_still.py --shard blocks --sim-world 8 > gpurun_out/r05/still_shards.json 2>> gpurun_out/r05/still_err.txt
