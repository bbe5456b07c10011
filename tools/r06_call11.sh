#!/bin/bash
# Round 6, final profile refresh on the committed tree: tools/make_profiles.sh r06 (bench under
# rocprofv3, PMC passes, the bench line, the cfg3 step under rocprofv3), then the 2-rank gloo
# rehearsal of bench.py's N>1 path with the fp16 inference leg.
set -o pipefail
mkdir -p gpurun_out/r06
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/make_profiles.sh r06 > gpurun_out/r06/make_profiles2.txt 2>&1 || exit 1
bash tools/rehearse_multi.sh > gpurun_out/r06/rehearse2.txt 2>&1
echo "rehearsal rc=$?"
