#!/bin/bash
# Stability re-run of the round-end tiers on a fresh box: the full -m gpu suite and smoke().
set -o pipefail
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r05/recheck_tests.txt 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05/recheck_smoke.txt 2>&1
