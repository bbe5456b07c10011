#!/bin/bash
# Round-5 final GPU check on the committed code: the full -m gpu suite, smoke(), the default bench
# line and the 2-rank gloo rehearsal of the N>1 fields.
set -o pipefail
mkdir -p gpurun_out/r05
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r05/final_tests.txt 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05/final_smoke.txt 2>&1 &&
timeout -k 10 420 python -u bench.py > gpurun_out/r05/final_bench.json 2> gpurun_out/r05/final_bench_err.txt &&
timeout -k 10 420 bash tools/rehearse_multi.sh > gpurun_out/r05/final_rehearse.txt 2>&1
