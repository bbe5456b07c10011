#!/bin/bash
# Round 6: the round-end tiers as the driver runs them, on the final tree (after the last rebuild).
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r06
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/r06/t23_suite.txt 2>&1
rc=$?; echo "suite rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/t23_smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/r06/t23_bench.json 2> gpurun_out/r06/t23_bench.err
echo "bench rc=$?"
