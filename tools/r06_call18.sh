#!/bin/bash
# Round 6, final verification on the committed tree: the whole -m gpu suite, smoke().
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r06
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests/ > gpurun_out/r06/t18_suite.txt 2>&1
rc=$?; echo "suite rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/t18_smoke.txt 2>&1
echo "smoke rc=$?"
