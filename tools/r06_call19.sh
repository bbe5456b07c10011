#!/bin/bash
# Round 6: effective clock of every trunk dispatch over one bench.py run (GRBM_GUI_ACTIVE / 8 /
# dispatch time): the sustained forwards of the timed region vs the isolated launches of the old
# per-kernel timing, which ran faster.
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r06
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES --output-format csv -d gpurun_out/r06/pmc_clk19 -o clk -- \
  python3 bench.py --no-cpu-baseline --no-storage-ab --train-steps 0 > gpurun_out/r06/t19_bench.json 2> gpurun_out/r06/t19_bench.err
echo "rc=$?"
