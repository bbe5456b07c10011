#!/bin/bash
# PMC counters of the cfg3 training step (one counter group per pass), summarised per kernel.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
T=/tmp/isr_pmc_train_end
mkdir -p $O $T
bash tools/profile_pmc.sh $T tools/bench_train.py --steps 2 --warmup 1 > $O/train_pmc_end.log 2>&1 || { tail -5 $O/train_pmc_end.log; exit 1; }
python3 tools/pmc_summary.py $T --json $O/r04_train_pmc_summary_end.json > /dev/null && echo summary ok
