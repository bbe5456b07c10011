#!/bin/bash
# Host side of the cfg3 step: cProfile of tools/bench_train.py (5 timed steps) and the aten ops
# a step issues with their call sites (ISR_TORCH_PROFILE_ALL).
set -u
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r05
mkdir -p $O
timeout -k 10 300 python -u -m cProfile -o /tmp/host.prof tools/bench_train.py --steps 5 --warmup 2 > $O/host_prof_bench.json 2> $O/host_prof_err.txt || exit 1
python3 - > $O/host_prof.txt <<'PY'
import pstats
s = pstats.Stats('/tmp/host.prof')
s.sort_stats('tottime').print_stats(45)
s.sort_stats('cumulative').print_stats(70)
PY
ISR_TORCH_PROFILE_ALL=1 timeout -k 10 300 python -u tools/bench_train.py --steps 2 --warmup 1 --torch-profile > $O/torch_ops.txt 2>> $O/host_prof_err.txt || exit 1
