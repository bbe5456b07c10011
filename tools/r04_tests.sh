#!/bin/bash
# Targeted -m gpu tests for this round's changes, then the ablation matrix.  Each step time-limited.
set -u
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
step() { local t=$1; shift; local name=$1; shift; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.out 2> $O/$name.err; local rc=$?; echo "rc=$rc"; tail -4 $O/$name.out; return $rc; }
step 400 tests_new python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_data.py \
    "tests/test_gpu_chain.py::test_give_up_training_step_leaves_parameters_unchanged" \
    "tests/test_gpu_parity.py::test_model_float_input_skips_the_255_division" tests/test_gpu_dist_train.py &&
bash tools/r04_ablate.sh "$@"
