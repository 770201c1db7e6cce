#!/bin/bash
# GPU call: gradient tests, training-iteration timing, kernel stats of the training loop
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_grad.py > gpurun_out/grad.log 2>&1
rc=$?; echo "grad rc=$rc"; tail -5 gpurun_out/grad.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u tools/diag/train_prof.py > gpurun_out/train_prof.log 2>&1; rc=$?; echo "prof rc=$rc"; cat gpurun_out/train_prof.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o run --output-format csv -- python3 tools/diag/train_prof.py > gpurun_out/prof_train.log 2>&1; echo "rocprof rc=$?"
head -12 gpurun_out/prof_train/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
