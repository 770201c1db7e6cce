#!/bin/bash
# wide VJP parity (Ferro one-pass, KANLinear MFMA, the KANFET layer under autograd), then the ETT
# training step: non-finite check, wall time at two batches and its profile
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wide.py > $O/wide_bwd_test.log 2>&1; rc=$?; tail -15 $O/wide_bwd_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/diag/ett_nan.py > $O/ett_nan.log 2>&1; rc=$?; grep -v amdgpu.ids $O/ett_nan.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/diag/ett_train.py > $O/ett_train_1024.log 2>&1 && grep -v amdgpu.ids $O/ett_train_1024.log &&
B=8192 timeout -k 10 300 python -u tools/diag/ett_train.py > $O/ett_train_8192.log 2>&1 && grep -v amdgpu.ids $O/ett_train_8192.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ett_train_prof -o run --output-format csv -- python3 tools/diag/ett_train.py > $O/ett_train_prof.log 2>&1 &&
echo prof ok
