#!/bin/bash
# input slicing up to 8: the wide / ETT / ECG-FerroNet suites and the resident dopri5 parity, timing
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_wide_dopri5.py tests/test_gpu_wide.py tests/test_gpu_ett.py tests/test_gpu_ecg.py > $O/slices_test.log 2>&1; rc=$?; tail -15 $O/slices_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/diag/wide_dopri5_time.py > $O/wide_dopri5_time.log 2>&1; rc=$?; grep -v amdgpu.ids $O/wide_dopri5_time.log | tail -12; exit $rc
