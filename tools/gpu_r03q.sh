#!/bin/bash
# wide resident dopri5: parity vs the host loop, the wide / ETT suites (tile refactor), timing
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_wide_dopri5.py > $O/wide_dopri5_test.log 2>&1; rc=$?; tail -25 $O/wide_dopri5_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/diag/wide_dopri5_time.py > $O/wide_dopri5_time.log 2>&1; rc=$?; grep -v amdgpu.ids $O/wide_dopri5_time.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_ett.py > $O/wide_ett_test.log 2>&1; rc=$?; tail -5 $O/wide_ett_test.log; exit $rc
