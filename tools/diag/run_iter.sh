#!/bin/bash
# one optimisation iteration: stamped phase attribution + quick timing (+ optional GPU tests)
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
STAMP_B=4096 FETODE_LIB=$PWD/fet-ode_amd/libfetode_stamps.so timeout -k 10 300 python tools/diag/stamps.py || exit 3
timeout -k 10 300 python tools/quick_bench.py || exit 3
if [ -n "$RUN_TESTS" ]; then
  timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log; exit $rc
fi
