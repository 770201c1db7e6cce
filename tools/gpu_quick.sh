#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
for nt in 256 64; do
  FETODE_FUSED_NT=$nt timeout -k 10 300 python tools/quick_bench.py > gpurun_out/qb_$nt.log 2>&1 || exit 3
  echo "NT=$nt"; cat gpurun_out/qb_$nt.log | grep B=
done
