#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
for v in 4 3; do
  FETODE_FUSED_LPT=$v timeout -k 10 300 python tools/quick_bench.py > gpurun_out/qb_$v.log 2>&1 || exit 3
  echo "variant=$v"; grep B= gpurun_out/qb_$v.log
done
