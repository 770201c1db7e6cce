#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for lpt in 32 64; do for nt in 64 256; do
  FETODE_FUSED_LPT=$lpt FETODE_FUSED_NT=$nt timeout -k 10 300 python tools/quick_bench.py > gpurun_out/qb_${lpt}_${nt}.log 2>&1 || exit 3
  echo "LPT=$lpt NT=$nt"; grep B= gpurun_out/qb_${lpt}_${nt}.log
done; done
FETODE_FUSED_LPT=64 FETODE_FUSED_NT=256 timeout -k 10 600 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo "pytest(LPT64,NT256) rc=$?"; tail -2 gpurun_out/pytest_gpu.log
