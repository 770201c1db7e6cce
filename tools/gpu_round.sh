#!/bin/bash
# one GPU call: tests, smoke, quick bench; stops after any crash/timeout (status >1)
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc2=$?; echo "smoke rc=$rc2" | tee -a gpurun_out/smoke.log
if [ $rc2 -gt 1 ]; then exit $rc2; fi
timeout -k 10 300 python tools/quick_bench.py > gpurun_out/quick_bench.log 2>&1
echo "bench rc=$?" | tee -a gpurun_out/quick_bench.log
tail -5 gpurun_out/pytest_gpu.log; cat gpurun_out/smoke.log gpurun_out/quick_bench.log
