#!/bin/bash
# round 3 call E: sharded resident dopri5 (2 ranks on cuda:0, IPC inboxes) + the single-device dopri5 suite
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_dopri5.py tests/test_gpu_dopri5.py -v --timeout 400 --timeout-method thread > $O/r03e_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|assert" $O/r03e_tests.log | head -40
