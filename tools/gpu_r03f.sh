#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_dopri5.py tests/test_gpu_dopri5.py -v -s --timeout 400 --timeout-method thread > $O/r03f_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|assert|sharded|single resident|^host" $O/r03f_tests.log | head -40
