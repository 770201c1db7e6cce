#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_dopri5.py tests/test_gpu_dist_train.py -v --timeout 400 --timeout-method thread > $O/r03i_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|assert" $O/r03i_tests.log | head -30
[ $rc -le 1 ] || exit $rc
NS=2 bash tools/gpu_rehearse_dist.sh
