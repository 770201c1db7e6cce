#!/bin/bash
# round 3 call C: KAN-RNN tests + timing after the backward rework, bench smoke of the encoder line,
# then the exit probe (mode $1) last.
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
MODE=${1:-rk4only}
timeout -k 10 600 python -u -m pytest tests/test_gpu_kanrnn.py tests/test_gpu_wide.py -v --timeout 300 --timeout-method thread > $O/r03c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAIL|Error" $O/r03c_tests.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/diag/kanrnn_time.py > $O/r03c_time.log 2>&1
rc=$?; echo "time rc=$rc"; tail -3 $O/r03c_time.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "
import bench, torch, json
print(json.dumps(bench.ett_encoder_rate(torch.device('cuda:0'))))" > $O/r03c_enc.log 2>&1
rc=$?; echo "enc rc=$rc"; tail -2 $O/r03c_enc.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/pexit_$MODE -o run --output-format csv -- python3 tools/diag/prof_exit.py $MODE > $O/pexit_$MODE.log 2>&1
echo "prof rc=$?"; tail -3 $O/pexit_$MODE.log
