#!/bin/bash
# round 3 call B: KAN-RNN encoder parity + timing, then the exit-crash probe (mode $1) last.
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
MODE=${1:-fetode}
timeout -k 10 600 python -u -m pytest tests/test_gpu_kanrnn.py tests/test_gpu_parity.py -k "kanrnn or kancell or bench_config" -v --timeout 300 --timeout-method thread > $O/r03b_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|assert" $O/r03b_tests.log | head -40
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/diag/kanrnn_time.py > $O/r03b_time.log 2>&1
rc=$?; echo "time rc=$rc"; cat $O/r03b_time.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/pexit_$MODE -o run --output-format csv -- python3 tools/diag/prof_exit.py $MODE > $O/pexit_$MODE.log 2>&1
echo "prof rc=$?"; tail -30 $O/pexit_$MODE.log
