#!/bin/bash
# round 3 call A: the new wide-layer parity tests, the bench-config robust-subset stats at 1e-5,
# then ONE exit-crash probe under rocprofv3 (mode $1) as the last step (a crash ends the call).
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
MODE=${1:-torch}
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_parity.py -k "b8192 or noncontiguous or robust_subset" -v -s --timeout 300 --timeout-method thread > $O/r03a_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $O/r03a_tests.log; grep -o "robust-subset parity (bench config).*" $O/r03a_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/pexit_$MODE -o run --output-format csv -- python3 tools/diag/prof_exit.py $MODE > $O/pexit_$MODE.log 2>&1
echo "prof rc=$?"; tail -30 $O/pexit_$MODE.log
