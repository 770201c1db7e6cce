#!/bin/bash
# round 3 call D: resident solvers with the ordinary launch, graph-captured training, exit probe last.
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dopri5.py tests/test_gpu_ecg.py -q --timeout 300 --timeout-method thread > $O/r03d_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/r03d_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/diag/train_graph.py > $O/r03d_graph.log 2>&1
rc=$?; echo "graph rc=$rc"; tail -4 $O/r03d_graph.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/pexit_fetode2 -o run --output-format csv -- python3 tools/diag/prof_exit.py fetode > $O/pexit_fetode2.log 2>&1
echo "prof rc=$?"; tail -3 $O/pexit_fetode2.log
