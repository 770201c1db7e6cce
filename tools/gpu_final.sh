#!/bin/bash
# GPU call: full gpu suite, smoke, default bench (contract line), then the rocprofv3 kernel-trace
# stats of the same bench (last: rocprofv3 has crashed at its own exit after writing the CSVs)
cd "$(dirname "$0")/.."
R=${ROUND:-r01_s6}
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; return 0; }
step pytest_gpu timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench timeout -k 10 500 python bench.py
tail -1 $O/bench.log > $O/bench_$R.json
tail -3 $O/pytest_gpu.log; tail -1 $O/smoke.log; cat $O/bench_$R.json
step prof_stats timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$R -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --ett-batch 1024
