#!/bin/bash
# GPU call: gpu suite (no -x: see every failure), smoke, default bench (the contract line), then
# the rocprofv3 kernel-trace stats of a short bench.  Every step has its own time limit; a step
# that crashes / times out (rc > 1) ends the call.
cd "$(dirname "$0")/.."
R=${ROUND:-r04}
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; return 0; }
step pytest_gpu timeout -k 10 ${PYTEST_LIMIT:-900} python -u -m pytest tests -q -m gpu ${PYTEST_ARGS:-} --timeout 240 --timeout-method thread
tail -25 $O/pytest_gpu.log
[ -n "$NO_BENCH" ] && exit 0
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
tail -1 $O/smoke.log
step bench timeout -k 10 600 python bench.py
tail -1 $O/bench.log > $O/bench_$R.json
cat $O/bench_$R.json
[ -n "$NO_PROF" ] && exit 0
step prof_stats timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$R -o run --output-format csv -- python3 bench.py --steps 200 --warmup 100 --no-cpu-baseline --train-iters 20
# keep gpurun_out small (it is merged back only below 64 MiB): the stats CSV, not the traces
f=$(find $O/prof_$R -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" $O/${R}_kernel_stats.csv
rm -rf $O/prof_$R
