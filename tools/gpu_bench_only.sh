#!/bin/bash
# GPU call: default bench (the contract line) then the rocprofv3 kernel-trace stats of a short bench
cd "$(dirname "$0")/.."
R=${ROUND:-r04}
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; return 0; }
step bench timeout -k 10 600 python bench.py
tail -1 $O/bench.log > $O/bench_$R.json
cat $O/bench_$R.json | head -c 600; echo
[ -n "$NO_PROF" ] && exit 0
step prof_stats timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$R -o run --output-format csv -- python3 bench.py --steps 200 --warmup 100 --no-cpu-baseline --train-iters 20
rm -f $O/prof_$R/run_kernel_trace.csv
