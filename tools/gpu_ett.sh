#!/bin/bash
# GPU call: ETT parity tests + ETT forecaster timing at two batch sizes (each step time-limited)
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; return 0; }
step ett_tests timeout -k 10 300 python -u -m pytest tests/test_gpu_ett.py -x -v --timeout 120 --timeout-method thread
step ett_time timeout -k 10 300 python -u -c "
import json, torch, bench
dev = torch.device('cuda:0')
for b in (1024, 8192):
    print(b, json.dumps(bench.ett_rate(dev, batch=b, reps=2, with_cpu=False)), flush=True)
"
step ett_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ett -o run --output-format csv -- python3 -c "
import torch, bench
bench.ett_rate(torch.device('cuda:0'), batch=1024, reps=1, with_cpu=False)
"
tail -15 $O/ett_tests.log; cat $O/ett_time.log; head -12 $O/prof_ett/run_kernel_stats.csv | cut -c1-200
