#!/bin/bash
# GPU call: ETT forecaster timing for outputs-per-wave thresholds + the ECG/ETT gpu tests
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; return 0; }
step ett_tests timeout -k 10 300 python -u -m pytest tests/test_gpu_ett.py tests/test_gpu_ecg.py -x -q --timeout 120 --timeout-method thread
for mb in 512 1024 2048; do
FETODE_WAVE_MIN_BLOCKS=$mb step ett_time_$mb timeout -k 10 200 python -u -c "
import json, torch, bench
dev = torch.device('cuda:0')
for b in (1024, 8192):
    r = bench.ett_rate(dev, batch=b, reps=2, with_cpu=False); print($mb, b, r['ms_per_batch'], flush=True)
"
done
tail -2 $O/ett_tests.log; cat $O/ett_time_*.log | grep -v amdgpu.ids
