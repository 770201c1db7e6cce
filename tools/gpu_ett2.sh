#!/bin/bash
# GPU call: tests touching the wide per-stage kernels + ETT timing + ETT kernel stats
cd "$(dirname "$0")/.."
R=${ROUND:-r01_s7}
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; return 0; }
step wide_tests timeout -k 10 400 python -u -m pytest tests/test_gpu_ett.py tests/test_gpu_ecg.py tests/test_gpu_parity.py tests/test_gpu_grad.py -x -q --timeout 120 --timeout-method thread
step ett_time timeout -k 10 200 python -u -c "
import torch, bench
dev = torch.device('cuda:0')
for b in (1024, 8192):
    r = bench.ett_rate(dev, batch=b, reps=2, with_cpu=False); print(b, r['ms_per_batch'], r['finite'], flush=True)
"
step ett_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ett_$R -o run --output-format csv -- python3 -c "
import torch, bench
bench.ett_rate(torch.device('cuda:0'), batch=8192, reps=1, with_cpu=False)
"
tail -2 $O/wide_tests.log; grep -v amdgpu.ids $O/ett_time.log; head -4 $O/prof_ett_$R/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
