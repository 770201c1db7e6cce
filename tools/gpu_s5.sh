#!/bin/bash
# GPU call: full gpu suite, ETT timing, then the PMC traffic passes of the LV bench kernel
cd "$(dirname "$0")/.."
R=${ROUND:-r01_s5}
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; return 0; }
step pytest_gpu timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread
step ett_time timeout -k 10 300 python -u -c "
import json, torch, bench
dev = torch.device('cuda:0')
for b in (1024, 8192):
    print(b, json.dumps(bench.ett_rate(dev, batch=b, reps=2, with_cpu=False)), flush=True)
"
step ett_prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ett_$R -o run --output-format csv -- python3 -c "
import torch, bench
bench.ett_rate(torch.device('cuda:0'), batch=1024, reps=1, with_cpu=False)
"
B="--steps 5 --warmup 1 --no-cpu-baseline --train-iters 0 --no-ecg --no-mnist --no-ett"
step pmc_fetch timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$R -o run --output-format csv -- python3 bench.py $B
step pmc_write timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$R -o run --output-format csv -- python3 bench.py $B
step pmc_sq timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d $O/pmc_sq_$R -o run --output-format csv -- python3 bench.py $B
python tools/pmc_traffic.py $O/pmc_fetch_$R $O/pmc_write_$R $O/pmc_sq_$R --out $O/${R}_pmc_traffic.json > /dev/null
tail -3 $O/pytest_gpu.log; cat $O/ett_time.log; head -6 $O/prof_ett_$R/run_kernel_stats.csv | cut -c1-160; cat $O/${R}_pmc_traffic.json | head -30
