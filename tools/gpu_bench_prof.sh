#!/bin/bash
# GPU call: pytest -m gpu, bench (contract line), rocprofv3 kernel-trace stats, PMC passes.
# Every GPU step has its own time limit; a crash/timeout (status > 1) ends the script.
cd "$(dirname "$0")/.."
R=${ROUND:-r01}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; return 0; }
step pytest_gpu timeout -k 10 600 python -m pytest tests -q -m gpu
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench timeout -k 10 400 python bench.py
tail -1 $O/bench.log > $O/bench_$R.json
step prof_stats timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$R -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline
step pmc_fetch timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$R -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --train-iters 0 --no-ecg --no-mnist --no-ett
step pmc_write timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$R -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --train-iters 0 --no-ecg --no-mnist --no-ett
step pmc_sq timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d $O/pmc_sq_$R -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --train-iters 0 --no-ecg --no-mnist --no-ett
python tools/pmc_traffic.py $O/pmc_fetch_$R $O/pmc_write_$R $O/pmc_sq_$R --out $O/${R}_pmc_traffic.json > /dev/null
tail -3 $O/pytest_gpu.log; cat $O/smoke.log | tail -2; cat $O/bench_$R.json
