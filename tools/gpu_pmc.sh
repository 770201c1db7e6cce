#!/bin/bash
# One measurement round on the GPU box: rocprofv3 PMC passes (one counter group per pass, no
# tracing domains), the kernel-trace stats, then the contract bench.  The HBM-traffic summary
# is written before the bench runs so the bench line cites this round's counters.
cd "$(dirname "$0")/.."
R=${ROUND:-r01_v4}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; return 0; }
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --train-iters 0"
step pmc_a timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/pmc_a_$R -o run --output-format csv -- $B
step pmc_b timeout -k 10 400 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_b_$R -o run --output-format csv -- $B
step pmc_fetch timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$R -o run --output-format csv -- $B
step pmc_write timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$R -o run --output-format csv -- $B
step prof_stats timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_$R -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --train-iters 0
python tools/pmc_traffic.py $O/pmc_fetch_$R $O/pmc_write_$R $O/pmc_a_$R $O/pmc_b_$R --out $O/${R}_pmc_traffic.json > $O/pmc_traffic.log 2>&1 || exit 3
mkdir -p profiles && cp $O/${R}_pmc_traffic.json profiles/${R}_pmc_traffic.json
step bench timeout -k 10 400 python bench.py
tail -1 $O/bench.log > $O/bench_$R.json
cat $O/bench_$R.json
