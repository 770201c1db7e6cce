#!/bin/bash
# One PMC round on the GPU box (one counter group per pass, --kernel-trace only beside --pmc):
#  (1) the LV rk4 fused kernel: SQ groups + FETCH_SIZE / WRITE_SIZE -> the HBM-traffic summary the
#      bench line cites (profiles/<R>_v4_pmc_traffic.json);
#  (2) tools/pmc_kernels.sh over tools/diag/prof_targets.py (wide ETT layers, MNIST head, training
#      step) -> a per-kernel summary.
cd "$(dirname "$0")/.."
R=${ROUND:-r03}
O=gpurun_out
mkdir -p $O profiles
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; return 0; }
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --train-iters 0 --no-ecg --no-mnist --no-ett --no-dopri5"
step pmc_a timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $O/pmc_a_$R -o run --output-format csv -- $B
step pmc_b timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_b_$R -o run --output-format csv -- $B
step pmc_fetch timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_fetch_$R -o run --output-format csv -- $B
step pmc_write timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_write_$R -o run --output-format csv -- $B
FETODE_PMC_KERNEL="fused4_kernel<10, 10, 10, 12, true, true" python tools/pmc_traffic.py $O/pmc_fetch_$R $O/pmc_write_$R $O/pmc_a_$R $O/pmc_b_$R --out $O/${R}_v4_pmc_traffic.json > $O/pmc_traffic.log 2>&1 || exit 3
cp $O/${R}_v4_pmc_traffic.json profiles/${R}_v4_pmc_traffic.json
TAG=${R}_k bash tools/pmc_kernels.sh
python tools/pmc_summary.py $O/pmc_${R}_k_a $O/pmc_${R}_k_b $O/pmc_${R}_k_c --json $O/${R}_kernels_pmc.json > $O/${R}_kernels_pmc.txt
