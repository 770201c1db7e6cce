#!/bin/bash
# One PMC round on the GPU box (one counter group per pass, --kernel-trace only beside --pmc):
#  (1) the LV rk4 fused kernel: SQ groups + FETCH_SIZE / WRITE_SIZE -> the HBM-traffic summary the
#      bench line cites (profiles/<R>_v4_pmc_traffic.json);
#  (2) tools/pmc_kernels.sh over tools/diag/prof_targets.py (wide ETT layers, MNIST head, training
#      step) -> a per-kernel summary.
cd "$(dirname "$0")/.."
R=${ROUND:-r04}
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
# issue / MFMA / wait accounting per kernel (tools/pmc_issue.py -> the bench line's `issue` and `mfma`)
TAG=${R}_i ISSUE=1 ONLY_ISSUE=1 bash tools/pmc_kernels.sh
python tools/pmc_summary.py $O/pmc_${R}_i_v $O/pmc_${R}_i_m $O/pmc_${R}_i_w --json $O/${R}_pmc_issue_raw.json > $O/${R}_pmc_issue_raw.txt || exit 3
python tools/pmc_issue.py $O/${R}_pmc_issue_raw.json --out $O/${R}_pmc_issue.json > $O/${R}_pmc_issue.txt || exit 3
cp $O/${R}_pmc_issue.json $O/${R}_pmc_issue_raw.json profiles/
