#!/bin/bash
# fused-forward variants: bench-config robust-subset parity, then the kernel time per batch size
# (tools/diag/batch_sweep.py, SWEEP_B) of each library; VARIANTS="name=libpath ..."
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in $VARIANTS; do
  n=${v%%=*}; lib=$PWD/${v#*=}
  FETODE_LIB=$lib timeout -k 10 300 python tools/diag/robust_check.py > gpurun_out/rob_$n.log 2>&1
  rc=$?; echo "== $n robust rc=$rc: $(tail -1 gpurun_out/rob_$n.log | cut -c1-600)"; [ $rc -le 1 ] || exit $rc
done
for v in $VARIANTS; do
  n=${v%%=*}; lib=$PWD/${v#*=}
  FETODE_LIB=$lib timeout -k 10 200 python tools/diag/batch_sweep.py > gpurun_out/sweep_$n.log 2>&1
  rc=$?; echo "== $n sweep rc=$rc"; cat gpurun_out/sweep_$n.log | grep '^{'; [ $rc -le 1 ] || exit $rc
done
