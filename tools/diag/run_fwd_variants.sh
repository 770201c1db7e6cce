#!/bin/bash
# forward variants: robust-subset parity at the bench config, then kernel times of the training
# loop (fused4 with tape + reverse sweep) under rocprofv3; VARIANTS="name=libpath ..."
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
for v in $VARIANTS; do
  n=${v%%=*}; lib=$PWD/${v#*=}
  FETODE_LIB=$lib timeout -k 10 300 python tools/diag/robust_check.py > gpurun_out/rob_$n.log 2>&1
  rc=$?; echo "== $n robust rc=$rc: $(tail -1 gpurun_out/rob_$n.log | cut -c1-400)"; [ $rc -le 1 ] || exit $rc
done
for v in $VARIANTS; do
  n=${v%%=*}; lib=$PWD/${v#*=}
  FETODE_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/fv_$n -o run --output-format csv -- python3 tools/diag/train_iter.py > gpurun_out/fv_$n.log 2>&1
  rc=$?; echo "== $n (rc=$rc)"; [ $rc -le 1 ] || exit $rc
  python tools/diag/kstats.py gpurun_out/fv_$n 2
done
