#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
NS=2 bash tools/gpu_rehearse_dist.sh || exit $?
for cfg in "256 1e-3 1e-4" "256 1e-7 1e-9"; do
  set -- $cfg
  B=$1 RTOL=$2 ATOL=$3 timeout -k 10 240 python -u tools/diag/ett_dopri5.py > $O/ett_dp5_$1_$2.log 2>&1
  rc=$?; echo "ett dopri5 $cfg rc=$rc"; grep "B=" $O/ett_dp5_$1_$2.log; [ $rc -eq 0 ] || exit $rc
done
