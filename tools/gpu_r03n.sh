#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
for v in "" acc2 unr both; do
  if [ -n "$v" ]; then L=$PWD/fet-ode_amd/libfetode_$v.so; else L=$PWD/fet-ode_amd/libfetode.so; fi
  FETODE_LIB=$L timeout -k 10 120 python -u tools/diag/mnist_head_time.py 2>&1 | grep head || exit 1
done
timeout -k 10 300 python -u tools/diag/train_graph2.py > $O/r03n_graph.log 2>&1; echo "graph rc=$?"; grep -v amdgpu $O/r03n_graph.log | tail -8
