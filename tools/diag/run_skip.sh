#!/bin/bash
# Phase-cost attribution of the reverse sweep: fixed_bwd time with each FETODE_EXP_SKIP variant
# (built by: make OBJDIR=build_x$n OUT=../libfetode_x$n.so EXTRA="-DFETODE_DIAG -DFETODE_EXP_SKIP=$n").
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
for n in 0 ${SKIPS:-1 2 4 8 16}; do
  lib=$PWD/fet-ode_amd/libfetode.so; [ $n = 0 ] || lib=$PWD/fet-ode_amd/libfetode_x$n.so
  FETODE_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/skip_$n -o run --output-format csv -- python3 tools/diag/train_iter.py > gpurun_out/skip_$n.log 2>&1
  echo "skip=$n: $(python tools/diag/kstats.py gpurun_out/skip_$n 1)"
done
