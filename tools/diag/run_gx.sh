#!/bin/bash
# MNIST head backward variants: MNIST GPU tests on the new library, then rocprofv3 kernel stats of
# tools/diag/mnist_prof.py per library; plus the forward output-write experiment (fwd_time.py)
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mnist.py > gpurun_out/gx_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gx_tests.log; [ $rc -eq 0 ] || exit 3
for v in new=libfetode.so old=libfetode_gx1.so; do
  n=${v%%=*}; lib=$PWD/fet-ode_amd/${v#*=}
  FETODE_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/gx_$n -o run --output-format csv -- python3 tools/diag/mnist_prof.py > gpurun_out/gx_$n.log 2>&1
  rc=$?; echo "== $n (rc=$rc)"; [ $rc -le 1 ] || exit $rc
  python tools/diag/kstats.py gpurun_out/gx_$n 5
done

