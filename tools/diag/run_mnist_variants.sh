#!/bin/bash
# MNIST kernels of library variants: VARIANTS="name=libpath ..." -> MNIST GPU tests + rocprof
# stats of tools/diag/mnist_prof.py per variant.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
for v in $VARIANTS; do
  name=${v%%=*}; lib=$PWD/${v#*=}
  FETODE_LIB=$lib timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mnist.py > gpurun_out/mn_$name.log 2>&1
  rc=$?; echo "== $name tests rc=$rc: $(tail -1 gpurun_out/mn_$name.log)"; [ $rc -le 1 ] || exit $rc
  FETODE_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/mnp_$name -o run --output-format csv -- python3 tools/diag/mnist_prof.py > gpurun_out/mnp_$name.log 2>&1
  rc=$?; [ $rc -le 1 ] || exit $rc
  python tools/diag/kstats.py gpurun_out/mnp_$name 6 | grep -E "wide_fwd|kuramoto"
done
