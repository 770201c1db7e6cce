#!/bin/bash
# Reverse-sweep timing of library variants: VARIANTS="name=libpath[,ENV=val...] ..." -> the
# training loop (tools/diag/train_iter.py) under rocprofv3 per variant, top kernels printed.
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
for v in $VARIANTS; do
  name=${v%%=*}; rest=${v#*=}; lib=${rest%%,*}; envs=""
  [ "$rest" != "$lib" ] && envs=$(echo "${rest#*,}" | tr ',' ' ')
  env FETODE_LIB=$PWD/$lib $envs timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/var_$name -o run \
    --output-format csv -- python3 tools/diag/train_iter.py > gpurun_out/var_$name.log 2>&1
  rc=$?; echo "== $name (rc=$rc)"; [ $rc -le 1 ] || exit $rc
  python tools/diag/kstats.py gpurun_out/var_$name 2
done
