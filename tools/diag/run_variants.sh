#!/bin/bash
cd "$(dirname "$0")/../.."
for v in ${VARIANTS:-4 5}; do
  FETODE_FUSED_LPT=$v timeout -k 10 300 python tools/diag/variants.py || exit 3
done
if [ -f fet-ode_amd/libfetode_w4.so ]; then
  FETODE_FUSED_LPT=5 FETODE_LIB=$PWD/fet-ode_amd/libfetode_w4.so timeout -k 10 300 python tools/diag/variants.py || exit 3
fi
