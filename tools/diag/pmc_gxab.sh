#!/bin/bash
# PMC passes over the MNIST training step (tools/diag/mnist_prof.py), each pass its own run
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
pass() { local name=$1; shift; timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $O/pmc_gx_$name -o run --output-format csv -- python3 tools/diag/mnist_prof.py > $O/pmc_gx_$name.log 2>&1; echo "pass $name rc=$?"; }
pass a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
pass b SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD
