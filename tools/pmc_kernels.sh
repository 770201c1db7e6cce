#!/bin/bash
# rocprofv3 PMC passes (each pass its own run, --kernel-trace only beside --pmc) over
# tools/diag/prof_targets.py; CSVs under gpurun_out/pmc_<tag>_<pass>.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
TAG=${TAG:-r04}
timeout -s KILL 60 rocprofv3 -L > $O/rocprof_counters.txt 2>&1 || true
pass() { local name=$1; shift; timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $O/pmc_${TAG}_$name -o run --output-format csv -- python3 tools/diag/prof_targets.py ${PROF_WHICH:-all} > $O/pmc_${TAG}_$name.log 2>&1; echo "pass $name rc=$?"; }
[ -z "$ONLY_ISSUE" ] && pass a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
[ -z "$ONLY_ISSUE" ] && pass b SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS
[ -z "$ONLY_ISSUE" ] && pass c SQ_INSTS_MFMA SQ_ACTIVE_INST_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT
# issue accounting: VALU-active quad-cycles per SIMD against the elapsed cycles
[ -n "$ISSUE" ] && pass v SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
# MFMA utilisation (north_star: "MFMA utilisation against chip peak") and the wait shares
[ -n "$ISSUE" ] && pass m SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MFMA GRBM_GUI_ACTIVE
[ -n "$ISSUE" ] && pass w SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
