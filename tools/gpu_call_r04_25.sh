cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp SECT=1 FUSED_ONLY=1 N=2
pass() { local name=$1; shift; timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $O/pmc_fn_$name -o run --output-format csv -- python3 tools/diag/fieldn_train_time.py > $O/pmc_fn_$name.log 2>&1; local rc=$?; echo "pass $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
pass a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
pass b SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS
pass c SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT
