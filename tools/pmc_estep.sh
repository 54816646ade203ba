# PMC passes over the E-step alone (tools/estep_ablate.py), plus the counter list of the box
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/pmce; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$name -o $name \
    -- python3 $R/tools/estep_ablate.py > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU && \
run p2 SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM && \
run p3 GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM
