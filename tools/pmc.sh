#!/bin/bash
# PMC counter passes over a short serial bench (each pass its own rocprofv3 run; no trace
# domains).  FETCH_SIZE on gfx950 counts half the bytes of 16-B/lane streaming reads
# (MI355X_MICROARCH.md §HBM): tools/pmc_summary.py reports it doubled.
#   PMC_NAME  output directory under gpurun_out/ (default pmc)
#   PMC_ARGS  bench.py arguments (default: the C2 step, serial)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${PMC_NAME:-pmc}; mkdir -p $OUT
ARGS=${PMC_ARGS:---steps 2 --warmup 1 --no-cpu-baseline --serial --c3-steps 0 --cold-steps 0 --settle-ms 0}
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$name -o $name \
    -- python $R/bench.py $ARGS > $OUT/$name.json 2> $OUT/$name.err
  local rc=$?; echo "$name rc=$rc"; return $rc
}
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU && \
run p2 FETCH_SIZE && run p3 WRITE_SIZE && \
run p4 GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES
