#!/bin/bash
# The committed PMC profiles bench.py reads for roofline.traffic / roofline_decode_valu /
# roofline_count.traffic:
#   pmc_latest.json  the C2 step (46 Mbp), serial
#   pmc_c3.json      the C3 step (3.1 Gbp on one GPU), serial
#   pmc_count.json   the count kernel alone over the 3.1 Gbp genome (tools/count_hbm.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd)
PMC_NAME=pmc bash tools/pmc.sh || exit 1
python tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_latest.json 46000000 "bench.py --serial (C2)" > gpurun_out/pmc_summary.txt || exit 1
PMC_NAME=pmc_c3 PMC_ARGS="--workload c3 --steps 2 --warmup 1 --no-cpu-baseline --settle-ms 0" bash tools/pmc.sh || exit 1
python tools/pmc_summary.py gpurun_out/pmc_c3 gpurun_out/pmc_c3.json 3100000000 "bench.py --workload c3 (two streams)" > gpurun_out/pmc_c3_summary.txt || exit 1
OUT=$R/gpurun_out/pmc_count; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for p in "p1 SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD" "p2 FETCH_SIZE" "p3 WRITE_SIZE"; do
  set -- $p; name=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$name -o $name \
    -- python $R/tools/count_hbm.py --bases 3100000000 --no-sweep --reps 3 > $OUT/$name.json 2> $OUT/$name.err || exit 1
done
cd $R && python tools/pmc_summary.py gpurun_out/pmc_count gpurun_out/pmc_count.json 3099983872 "tools/count_hbm.py (count kernel alone)" > gpurun_out/pmc_count_summary.txt || exit 1
cut -c1-240 gpurun_out/pmc_summary.txt gpurun_out/pmc_c3_summary.txt gpurun_out/pmc_count_summary.txt
