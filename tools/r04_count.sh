#!/bin/bash
# Round 4: the labelled-count kernel on an HBM-resident 3.1 Gbp genome — event timing against a
# plain read sweep, the rocprofv3 kernel statistics of the same command, and a FETCH_SIZE /
# WRITE_SIZE / SQ pass (each counter group its own run).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04_count}; mkdir -p $OUT
B=${BASES:-3100000000}
timeout -k 10 300 python -u tools/count_hbm.py --bases $B ${TRAIN_ARG:---train} > $OUT/count_hbm.json 2> $OUT/count_hbm.err || { tail -5 $OUT/count_hbm.err; exit 1; }
cat $OUT/count_hbm.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o prof \
  -- python $R/tools/count_hbm.py --bases $B --no-sweep --reps 10 > $OUT/prof.json 2> $OUT/prof.err || { tail -5 $OUT/prof.err; exit 1; }
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc/p2 -o p2 \
  -- python $R/tools/count_hbm.py --bases $B --no-sweep --reps 3 > /dev/null 2> $OUT/p2.err || exit 1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc/p3 -o p3 \
  -- python $R/tools/count_hbm.py --bases $B --no-sweep --reps 3 > /dev/null 2> $OUT/p3.err || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d $OUT/pmc/p1 -o p1 \
  -- python $R/tools/count_hbm.py --bases $B --no-sweep --reps 3 > /dev/null 2> $OUT/p1.err || exit 1
cd $R && python tools/pmc_summary.py $OUT/pmc > $OUT/pmc_summary.txt && cat $OUT/pmc_summary.txt
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \; ; head -5 $OUT/kernel_stats.csv
