#!/bin/bash
# Round 4: the rewritten labelled-count kernel and the E-step's 64-lane row walk — parity tests,
# then the HBM-resident 3.1 Gbp timing for the default build and the batch / grid variants
# (build/abl), the E-step alone against the round-3 build (build/abl/libcpg_base.so),
# rocprofv3 kernel statistics and an SQ / FETCH_SIZE pass of the default count kernel.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04_count2}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 200 \
  --timeout-method thread -k "count or train_pass or golden or estep" > $OUT/pytest_count.log 2>&1 || { tail -30 $OUT/pytest_count.log; exit 1; }
tail -2 $OUT/pytest_count.log
B=${BASES:-3100000000}
timeout -k 10 300 python -u tools/count_hbm.py --bases $B --train > $OUT/count_hbm.json 2> $OUT/count_hbm.err || { tail -5 $OUT/count_hbm.err; exit 1; }
cat $OUT/count_hbm.json
for v in ${VARIANTS:-base b2g1024 b3g1024 b4g512 b4g2048}; do
  CPG_LIB_OVERRIDE=$R/build/abl/libcpg_$v.so timeout -k 10 200 python -u tools/count_hbm.py --bases $B --no-sweep --reps 10 --train > $OUT/count_$v.json 2> $OUT/count_$v.err || { tail -5 $OUT/count_$v.err; exit 1; }
  echo "$v $(cat $OUT/count_$v.json)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o prof \
  -- python $R/tools/count_hbm.py --bases $B --no-sweep --reps 10 > $OUT/prof.json 2> $OUT/prof.err || { tail -5 $OUT/prof.err; exit 1; }
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc/p2 -o p2 \
  -- python $R/tools/count_hbm.py --bases $B --no-sweep --reps 3 > /dev/null 2> $OUT/p2.err || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d $OUT/pmc/p1 -o p1 \
  -- python $R/tools/count_hbm.py --bases $B --no-sweep --reps 3 > /dev/null 2> $OUT/p1.err || exit 1
cd $R && python tools/pmc_summary.py $OUT/pmc > $OUT/pmc_summary.txt && cat $OUT/pmc_summary.txt
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \; ; head -3 $OUT/kernel_stats.csv
