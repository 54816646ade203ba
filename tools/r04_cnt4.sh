#!/bin/bash
# Round 4: count kernel with 32-bit moment counters ('+' work straight to LDS) — parity,
# 3.1 Gbp timing of the default and the batch / grid variants, one PMC pass of the default.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04_cnt4}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 200 \
  --timeout-method thread -k "count or train_pass or golden or estep" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
hbm() {
  CPG_LIB_OVERRIDE=$2 timeout -k 10 200 python -u tools/count_hbm.py --bases 3100000000 --no-sweep --reps 10 $3 > $OUT/$1.json 2> $OUT/$1.err || { tail -5 $OUT/$1.err; return 1; }
  echo "$1 $(python3 -c "import json; d=json.load(open('$OUT/$1.json')); print(round(d['count_ms_median'],4), round(d['count_GBps_median']), d.get('train_pass_ms_median'))")"
}
hbm default $R/cpgisland_amd/libcpg.so --train || exit 1
for v in ${VARIANTS:-r2g2048 r1g1024 r1g4096}; do hbm $v $R/build/abl/libcpg_$v.so || exit 1; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d $OUT/pmc/p1 -o p1 \
  -- python $R/tools/count_hbm.py --bases 3100000000 --no-sweep --reps 3 > /dev/null 2> $OUT/p1.err || { tail -3 $OUT/p1.err; exit 1; }
cd $R && python tools/pmc_summary.py $OUT/pmc > $OUT/pmc_summary.txt && cat $OUT/pmc_summary.txt
