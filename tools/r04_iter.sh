#!/bin/bash
# Round 4 iteration: parity of the count / E-step paths, the count kernel at 3.1 Gbp for the
# default build and the batch / grid variants, the training pass at 46 Mbp and 3.1 Gbp against
# the round-3 build (build/abl/libcpg_base.so), E-step phase stamps (new vs base).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04_iter}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 200 \
  --timeout-method thread -k "count or train_pass or golden or estep" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
hbm() {   # name lib bases extra
  CPG_LIB_OVERRIDE=$2 timeout -k 10 200 python -u tools/count_hbm.py --bases $3 --no-sweep --reps 10 $4 > $OUT/$1.json 2> $OUT/$1.err || { tail -5 $OUT/$1.err; return 1; }
  echo "$1 $(python3 -c "import json; d=json.load(open('$OUT/$1.json')); print(round(d['count_ms_median'],4), round(d['count_GBps_median']), d.get('train_pass_ms_median'))")"
}
L=$R/cpgisland_amd/libcpg.so
hbm default $L 3100000000 --train || exit 1
hbm base $R/build/abl/libcpg_base.so 3100000000 --train || exit 1
hbm default46 $L 46000000 --train || exit 1
hbm base46 $R/build/abl/libcpg_base.so 46000000 --train || exit 1
hbm default46b $L 46000000 --train || exit 1
hbm base46b $R/build/abl/libcpg_base.so 46000000 --train || exit 1
for v in ${VARIANTS:-n2g1024 n2g2048 n3g512 n4g1024}; do hbm $v $R/build/abl/libcpg_$v.so 3100000000 || exit 1; done
for v in stamp stampbase; do
  CPG_LIB_OVERRIDE=$R/build/abl/libcpg_$v.so timeout -k 10 120 python -u tools/stamp_estep.py > $OUT/$v.txt 2>&1 || { tail -5 $OUT/$v.txt; exit 1; }
  echo "== $v"; cat $OUT/$v.txt
done
