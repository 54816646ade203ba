#!/bin/bash
# Round 4: E-step two-step rows from a lane-private LDS copy (conflict-free; 147.5 KB of LDS per
# workgroup), build/abl/libcpg_rep0.so (used at every chunk count) — E-step
# parity with the variant, the training pass alone, then the driver's bench command (C2 +
# C3 leg), alternating with the working tree.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04_rep}; mkdir -p $OUT
L=$R/cpgisland_amd/libcpg.so; V=$R/build/abl/libcpg_rep0.so
CPG_LIB_OVERRIDE=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_contigs.py tests/test_gpu_c3.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "(estep or train or golden or count or c3 or baum) and not timeout" > $OUT/pytest_rep.log 2>&1 || { tail -30 $OUT/pytest_rep.log; exit 1; }
tail -1 $OUT/pytest_rep.log
hbm() {   # name lib bases
  CPG_LIB_OVERRIDE=$2 timeout -k 10 200 python -u tools/count_hbm.py --bases $3 --no-sweep --reps 10 --train > $OUT/$1.json 2> $OUT/$1.err || { tail -5 $OUT/$1.err; return 1; }
  echo "$1 train_pass_ms $(python3 -c "import json; d=json.load(open('$OUT/$1.json')); print(d.get('train_pass_ms_median'))")"
}
hbm t_new46 $L 46000000 || exit 1; hbm t_rep46 $V 46000000 || exit 1
hbm t_new3g $L 3100000000 || exit 1; hbm t_rep3g $V 3100000000 || exit 1
b() {   # name lib
  CPG_LIB_OVERRIDE=$2 timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/$1.json 2> $OUT/$1.err || { tail -5 $OUT/$1.err; return 1; }
  python3 -c "
import json; d=json.load(open('$OUT/$1.json'))
print('$1', round(d['value']/1e9,1), round(d['ms_per_step'],4), d['phases_ms'], 'c3', round(d['c3_single_gpu']['value']/1e9,1), round(d['c3_single_gpu']['ms_per_step'],3))"
}
for i in 1 2; do b new_$i $L || exit 1; b rep_$i $V || exit 1; done
