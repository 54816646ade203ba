#!/bin/bash
# Round 4: the C2 step's training / decode CU split with the E-step's lane-private rows at
# every size (build/abl/libcpg_rep0.so) against the working tree (L1 rows at 702 chunks).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04_cus}; mkdir -p $OUT
L=$R/cpgisland_amd/libcpg.so; V=$R/build/abl/libcpg_rep0.so
b() {   # name lib cus
  CPG_LIB_OVERRIDE=$2 timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 --train-cus $3 --c3-steps 0 --no-cpu-baseline --cold-steps 0 > $OUT/$1.json 2> $OUT/$1.err || { tail -5 $OUT/$1.err; return 1; }
  python3 -c "
import json; d=json.load(open('$OUT/$1.json'))
print('$1', round(d['value']/1e9,1), round(d['ms_per_step'],4), d['phases_ms'])"
}
for r in 1 2; do
  for c in 176 192 208; do b base_${c}_$r $L $c || exit 1; b rep_${c}_$r $V $c || exit 1; done
done
