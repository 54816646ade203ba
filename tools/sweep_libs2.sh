#!/bin/bash
# dev tool: 400-step bench of libcpg builds x training-CU counts ("name cus;name cus;..."), 2 rounds
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${TAG:-sl}; mkdir -p $OUT
IFS=";" read -ra CF <<< "$LCFGS"
for r in $(seq ${ROUNDS:-2}); do
for cfg in "${CF[@]}"; do
  set -- $cfg
  CPG_LIB_OVERRIDE=build/abl/libcpg_$1.so timeout -k 10 120 python bench.py --no-cpu-baseline --train-cus $2 > $OUT/$1_$2_$r.json 2> $OUT/$1_$2_$r.err || { tail -5 $OUT/$1_$2_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$1_$2_$r.json')); print('$1', $2, $r, round(d['value']/1e9,1), d['phases_ms'])"
done; done
