#!/bin/bash
# bench flag sweep (dev tool): each configuration of CFGS (';'-separated flag sets) ROUNDS times
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${TAG:-flags}; mkdir -p $OUT
IFS=';' read -ra C <<< "$CFGS"
for r in $(seq ${ROUNDS:-2}); do
  i=0
  for cfg in "${C[@]}"; do
    i=$((i+1))
    timeout -k 10 120 python bench.py --no-cpu-baseline $cfg > $OUT/c$i.$r.json 2> $OUT/c$i.$r.err || { tail -5 $OUT/c$i.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c$i.$r.json')); print('[$cfg]', $r, round(d['value']/1e9,1), d['phases_ms'])"
  done
done
