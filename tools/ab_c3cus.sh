#!/bin/bash
# the C3 workload on one GPU: training-stream CU mask sweep, alternating runs
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${TAG:-ab_c3cus}; mkdir -p $OUT
for r in 1 2; do
  for c in ${CUS:-0 240 224}; do
    timeout -k 10 300 python bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline --c3-train-cus $c \
      > $OUT/c${c}_$r.json 2> $OUT/c${c}_$r.err || { tail -5 $OUT/c${c}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/c${c}_$r.json').read().strip().splitlines()[-1])
print('c$c', $r, round(d['value']/1e9,1), round(d['ms_per_step'],3), d.get('fingerprint',{}).get('oracle_match'))"
  done
done
