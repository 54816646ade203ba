#!/bin/bash
# the C2 step with two pipeline lanes (the default): training CU-mask and decode-split sweep
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${TAG:-ab_lanes3}; mkdir -p $OUT
for r in 1 2; do
  for v in ${VARS:-"cus192:" "cus224:--train-cus 224"}; do
    n=${v%%:*}; f=${v#*:}
    timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --c3-steps 0 --cold-steps 0 $f \
      > $OUT/${n}_$r.json 2> $OUT/${n}_$r.err || { tail -5 $OUT/${n}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/${n}_$r.json').read().strip().splitlines()[-1])
print('$n', $r, round(d['value']/1e9,1), d['ms_per_step'], d.get('fingerprint',{}).get('oracle_match'), d['roofline']['aggregate_achieved'])"
  done
done
