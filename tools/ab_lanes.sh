#!/bin/bash
# A/B of the C2 step's pipelining options (bench.py flags), alternating runs on one box
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${TAG:-ab_lanes}; mkdir -p $OUT
for r in 1 2; do
  for v in "base:" "dl2:--decode-lanes 2" "ln2:--lanes 2" "ds2:--decode-split 2"; do
    n=${v%%:*}; f=${v#*:}
    timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --c3-steps 0 --cold-steps 0 $f \
      > $OUT/${n}_$r.json 2> $OUT/${n}_$r.err || { tail -5 $OUT/${n}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/${n}_$r.json').read().strip().splitlines()[-1])
print('$n', $r, round(d['value']/1e9,1), d['ms_per_step'], d.get('fingerprint',{}).get('oracle_match'))"
  done
done
