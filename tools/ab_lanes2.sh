#!/bin/bash
# A/B of pipeline lanes at the driver's step counts (20 timed, 5 warm-up) and at 200 steps
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${TAG:-ab_lanes2}; mkdir -p $OUT
for r in 1 2; do
  for v in "l1s20:--steps 20 --warmup 5" "l2s20:--lanes 2 --steps 20 --warmup 5" "l3s20:--lanes 3 --steps 20 --warmup 5" "l4s20:--lanes 4 --steps 20 --warmup 5" "l3:--lanes 3 --steps 200 --warmup 20" "l4:--lanes 4 --steps 200 --warmup 20" "l2dl2:--lanes 2 --decode-lanes 2 --steps 200 --warmup 20"; do
    n=${v%%:*}; f=${v#*:}
    timeout -k 10 200 python bench.py --no-cpu-baseline --c3-steps 0 --cold-steps 0 $f \
      > $OUT/${n}_$r.json 2> $OUT/${n}_$r.err || { tail -5 $OUT/${n}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/${n}_$r.json').read().strip().splitlines()[-1])
print('$n', $r, round(d['value']/1e9,1), d['ms_per_step'], d.get('fingerprint',{}).get('oracle_match'))"
  done
done
