#!/bin/bash
# Round 4: the C3 workload (3.1 Gbp on this GPU) across training-stream CU masks and decode
# priority, with the E-step's lane-private rows (>= 2,048 chunks).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${TAG:-r04_c3cus}; mkdir -p $OUT
for cfg in "0 1" "0 0" "224 1" "240 1" "192 1" "0 1"; do
  set -- $cfg
  n=c3_cus$1_prio$2
  timeout -k 10 300 python -u bench.py --workload c3 --steps 30 --warmup 3 --c3-train-cus $1 --prio $2 --no-cpu-baseline > $OUT/$n.json 2> $OUT/$n.err || { tail -5 $OUT/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', round(d['value']/1e9,1), round(d['ms_per_step'],3), d['phases_ms'])"
done
