#!/bin/bash
# Round 4: the C3 workload (3.1 Gbp on one GPU) across training CU masks and decode priority,
# then the default bench line (C2 headline + C3 leg + count roofline).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04_c3sweep}; mkdir -p $OUT
for cfg in ${CFGS:-"0 1" "192 1" "224 1" "240 1" "0 0" "224 0"}; do
  set -- $cfg
  n=c3_cus$1_prio$2
  timeout -k 10 300 python -u bench.py --workload c3 --steps 30 --warmup 3 --c3-train-cus $1 --prio $2 > $OUT/$n.json 2> $OUT/$n.err || { tail -5 $OUT/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', round(d['value']/1e9,1), round(d['ms_per_step'],3), d['phases_ms'])"
done
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -5 $OUT/bench_driver.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench_driver.json'))
print('driver', round(d['value']/1e9,1), d['ms_per_step'], d['phases_ms'])
print('c3', {k: d['c3_single_gpu'][k] for k in ('value','ms_per_step','phases_ms')})
print('count', d['roofline_count'])
print('decode', d['roofline_decode'], d['roofline_decode_valu'])"
