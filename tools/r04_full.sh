#!/bin/bash
# Round 4 GPU session part 1: the whole -m gpu suite, smoke, the driver's bench command (C2
# headline + C3 leg + count roofline), then the C3 workload across training CU masks.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${TAG:-r04_full}; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -5 $OUT/bench_driver.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench_driver.json'))
print('driver', round(d['value']/1e9,1), d['ms_per_step'], d['phases_ms'])
print('c3', {k: d['c3_single_gpu'][k] for k in ('value','ms_per_step','phases_ms')})
print('count', d['roofline_count'])
print('decode', d['roofline_decode'], d['roofline_decode_valu'])
print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
for cfg in ${CFGS:-"192 1" "224 1" "240 1" "0 0"}; do
  set -- $cfg
  n=c3_cus$1_prio$2
  timeout -k 10 300 python -u bench.py --workload c3 --steps 30 --warmup 3 --c3-train-cus $1 --prio $2 > $OUT/$n.json 2> $OUT/$n.err || { tail -5 $OUT/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', round(d['value']/1e9,1), round(d['ms_per_step'],3), d['phases_ms'])"
done
