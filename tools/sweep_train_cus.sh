mkdir -p gpurun_out/sweep
for r in 1 2; do for tc in ${TCS:-192 208 224 240}; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --train-cus $tc > gpurun_out/sweep/tc${tc}_$r.json 2> gpurun_out/sweep/tc${tc}_$r.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/sweep/tc${tc}_$r.json')); print($tc, $r, round(d['value']/1e9,1), d['phases_ms'])"
done; done
