#!/bin/bash
# two-stream step with and without a high-priority decode stream (3 runs each, interleaved)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/prio; mkdir -p $OUT
for i in 1 2 3; do for p in 0 1; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 50 --prio $p > $OUT/b_${p}_$i.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$OUT/b_${p}_$i.json')); print('prio', $p, round(d['value']/1e9,2), d['phases_ms'])"
done; done
