#!/bin/bash
# bench.py at several CU splits between the training and decode streams (dev measurement).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/sweep
for c in ${CUS:-160 192 208 224 240}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS_N:-40} --train-cus $c ${EXTRA:-} \
      > gpurun_out/sweep/cus_$c.json 2> gpurun_out/sweep/cus_$c.err || { echo "cus $c failed"; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sweep/cus_$c.json'));print($c, round(d['value']/1e9,1), d['phases_ms'])"
done
