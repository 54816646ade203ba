#!/bin/bash
# dev tool: the fused forward+traceback (CPG_VIT_FUSE57=1) against the default at several
# training-CU counts, 400-step bench, alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/fz; mkdir -p $OUT
for r in 1 2; do
IFS=";" read -ra CF <<< "${FCFGS:-0 192;1 192;1 208;1 224}"
for cfg in "${CF[@]}"; do
  set -- $cfg
  if [ $1 = 1 ]; then export CPG_VIT_FUSE57=1; else unset CPG_VIT_FUSE57; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline --train-cus $2 > $OUT/f$1_$2_$r.json 2> $OUT/f$1_$2_$r.err || { tail -5 $OUT/f$1_$2_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/f$1_$2_$r.json')); print('fuse57=$1', $2, $r, round(d['value']/1e9,1), d['phases_ms'])"
done; done
