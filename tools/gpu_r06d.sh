#!/bin/bash
# round 6: count kernel ablations (no '+' work / no counting / no uniform word loads), C2 bench
# A/B against round 5, and a sweep of the training stream's CU count on the tree
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${T:-r06d}
TAG=${T}_cnt VARIANTS="nplus nocnt nowp" ROUNDS=2 TOOL="tools/count_hbm.py --no-sweep --reps 20" KEY=count_ms_median bash tools/ab_variants.sh || exit 1
TAG=${T}_bench VARIANTS=r05 ROUNDS=2 TOOL="tools/bench_variant.py --steps 400 --warmup 20 --no-cpu-baseline --c3-steps 0 --bw-iters 0 --cold-steps 0" KEY=value,ms_per_step bash tools/ab_variants.sh || exit 1
OUT=gpurun_out/${T}_cus; mkdir -p $OUT
for cus in 160 176 192 208; do
  timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-cpu-baseline --c3-steps 0 --bw-iters 0 --cold-steps 0 --train-cus $cus > $OUT/cus_$cus.json 2> $OUT/cus_$cus.err || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/cus_$cus.json').read().strip().splitlines()[-1]); print('cus', $cus, round(d['value']/1e9,1), d['phases_ms'])"
done
