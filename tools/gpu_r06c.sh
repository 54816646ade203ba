#!/bin/bash
# round 6: GPU tests of the tree (count rewrite), then count kernel / training pass A/B (tree,
# round 5, wave/grid variants) and the C2 bench A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${T:-r06c}
SKIP_BENCH=1 TAG=$T bash tools/gpu_check.sh || exit 1
TAG=${T}_cnt VARIANTS="r05 cw5 cg1k" ROUNDS=2 TOOL="tools/count_hbm.py --no-sweep --reps 20 --train" KEY=count_ms_median,train_pass_ms_median,identities_ok bash tools/ab_variants.sh || exit 1
TAG=${T}_bench VARIANTS=r05 ROUNDS=2 TOOL="tools/bench_variant.py --steps 400 --warmup 20 --no-cpu-baseline --c3-steps 0 --bw-iters 0 --cold-steps 0" KEY=value,ms_per_step bash tools/ab_variants.sh
