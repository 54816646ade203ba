#!/bin/bash
# round 6: tree check (tests, smoke, driver bench) + count / training pass / C2 bench A/B
# against round 5's sources
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${T:-r06i}
TAG=$T bash tools/gpu_check.sh || exit 1
TAG=${T}_cnt VARIANTS="r05" ROUNDS=2 TOOL="tools/count_hbm.py --no-sweep --reps 20 --train" KEY=count_ms_median,train_pass_ms_median,identities_ok bash tools/ab_variants.sh || exit 1
TAG=${T}_bench VARIANTS=r05 ROUNDS=3 TOOL="tools/bench_variant.py --steps 400 --warmup 20 --no-cpu-baseline --c3-steps 0 --bw-iters 0 --cold-steps 0" KEY=value,ms_per_step,phases_ms bash tools/ab_variants.sh
TAG=${T}_prof PKGS=r05 bash tools/prof_decode.sh
