#!/bin/bash
# round 6: GPU tests of the tree (K4 in < 40 KB of LDS), C3 A/B against the previous K4
# (k4old), C2 A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${T:-r06w}
SKIP_BENCH=1 TAG=$T bash tools/gpu_check.sh || exit 1
TAG=${T}_c3 VARIANTS="k4old" ROUNDS=2 TOOL="tools/bench_variant.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline" KEY=value,ms_per_step bash tools/ab_variants.sh || exit 1
TAG=${T}_c2 VARIANTS="k4old" ROUNDS=2 TOOL="tools/bench_variant.py --steps 200 --warmup 20 --no-cpu-baseline --c3-steps 0 --cold-steps 0" KEY=value,ms_per_step bash tools/ab_variants.sh || exit 1
BASES=3100000000 REPS=3 TAG=${T}_prof PKGS="k4old" bash tools/prof_decode.sh > gpurun_out/${T}_prof.txt 2>&1
