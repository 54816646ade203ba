#!/bin/bash
# round 6: GPU tests of the tree ('+' moments in registers), count A/B (round 5, lane-0 word
# loads), K4 ablation profiles (timing only)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${T:-r06k}
SKIP_BENCH=1 TAG=$T bash tools/gpu_check.sh || exit 1
TAG=${T}_cnt VARIANTS="r05 l0" ROUNDS=2 TOOL="tools/count_hbm.py --no-sweep --reps 20" KEY=count_ms_median,identities_ok bash tools/ab_variants.sh || exit 1
IGNORE_STATUS=1 TAG=${T}_prof PKGS="k4nc k4ea" bash tools/prof_decode.sh
