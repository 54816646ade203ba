#!/bin/bash
# round 6: GPU tests of the tree (K2's segment work inside K3's launch), decode kernel
# statistics of the tree and HEAD (k4old), decode A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${T:-r06r}
SKIP_BENCH=1 TAG=$T bash tools/gpu_check.sh || exit 1
TAG=${T}_prof PKGS="k4old" bash tools/prof_decode.sh > gpurun_out/${T}_prof.txt 2>&1 || exit 1
TAG=${T}_ab VARIANTS="k4old" ROUNDS=3 TOOL="tools/decode_c3.py" KEY=ms_median BASES=46000000 REPS=41 bash tools/ab_variants.sh
