#!/bin/bash
# round 6: GPU tests of the tree (K4 walk as one batched stream), decode A/B against HEAD's
# K4 (k4old) at the C2 size, and the decode kernel statistics of both
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${T:-r06l}
SKIP_BENCH=1 TAG=$T bash tools/gpu_check.sh || exit 1
TAG=${T}_ab VARIANTS="k4old" ROUNDS=3 TOOL="tools/decode_c3.py" KEY=ms_median BASES=46000000 REPS=41 bash tools/ab_variants.sh || exit 1
TAG=${T}_prof PKGS="k4old" bash tools/prof_decode.sh
mkdir -p gpurun_out/${T}_diag && CPG_DEV_PKG=build/abl/pkg_k4diag timeout -k 10 100 python -u tools/k4diag.py > gpurun_out/${T}_diag/new.txt 2>&1
