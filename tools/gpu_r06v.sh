#!/bin/bash
# round 6: GPU tests of the tree (relaxed window rule), decode kernel statistics of the tree and
# of the strict rule (k4old), decode A/B, K4 phase stamps
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${T:-r06v}
SKIP_BENCH=1 TAG=$T bash tools/gpu_check.sh || exit 1
TAG=${T}_prof PKGS="k4old" bash tools/prof_decode.sh > gpurun_out/${T}_prof.txt 2>&1 || exit 1
TAG=${T}_ab VARIANTS="k4old" ROUNDS=4 TOOL="tools/decode_c3.py" KEY=ms_median BASES=46000000 REPS=41 bash tools/ab_variants.sh || exit 1
mkdir -p gpurun_out/${T}_diag && CPG_DEV_PKG=build/abl/pkg_k4diag timeout -k 10 100 python -u tools/k4diag.py > gpurun_out/${T}_diag/k4.txt 2>&1
