#!/bin/bash
# round 6: GPU tests of the tree (K4 walk with its constants by v_readlane, relaxed window rule), decode kernel
# statistics of the tree of the previous K4 (k4old) and of the strict window rule (strict), decode A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${T:-r06u}
SKIP_BENCH=1 TAG=$T bash tools/gpu_check.sh || exit 1
TAG=${T}_prof PKGS="k4old strict" bash tools/prof_decode.sh > gpurun_out/${T}_prof.txt 2>&1 || exit 1
TAG=${T}_ab VARIANTS="k4old strict" ROUNDS=3 TOOL="tools/decode_c3.py" KEY=ms_median BASES=46000000 REPS=41 bash tools/ab_variants.sh
mkdir -p gpurun_out/${T}_diag && CPG_DEV_PKG=build/abl/pkg_k4diag timeout -k 10 100 python -u tools/k4diag.py > gpurun_out/${T}_diag/k4.txt 2>&1
