#!/bin/bash
# round 6: GPU tests of the tree (K2's segment work inside K3's launch, K4 walk as one flat
# stream), decode kernel statistics of the tree, HEAD (k4old) and K4 walk variants
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${T:-r06q}
SKIP_BENCH=1 TAG=$T bash tools/gpu_check.sh || exit 1
timeout -k 5 60 ./tools/ubench_walk > gpurun_out/${T}_ubench_walk.jsonl 2>&1
IGNORE_STATUS=1 TAG=${T}_prof PKGS="k4old nowalk nosb ahead2" bash tools/prof_decode.sh > gpurun_out/${T}_prof.txt 2>&1
