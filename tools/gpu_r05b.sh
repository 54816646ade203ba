#!/bin/bash
# E-step round-5 batch: tree tests, rn4 variant parity, then A/B of tree / nosep / rn4 / old
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r05b}; mkdir -p $OUT
CPG_DEV_PKG=$R/build/abl/pkg_rn4 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread -k "estep or train or baum or cli or golden or general or contig" > $OUT/pytest_rn4.log 2>&1 || { tail -30 $OUT/pytest_rn4.log; exit 1; }
echo "rn4 tests: $(tail -1 $OUT/pytest_rn4.log)"
TAG=${TAG:-r05b} VARIANTS="$VARIANTS" bash tools/gpu_train_ab.sh
