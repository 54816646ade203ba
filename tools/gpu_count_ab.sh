#!/bin/bash
# count-kernel variants: parity (count tests) for the tree and each variant, then count_hbm A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-count_ab}; mkdir -p $OUT
for v in base $VARIANTS; do
  if [ $v = base ]; then P=""; else P=$R/build/abl/pkg_$v; fi
  CPG_DEV_PKG=$P timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py -m gpu -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread -k "count or train or stream" > $OUT/pytest_$v.log 2>&1 || { tail -30 $OUT/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/pytest_$v.log)"
done
VARIANTS="$VARIANTS" TAG=${TAG:-count_ab} TOOL="tools/count_hbm.py --reps 20 ${SWEEP:---no-sweep}" KEY=count_ms_median,count_GBps_median,readsweep_GBps bash tools/ab_variants.sh
