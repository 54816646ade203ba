#!/bin/bash
# A/B of variant builds (tools/build_variant.sh) on one timing tool, alternating with the tree's
# own build: VARIANTS="d22 d33" TOOL="tools/count_hbm.py --train --no-sweep --reps 12" KEY=train_pass_ms_median
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-ab}; mkdir -p $OUT
for round in $(seq 1 ${ROUNDS:-2}); do
  for v in base $VARIANTS; do
    if [ $v = base ]; then P=""; else P=$R/build/abl/pkg_$v; fi
    CPG_DEV_PKG=$P timeout -k 10 200 python -u $TOOL > $OUT/${v}_$round.json 2> $OUT/${v}_$round.err || { tail -5 $OUT/${v}_$round.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$OUT/${v}_$round.json').read().strip().splitlines()[-1])
print('$v', $round, {k: round(d[k], 4) if isinstance(d[k], float) else d[k] for k in '$KEY'.split(',') if k in d})"
  done
done
