#!/bin/bash
# training-pass changes: the training tests (tree), then the pass alone at 46 Mbp and 3.1 Gbp
# and the driver's bench command, tree against the variants
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-train_ab}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "${PYTEST_K:-estep or train or count or c3 or baum or stream or halo or cli or golden}" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
echo "tests: $(tail -1 $OUT/pytest.log)"
VARIANTS="$VARIANTS" TAG=${TAG:-train_ab}_46m TOOL="tools/count_hbm.py --bases 46000000 --train --no-sweep --reps 40" KEY=train_pass_ms_median bash tools/ab_variants.sh || exit 1
VARIANTS="$VARIANTS" TAG=${TAG:-train_ab}_3g TOOL="tools/count_hbm.py --train --no-sweep --reps 12" KEY=train_pass_ms_median bash tools/ab_variants.sh || exit 1
VARIANTS="$VARIANTS" TAG=${TAG:-train_ab}_bench TOOL="bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --bw-iters 0 --cold-steps 0" KEY=value,ms_per_step bash tools/ab_variants.sh
