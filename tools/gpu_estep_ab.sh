#!/bin/bash
# E-step changes: parity of the training-pass tests (tree), then the training pass alone at
# 3.1 Gbp and the C3 bench leg, tree against the variants (tools/ab_variants.sh)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-estep_ab}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_halo.py -m gpu -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread -k "${PYTEST_K:-estep or train or c3 or baum or stream or halo or decode or island}" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
echo "tests: $(tail -1 $OUT/pytest.log)"
VARIANTS="$VARIANTS" TAG=${TAG:-estep_ab} TOOL="tools/count_hbm.py --train --no-sweep --reps 12" KEY=train_pass_ms_median bash tools/ab_variants.sh || exit 1
VARIANTS="$VARIANTS" TAG=${TAG:-estep_ab}_dec TOOL="tools/decode_c3.py" KEY=ms_median bash tools/ab_variants.sh || exit 1
VARIANTS="$VARIANTS" TAG=${TAG:-estep_ab}_c3 TOOL="bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline --bw-iters 0" KEY=value,ms_per_step bash tools/ab_variants.sh
