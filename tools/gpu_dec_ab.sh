#!/bin/bash
# decode changes: the decode / island / Viterbi tests (tree), then the decode alone at 3.1 Gbp
# and at 46 Mbp, tree against the variants
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-dec_ab}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "${PYTEST_K:-viterbi or decode or island or c3 or golden or general or halo or stream or contig}" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
echo "tests: $(tail -1 $OUT/pytest.log)"
VARIANTS="$VARIANTS" TAG=${TAG:-dec_ab}_3g TOOL="tools/decode_c3.py" KEY=ms_median bash tools/ab_variants.sh || exit 1
BASES=46137344 REPS=50 VARIANTS="$VARIANTS" TAG=${TAG:-dec_ab}_46m TOOL="tools/decode_c3.py" KEY=ms_median bash tools/ab_variants.sh
