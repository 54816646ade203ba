#!/bin/bash
# round 6: tree check (tests, smoke, load-shape tool, driver bench) + decode / bench A/B against
# round 5's sources (tools/build_rev.sh r05 14bc45d)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${T:-r06b} EXTRA="python tools/loadshape.py" bash tools/gpu_check.sh || exit 1
TAG=${T:-r06b}_dec VARIANTS=r05 ROUNDS=3 TOOL="tools/decode_c3.py" KEY=ms_median BASES=46000000 REPS=41 bash tools/ab_variants.sh || exit 1
TAG=${T:-r06b}_bench VARIANTS=r05 ROUNDS=2 TOOL="tools/bench_variant.py --steps 400 --warmup 20 --no-cpu-baseline --c3-steps 0 --bw-iters 0 --cold-steps 0" KEY=value,ms_per_step bash tools/ab_variants.sh
