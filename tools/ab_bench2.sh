#!/bin/bash
# Same-box A/B of libcpg builds (dev tool): the 400-step overlapped bench for each lib in LIBS,
# ROUNDS times alternating.  Each step under its own limit; first failure ends it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${TAG:-abb}; mkdir -p $OUT
for r in $(seq ${ROUNDS:-2}); do
  for L in $LIBS; do
    n=$(basename $L .so)
    CPG_LIB_OVERRIDE=$L timeout -k 10 120 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/$n.$r.json 2> $OUT/$n.$r.err || exit 1
    python3 -c "import json; d=json.load(open('$OUT/$n.$r.json')); print('$n', $r, round(d['value']/1e9,1), d['phases_ms'])"
  done
done
