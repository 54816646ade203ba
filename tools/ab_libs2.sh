#!/bin/bash
# Same-box A/B of libcpg builds (dev tool): ktime of PHASES for each lib in LIBS, ROUNDS times
# alternating.  Each step under its own limit; first failure ends it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${TAG:-ab}; mkdir -p $OUT
for r in $(seq ${ROUNDS:-2}); do
  for L in $LIBS; do
    CPG_LIB_OVERRIDE=$L PHASES="${PHASES:-train}" timeout -k 10 200 python tools/ktime.py >> $OUT/ktime.log 2>&1 || exit 1
  done
done
grep median $OUT/ktime.log
