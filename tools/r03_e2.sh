#!/bin/bash
# E-step iteration: the E-step / training-pass GPU tests, per-phase stamps (ABL_STAMP build),
# kernel times of the product build.  Each GPU step under its own limit; first failure ends it.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${TAG:-e2}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
    --timeout-method thread -k "${PYTEST_K:-estep or train or fused or stream or contig or cli or smoke}" > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
CPG_LIB_OVERRIDE=build/abl/libcpg_stamp.so timeout -k 10 200 python tools/stamp_estep.py > $OUT/stamp.log 2>&1 || exit 1
grep -v amdgpu.ids $OUT/stamp.log
PHASES="train estep" timeout -k 10 200 python tools/ktime.py > $OUT/ktime.log 2>&1 || exit 1
cat $OUT/ktime.log | grep median
