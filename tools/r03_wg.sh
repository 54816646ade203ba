#!/bin/bash
# A/B of the two-workgroups-per-CU E-step (CPG_EST_WG=1) against the default kernel:
# E-step / training-pass times at 46 Mbp, its parity tests, the overlapped bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/wg; mkdir -p $OUT
timeout -k 10 150 python tools/estep_chunks.py 2>&1 | grep -v amdgpu.ids > $OUT/chunks_default.txt || exit $?
cat $OUT/chunks_default.txt
CPG_EST_WG=1 timeout -k 10 150 python tools/estep_chunks.py 2>&1 | grep -v amdgpu.ids > $OUT/chunks_wg.txt || exit $?
echo "--- WG"; cat $OUT/chunks_wg.txt
CPG_EST_WG=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "estep or train or fused or stream or c3 or halo" > $OUT/pytest_wg.log 2>&1; rc=$?
tail -3 $OUT/pytest_wg.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for v in 0 1; do
  CPG_EST_WG=$v timeout -k 10 300 python bench.py --no-cpu-baseline --cold-steps 0 > $OUT/b400_${v}_$i.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('$OUT/b400_${v}_$i.json')); print('WG=$v', round(d['value']/1e9,1), d['ms_per_step'], d['phases_ms'])"
done; done
