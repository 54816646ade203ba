# labelled counts + fused training pass: GPU tests, phase timing, fused-vs-separate bench A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -k "count or train or fused or estep" > gpurun_out/pt.log 2>&1; rc=$?; tail -3 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
PHASES="counts estep" timeout -k 10 100 python tools/ktime.py || exit 1
[ -n "$STAMP" ] && { CPG_LIB_OVERRIDE=build/abl/libcpg_cstamp.so PHASES=counts timeout -k 10 100 python tools/ktime.py 2>&1 | tail -8 || exit 1; }
for a in "" "--separate-train" "" "--separate-train"; do timeout -k 10 120 python bench.py --no-cpu-baseline --cold-steps 0 --steps 40 $a > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }; python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$a','value %.1f'%(d['value']/1e9),'ms %.4f'%d['ms_per_step'],d['phases_ms'])"; done
