# Viterbi change check: GPU tests, phase timing, serial kernel trace, bench
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pt.log 2>&1; rc=$?; tail -5 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
PHASES="viterbi estep" timeout -k 10 100 python tools/ktime.py || exit 1
R=$(pwd); cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/vprof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --serial --cold-steps 0 > /dev/null 2>&1 || exit 1
cd $R; python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/vprof/run_kernel_stats.csv')):
    n=r['Name'].split('(')[0].split('::')[-1]; print(f"{n:22s} avg_us {float(r['AverageNs'])/1e3:7.1f} calls {r['Calls']}")
PY
for a in "" ""; do timeout -k 10 120 python bench.py --no-cpu-baseline --cold-steps 0 --steps 40 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }; python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('value %.1f'%(d['value']/1e9),'ms %.4f'%d['ms_per_step'],d['phases_ms'])"; done
