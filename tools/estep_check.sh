cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread 2>&1 | tail -2 || exit 1
PHASES="estep" timeout -k 10 100 python tools/ktime.py || exit 1
R=$(pwd); cd /tmp; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmcw -o w -- python3 $R/tools/ktime.py > /dev/null 2>&1; echo "pmc rc=$?"
cd $R; python - <<'PY'
import csv,glob
v=[float(r['Counter_Value']) for f in glob.glob('gpurun_out/pmcw/*/*counter_collection.csv') for r in csv.DictReader(open(f)) if 'k_estep_chunk' in r['Kernel_Name']]
print('estep WRITE_SIZE KB median', sorted(v)[len(v)//2] if v else None)
PY
bash tools/ab_libs.sh
