#!/bin/bash
# Round 4 final tree: the whole -m gpu suite, smoke, the driver's bench command, and the
# kernel statistics of the C3 workload on this GPU (two streams) for profiles/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04_final4}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -5 $OUT/bench_driver.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench_driver.json'))
print('driver', round(d['value']/1e9,1), d['ms_per_step'], d['phases_ms'])
print('c3', {k: d['c3_single_gpu'][k] for k in ('value','ms_per_step','phases_ms')})
print('count', d['roofline_count']['achieved'], d['roofline_count']['ms_median'])"
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3 -o c3 \
  -- python $R/bench.py --workload c3 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err) || { tail -5 $OUT/c3.err; exit 1; }
find $OUT/c3 -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_c3.csv \;
python3 -c "import json; d=json.load(open('$OUT/c3.json')); print('c3 (rocprof)', round(d['value']/1e9,1), d['ms_per_step'])"
