#!/bin/bash
# Round 4 final tree, part 1: the whole -m gpu suite, smoke, the driver's bench command (C2
# headline + C3 leg + count roofline), rocprofv3 kernel statistics of the serial bench and of
# the driver's command.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04_final}; mkdir -p $OUT
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
print('count', d['roofline_count'])
print('decode', d['roofline_decode'], d['roofline_decode_valu'])
print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/serial -o serial \
  -- python $R/bench.py --serial --steps 100 --warmup 20 --c3-steps 0 --no-cpu-baseline --cold-steps 0 > $OUT/serial.json 2> $OUT/serial.err) || { tail -5 $OUT/serial.err; exit 1; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/driver -o driver \
  -- python $R/bench.py --steps 20 --warmup 5 --c3-steps 0 --no-cpu-baseline > $OUT/driver.json 2> $OUT/driver.err) || { tail -5 $OUT/driver.err; exit 1; }
for n in serial driver; do find $OUT/$n -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_$n.csv \; ; done
echo "serial phases: $(python3 -c "import json; print(json.load(open('$OUT/serial.json'))['phases_ms'])")"
