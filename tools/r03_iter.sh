#!/bin/bash
# One build -> measure iteration: the -m gpu suite (or a -k subset), the driver's bench command,
# the 400-step bench, and rocprofv3 kernel stats of a serial and of the overlapped command.
# Each GPU step under its own limit; the first failure ends the script (no retries).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-iter}; mkdir -p $OUT
STEPS=${STEPS:-test,bench,prof}
if [[ $STEPS == *test* ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
      --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -20 $OUT/bench_driver.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_driver.json')); print('driver', round(d['value']/1e9,1), d['ms_per_step'], d['phases_ms'])"
  timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_400.json 2> $OUT/bench_400.err || { tail -20 $OUT/bench_400.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_400.json')); print('400', round(d['value']/1e9,1), d['ms_per_step'], d['phases_ms'])"
fi
if [[ $STEPS == *prof* ]]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_serial -o run --output-format csv -- \
    python3 $R/bench.py --steps 100 --warmup 20 --serial --no-cpu-baseline --cold-steps 0 > $OUT/prof_serial_bench.json 2> $OUT/prof_serial.err || { tail -20 $OUT/prof_serial.err; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
  cd $R
  for f in $OUT/prof_serial/run_kernel_stats.csv $OUT/prof/run_kernel_stats.csv; do
    echo "== $f"; python3 tools/kstats.py $f
  done
fi
echo done
