#!/bin/bash
# Whole-tree GPU check: the -m gpu suite, smoke, the driver's bench command (C2 line with the
# C3 leg), optionally a measurement tool (EXTRA="python tools/x.py ...", its stdout to
# extra.jsonl) and (PROF=1) the rocprof kernel statistics of the bench command.  The bench line
# is the un-instrumented run; the rocprof run's statistics are kernel_stats_prof.csv (its own
# run, its own bench line: bench_prof.json).
# Usage: TAG=r06_x gpurun -- bash tools/gpu_check.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-gpu_check}; mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
      --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1; rc=$?
  tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
  echo smoke ok
fi
if [ -n "$EXTRA" ]; then
  timeout -k 10 ${EXTRA_TIMEOUT:-300} $EXTRA > $OUT/extra.jsonl 2> $OUT/extra.err || { tail -5 $OUT/extra.err; exit 1; }
  tail -2 $OUT/extra.jsonl
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || { tail -5 $OUT/bench_driver.err; exit 1; }
  python3 tools/bench_summary.py $OUT/bench_driver.json
fi
if [ "${PROF:-0}" = 1 ]; then
  export TMPDIR=/tmp
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o prof \
    -- python $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_prof.json 2> $OUT/bench_prof.err) || { tail -5 $OUT/bench_prof.err; exit 1; }
  find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_prof.csv \;
  python3 tools/bench_summary.py $OUT/bench_prof.json
fi
