#!/bin/bash
# Round 3 GPU session: parity tests, smoke, the driver's bench command and the 400-step bench.
# Each GPU step has its own time limit; any failure ends the script (no retries).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r03}; mkdir -p $OUT
STEPS=${STEPS:-test,smoke,bench}
if [[ $STEPS == *test* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
      --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -4 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err
  rc=$?; echo "bench(driver cmd) rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_driver.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$OUT/bench_driver.json')); print('driver', round(d['value']/1e9,1), d['ms_per_step'], d['phases_ms'], d['roofline']['frac'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None)"
  timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/bench_400.json 2> $OUT/bench_400.err
  rc=$?; echo "bench(400) rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench_400.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$OUT/bench_400.json')); print('400', round(d['value']/1e9,1), d['ms_per_step'], d['phases_ms'])"
fi
if [[ $STEPS == *c3* ]]; then
  # the north_star workload: the whole 3.1 Gbp genome on this GPU, then the 2-rank path
  # rehearsed on the one GPU (gloo collectives staged through host memory)
  timeout -k 10 600 python bench.py --workload c3 --steps 10 --warmup 3 > $OUT/c3_n1.json 2> $OUT/c3_n1.err
  rc=$?; echo "c3 n1 rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/c3_n1.err; exit $rc; }
  python3 -c "import json; d=json.load(open('$OUT/c3_n1.json')); print('c3 n1', round(d['value']/1e9,1), d['ms_per_step'], d['phases_ms'], d['config']['islands_found'])"
  CPG_BENCH_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 \
      > $OUT/c3_gloo2.json 2> $OUT/c3_gloo2.err
  rc=$?; echo "c3 gloo2 rc=$rc"; [ $rc -eq 0 ] || { tail -30 $OUT/c3_gloo2.err; exit $rc; }
  python3 -c "import json; d=json.loads(open('$OUT/c3_gloo2.json').read().strip().splitlines()[-1]); print('c3 gloo2', round(d['value']/1e9,1), d['ms_per_step'], d['config']['islands_found'])"
fi
if [[ $STEPS == *prof* ]]; then
  R=$(pwd); cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof -o run --output-format csv \
      -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline ${PROF_ARGS:-} > $R/$OUT/prof_bench.json 2> $R/$OUT/prof.err
  rc=$?; echo "rocprof rc=$rc"; cd $R; [ $rc -eq 0 ] || { tail -20 $OUT/prof.err; exit $rc; }
  find $OUT/prof -name "*stats*"
fi
echo done
