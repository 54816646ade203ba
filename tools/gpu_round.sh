#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel trace.  Each GPU step has its
# own time limit; a crash/abort/timeout (rc >= 124 or signal) ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out
mkdir -p $OUT
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
STEPS=${STEPS:-all}
if [[ $STEPS == *all* || $STEPS == *test* ]]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 -rf \
      > $OUT/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log
  ok $rc || exit $rc
fi
if [[ $STEPS == *abl* ]]; then   # E-step timing of each ablation build vs the default build
  for lib in "" build/abl/*.so; do
    CPG_LIB_OVERRIDE=$lib timeout -k 10 300 python tools/estep_ablate.py >> $OUT/abl.log 2>&1
    rc=$?; echo "abl $lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  cat $OUT/abl.log
fi
if [[ $STEPS == *all* || $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == *all* || $STEPS == *bench* ]]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
  rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; [ $rc -eq 0 ] || { tail -20 $OUT/bench.err; exit $rc; }
fi
if [[ $STEPS == *all* || $STEPS == *prof* ]]; then
  R=$(pwd)
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof -o run --output-format csv \
      -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline ${PROF_ARGS:---serial} > $R/$OUT/prof_bench.json 2> $R/$OUT/prof.err
  rc=$?; echo "rocprof rc=$rc"; cd $R
  find $OUT/prof -name "*stats*" | head; [ $rc -eq 0 ] || { tail -20 $OUT/prof.err; exit $rc; }
fi
if [[ $STEPS == *pmc* ]]; then
  bash tools/pmc.sh; rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
echo done
