#!/bin/bash
# Round 3 probe: the driver's exact bench command (20 steps / 5 warm-up) against the 400-step
# default, plus a kernel trace of the driver command.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out/startup; mkdir -p $OUT
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --cold-steps 0 "$@" > $OUT/$n.json 2> $OUT/$n.err
  local rc=$?
  python3 -c "import json,sys; d=json.load(open('$OUT/$n.json')); print('$n', round(d['value']/1e9,1), d['ms_per_step'], d['phases_ms'], d['host_issue_ms_per_step'])"
  return $rc
}
run d20a --steps 20 --warmup 5 && run d20b --steps 20 --warmup 5 && \
run d400 --steps 400 --warmup 20 && run d20nomask --steps 20 --warmup 5 --train-cus 0 && \
run d20noev --steps 20 --warmup 5 --no-phase-events && run d100 --steps 100 --warmup 5 && \
run d20w50 --steps 20 --warmup 50 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tr20 -o run --output-format csv -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --cold-steps 0 \
  > $OUT/tr20.json 2> $OUT/tr20.err
echo "rocprof rc=$?"
cd $R && python3 tools/step_gaps.py $OUT/tr20 > $OUT/tr20_gaps.txt
echo done
