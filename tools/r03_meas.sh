#!/bin/bash
# Round 3 measurement session: driver-command bench (with the CPU baseline), 400-step bench,
# rocprofv3 kernel trace + stats of the driver command, PMC passes (roofline traffic), the C5
# streamed genome line.  Each GPU step under its own limit; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-meas}; mkdir -p $OUT
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || exit $?
python3 -c "import json; d=json.load(open('$OUT/bench_driver.json')); print('driver', round(d['value']/1e9,1), d['ms_per_step'], d['phases_ms'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_400.json 2> $OUT/bench_400.err || exit $?
python3 -c "import json; d=json.load(open('$OUT/bench_400.json')); print('400', round(d['value']/1e9,1), d['ms_per_step'], d['phases_ms'])"
timeout -k 10 300 python tools/bench_stream.py > $OUT/c5_stream_3p1G.json 2> $OUT/c5.err || exit $?
python3 -c "import json; d=json.load(open('$OUT/c5_stream_3p1G.json')); print('c5', round(d['value']/1e9,1), d['seconds'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_serial -o run --output-format csv -- \
  python3 $R/bench.py --steps 100 --warmup 20 --serial --no-cpu-baseline --cold-steps 0 > $OUT/prof_serial_bench.json 2> $OUT/prof_serial.err || exit $?
cd $R && bash tools/pmc_round.sh > $OUT/pmc_round.log 2>&1; rc=$?; tail -15 $OUT/pmc_round.log; exit $rc
