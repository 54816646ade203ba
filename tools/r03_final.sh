#!/bin/bash
# Round 3 closing GPU session: the full -m gpu suite, smoke, the driver's bench command, and
# the C3 path rehearsed with 4 gloo ranks on the one GPU (islands must equal the N=1 count).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; OUT=gpurun_out/${TAG:-final}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || exit $?
python3 -c "import json; d=json.load(open('$OUT/bench_driver.json')); print('driver', round(d['value']/1e9,1), d['ms_per_step'], d['phases_ms'])"
CPG_BENCH_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 4 --steps 5 --warmup 2 \
    > $OUT/c3_gloo4.out 2> $OUT/c3_gloo4.err || { tail -20 $OUT/c3_gloo4.err; exit 1; }
grep '^{' $OUT/c3_gloo4.out > $OUT/c3_gloo4.json
python3 -c "import json; d=json.load(open('$OUT/c3_gloo4.json')); print('c3 gloo4', round(d['value']/1e9,1), d['ms_per_step'], d['config']['islands_found'])"
