#!/bin/bash
# Round 4: the N-rank C3 bench path rehearsed with 2 gloo ranks sharing this one GPU (decode
# phases take turns), then the K3 compact-LDS variant measurement (tools/r04_k3l1.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04_final}; mkdir -p $OUT
CPG_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 \
    > $OUT/c3_gloo2.out 2> $OUT/c3_gloo2.err || { grep -v Warn $OUT/c3_gloo2.err | tail -20; exit 1; }
grep '^{' $OUT/c3_gloo2.out > $OUT/c3_gloo2.json
python3 -c "import json; d=json.load(open('$OUT/c3_gloo2.json')); print('c3 gloo2', round(d['value']/1e9,1), d['ms_per_step'], d['config']['islands_found'], d['config']['ranks_share_gpu'], d['roofline'].get('traffic'), d.get('cpu_baseline_note','')[:40])"
bash tools/r04_k3l1.sh
