#!/bin/bash
# Round 4 final tree, part 2: the PMC profiles bench.py reads (C2, C3, count kernel), configs
# C4 (10M contigs) and C5 (streamed 3.1 Gbp), and the N-rank C3 path rehearsed with 2 gloo
# ranks on this one GPU.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04_final}; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/pmc_round.sh > $OUT/pmc_round.log 2>&1 || { tail -20 $OUT/pmc_round.log; exit 1; }
cp gpurun_out/pmc_latest.json gpurun_out/pmc_c3.json gpurun_out/pmc_count.json gpurun_out/pmc_summary.txt gpurun_out/pmc_c3_summary.txt gpurun_out/pmc_count_summary.txt $OUT/
cut -c1-200 $OUT/pmc_summary.txt | head -12
timeout -k 10 600 python -u tools/bench_contigs.py --contigs 10000000 --reps 3 > $OUT/c4_contigs_10M.json 2> $OUT/c4.err || { tail -5 $OUT/c4.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c4_contigs_10M.json')); print('C4', round(d['value']/1e9,1), d.get('ms'))"
timeout -k 10 300 python -u tools/bench_stream.py > $OUT/c5_stream_3p1G.json 2> $OUT/c5.err || { tail -5 $OUT/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c5_stream_3p1G.json')); print('C5', {k: d[k] for k in list(d)[:6]})"
CPG_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 \
    > $OUT/c3_gloo2.out 2> $OUT/c3_gloo2.err || { tail -20 $OUT/c3_gloo2.err; exit 1; }
grep '^{' $OUT/c3_gloo2.out > $OUT/c3_gloo2.json
python3 -c "import json; d=json.load(open('$OUT/c3_gloo2.json')); print('c3 gloo2', round(d['value']/1e9,1), d['ms_per_step'], d['config']['islands_found'], d['roofline'].get('traffic'), d.get('cpu_baseline_note','')[:40])"
