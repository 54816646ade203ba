cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/pmc.sh || exit 1
python tools/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_latest.json 46000000 > gpurun_out/pmc_summary.txt
cat gpurun_out/pmc_summary.txt | cut -c1-220
# N-rank rehearsal of bench.py on the one GPU (gloo collectives through host memory)
[ -n "$PMC_DIST" ] && CPG_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/dist2_gloo.json 2> gpurun_out/dist2_gloo.err
echo "dist2 rc=$?"; cat gpurun_out/dist2_gloo.json | cut -c1-400
