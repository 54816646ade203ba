cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/ovl -o run --output-format csv -- python3 $R/bench.py --steps 100 --warmup 20 --no-cpu-baseline --cold-steps 0 > $R/gpurun_out/ovl_bench.json 2> $R/gpurun_out/ovl.err
echo rc=$?
