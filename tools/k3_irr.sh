cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); cd /tmp; export TMPDIR=/tmp
for v in "" noirr; do
  L=""; [ -n "$v" ] && L=$R/build/abl/libcpg_$v.so
  CPG_LIB_OVERRIDE=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/k3_$v -o run --output-format csv -- python3 $R/tools/ktime.py > /dev/null 2>&1 || exit 1
done
