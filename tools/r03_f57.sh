mkdir -p gpurun_out/f57
CPG_VIT_FUSE57=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/f57/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/f57/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in fused old; do
    if [ $v = fused ]; then export CPG_VIT_FUSE57=1; else unset CPG_VIT_FUSE57; fi
    timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/f57/$v.$r.json 2> gpurun_out/f57/$v.$r.err || { tail -5 gpurun_out/f57/$v.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/f57/$v.$r.json')); print('$v', $r, round(d['value']/1e9,1), d['phases_ms'])"
  done
done
export CPG_VIT_FUSE57=1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/f57/prof_serial -o run --output-format csv -- python3 /root/repo/bench.py --steps 100 --warmup 20 --serial --no-cpu-baseline --cold-steps 0 > /root/repo/gpurun_out/f57/prof_serial_bench.json 2> /root/repo/gpurun_out/f57/prof_serial.err || exit 1
cd /root/repo && python3 tools/kstats.py gpurun_out/f57/prof_serial/run_kernel_stats.csv
