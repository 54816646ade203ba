#!/bin/bash
# Experiment: serial vs two-stream step, kernargs in host vs device memory; per-kernel
# rocprof stats for the serial step under both kernarg placements.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/exp; mkdir -p $OUT
for kv in 0 1; do
  for mode in "" "--serial"; do
    tag=k${kv}${mode:+_serial}
    HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 $mode \
      > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { echo "bench $tag failed"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/bench_$tag.json')); print('$tag', round(d['value']/1e9,2), d['ms_per_step'], d['phases_ms'])"
  done
done
R=$(pwd); cd /tmp && export TMPDIR=/tmp
for kv in 0 1; do
  HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_k$kv -o run \
    --output-format csv -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --serial \
    > $R/$OUT/prof_k$kv.json 2> $R/$OUT/prof_k$kv.err || { echo "rocprof k$kv failed"; exit 1; }
done
echo done
