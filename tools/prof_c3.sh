#!/bin/bash
# C3 (3.1 Gbp on this one GPU): the decode alone under rocprofv3 (kernel statistics) and the
# two-stream C3 bench leg, for the current tree.  TAG names the output directory.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-prof_c3}; mkdir -p $OUT
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/dec -o dec \
  -- python $R/tools/decode_c3.py > $OUT/decode_c3.json 2> $OUT/decode_c3.err) || { tail -5 $OUT/decode_c3.err; exit 1; }
find $OUT/dec -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_decode_c3.csv \;
cat $OUT/decode_c3.json
python3 tools/kstats.py $OUT/kernel_stats_decode_c3.csv 2>/dev/null | head -20 || head -20 $OUT/kernel_stats_decode_c3.csv
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline --bw-iters 0 > $OUT/c3_$i.json 2> $OUT/c3_$i.err || { tail -5 $OUT/c3_$i.err; exit 1; }
  python3 tools/bench_summary.py $OUT/c3_$i.json
done
