#!/bin/bash
# rocprofv3 kernel statistics of the decode alone (tools/decode_c3.py) at BASES (default the
# C2 46 Mbp), for the tree and, with PKG=<name>, a variant package tree
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); export TMPDIR=/tmp
OUT=$R/gpurun_out/${TAG:-prof_decode}; mkdir -p $OUT
export BASES=${BASES:-46000000} REPS=${REPS:-41}
for v in base $PKGS; do
  if [ $v = base ]; then export CPG_DEV_PKG=""; else export CPG_DEV_PKG=$R/build/abl/pkg_$v; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o $v \
     -- python $R/tools/decode_c3.py > $OUT/$v.json 2> $OUT/$v.err) || { tail -5 $OUT/$v.err; exit 1; }
  f=$(find $OUT/$v -name '*kernel_stats.csv' | head -1); cp $f $OUT/kernel_stats_$v.csv
  python3 - $OUT/kernel_stats_$v.csv <<'PY'
import csv, sys, re
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    n = re.sub(r"\(.*", "", r["Name"]).split("::")[-1]
    print(f"  {n[:40]:40s} calls {int(r['Calls']):5d} avg_us {float(r['AverageNs'])/1e3:8.2f}")
PY
done
