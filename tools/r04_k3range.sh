#!/bin/bash
# Round 4: K3 with one 32 KB LDS union on the segment path (the binade range of a multi-binade segment in LDS,
# <= 16 binades), build/abl/libcpg_k3range.so, against the working tree: Viterbi parity with the
# variant, kernel statistics of the decode alone at 3.1 Gbp (twice each) and 46 Mbp.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04_k3range}; mkdir -p $OUT
L=$R/cpgisland_amd/libcpg.so; V=$R/build/abl/libcpg_k3range.so
CPG_LIB_OVERRIDE=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c3.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "(viterbi or decode or island or c3) and not timeout" > $OUT/pytest_k3range.log 2>&1 || { tail -30 $OUT/pytest_k3range.log; exit 1; }
tail -1 $OUT/pytest_k3range.log
cd /tmp && export TMPDIR=/tmp
run() {   # name lib bases
  CPG_LIB_OVERRIDE=$2 BASES=${3:-3100000000} REPS=5 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$1 -o prof \
    -- python $R/tools/decode_c3.py > $OUT/$1.json 2> $OUT/$1.err || { tail -5 $OUT/$1.err; return 1; }
  python3 - $OUT $1 <<'PY'
import csv, re, sys, glob, json
out, name = sys.argv[1], sys.argv[2]
d = json.load(open(f"{out}/{name}.json"))
f = glob.glob(f"{out}/prof_{name}/**/*kernel_stats.csv", recursive=True)
ks = []
for r in csv.DictReader(open(f[0])):
    m = re.search(r'::(k_[a-z0-9_]+)', r['Name'])
    if m and not m.group(1).startswith("k_estep"):
        ks.append(f"{m.group(1)} {float(r['AverageNs'])/1e3:.1f}")
print(name, "decode_ms", round(d["ms_median"], 4), "islands", d["islands"], "|", ", ".join(ks))
PY
}
run new $L || exit 1; run k3range $V || exit 1; run new_b $L || exit 1; run k3range_b $V || exit 1
run new46 $L 46000000 || exit 1; run k3range46 $V 46000000 || exit 1
