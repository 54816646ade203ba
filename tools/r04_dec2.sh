#!/bin/bash
# Round 4: decode variants at the C3 size (kernel statistics of the decode alone) — the
# working tree, the Viterbi and island scan as two calls (SEPARATE=1), K3 with lane-private
# 2-step rows (build/abl/libcpg_k3priv.so), K6 as its own launch (libcpg_k6sep.so); then the
# fused / separate island scan at 43, 256 and 1,024 decode chunks (where the fused traceback
# stops paying).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04_dec2}; mkdir -p $OUT
L=$R/cpgisland_amd/libcpg.so; K3=$R/build/abl/libcpg_k3priv.so; K6=$R/build/abl/libcpg_k6sep.so
CPG_LIB_OVERRIDE=$K3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c3.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "(viterbi or decode or island or c3) and not timeout" > $OUT/pytest_k3priv.log 2>&1 || { tail -30 $OUT/pytest_k3priv.log; exit 1; }
tail -1 $OUT/pytest_k3priv.log
cd /tmp && export TMPDIR=/tmp
run() {   # name lib separate bases
  CPG_LIB_OVERRIDE=$2 SEPARATE=$3 BASES=${4:-3100000000} REPS=5 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$1 -o prof \
    -- python $R/tools/decode_c3.py > $OUT/$1.json 2> $OUT/$1.err || { tail -5 $OUT/$1.err; return 1; }
  python3 - $OUT $1 <<'EOF'
import csv, re, sys, glob, json
out, name = sys.argv[1], sys.argv[2]
d = json.load(open(f"{out}/{name}.json"))
f = glob.glob(f"{out}/prof_{name}/**/*kernel_stats.csv", recursive=True)
ks = []
for r in csv.DictReader(open(f[0])):
    m = re.search(r'::(k_[a-z0-9_]+)', r['Name'])
    if m and not m.group(1).startswith("k_estep"):
        ks.append(f"{m.group(1)} {float(r['AverageNs'])/1e3:.0f}")
print(name, "decode_ms", round(d["ms_median"], 3), "islands", d["islands"], "|", ", ".join(ks))
EOF
}
run new $L 0 || exit 1
run sep $L 1 || exit 1
run k3priv $K3 0 || exit 1
run k6sep $K6 0 || exit 1
run k6sep_sep $K6 1 || exit 1
cd $R
dec() {   # name lib separate bases (event-timed, no profiler)
  CPG_LIB_OVERRIDE=$2 SEPARATE=$3 BASES=$4 REPS=9 timeout -k 10 200 python -u tools/decode_c3.py > $OUT/$1.json 2> $OUT/$1.err || { tail -5 $OUT/$1.err; return 1; }
  echo "$1 decode_ms $(python3 -c "import json; d=json.load(open('$OUT/$1.json')); print(round(d['ms_median'],4), d['decode_chunks'], d['islands'])")"
}
for n in 46000000 268435456 1073741824; do
  dec fused_$n $L 0 $n || exit 1; dec sep_$n $L 1 $n || exit 1
  dec fused2_$n $L 0 $n || exit 1; dec sep2_$n $L 1 $n || exit 1
done
