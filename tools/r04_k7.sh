#!/bin/bash
# Round 4: the traceback + island tiles (k_vit_trace<true>) at the C3 size — kernel statistics
# of the decode alone for the working tree's library, K7 built for 5 and 6 waves per SIMD
# (build/abl/libcpg_k7w5.so, _k7w6.so), and the Viterbi and island scan as two calls
# (SEPARATE=1: the traceback without the tile work, then k_isl_tile + k_isl_resolve).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04_k7}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {   # name lib separate
  CPG_LIB_OVERRIDE=$2 SEPARATE=$3 IGNORE_STATUS=${4:-0} REPS=5 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$1 -o prof \
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
L=$R/cpgisland_amd/libcpg.so
run new $L 0 || exit 1
run sep $L 1 || exit 1
run k7w5 $R/build/abl/libcpg_k7w5.so 0 || exit 1
run k7w6 $R/build/abl/libcpg_k7w6.so 0 || exit 1
run new2 $L 0 || exit 1
# front-kernel ablations (wrong paths by construction, timing only): no chain; no chain and
# no exact composites
run fabl1 $R/build/abl/libcpg_fabl1.so 0 1 || exit 1
run fabl3 $R/build/abl/libcpg_fabl3.so 0 1 || exit 1
run head $R/build/abl/libcpg_head.so 0 || exit 1
cd $R && timeout -k 10 60 ./build/ubench_bits > $OUT/ubench_bits.txt 2>&1 && grep "waves/SIMD 4" $OUT/ubench_bits.txt
