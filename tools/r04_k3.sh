#!/bin/bash
# Round 4: K3 (k_vit_exact) single-binade path with lane-private 2-step rows (conflict-free
# ds_read_b128) against the 4-step table: Viterbi parity with the variant library, the decode
# alone at 46 Mbp and 3.1 Gbp (alternating), and the LDS bank-conflict counters of both.
#   VARIANT=build/abl/libcpg_<name>.so bash tools/r04_k3.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04_k3}; mkdir -p $OUT
V=$R/${VARIANT:-build/abl/libcpg_k3priv.so}; B=$R/cpgisland_amd/libcpg.so
CPG_LIB_OVERRIDE=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c3.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread -k "viterbi or decode or island or c3" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
dec() {   # name lib bases
  CPG_LIB_OVERRIDE=$2 BASES=$3 REPS=${REPS:-9} timeout -k 10 200 python -u tools/decode_c3.py > $OUT/$1.json 2> $OUT/$1.err || { tail -5 $OUT/$1.err; return 1; }
  echo "$1 $(python3 -c "import json; d=json.load(open('$OUT/$1.json')); print(round(d['ms_median'],4), d['islands'])")"
}
for i in 1 2; do
  dec var46_$i $V 46000000 || exit 1; dec base46_$i $B 46000000 || exit 1
done
dec var3g $V 3100000000 || exit 1; dec base3g $B 3100000000 || exit 1
cd /tmp && export TMPDIR=/tmp
for lib in var base; do
  LL=$V; [ $lib = base ] && LL=$B
  CPG_LIB_OVERRIDE=$LL BASES=46000000 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$lib -o prof \
    -- python $R/tools/decode_c3.py > $OUT/prof_$lib.json 2> $OUT/prof_$lib.err || { tail -5 $OUT/prof_$lib.err; exit 1; }
  CPG_LIB_OVERRIDE=$LL BASES=46000000 timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS \
    --kernel-trace --output-format csv -d $OUT/pmc_$lib -o pmc -- python $R/tools/decode_c3.py > $OUT/pmc_$lib.json 2> $OUT/pmc_$lib.err || { tail -5 $OUT/pmc_$lib.err; exit 1; }
done
cd $R
for lib in var base; do
  find $OUT/prof_$lib -name '*kernel_stats.csv' -exec cp {} $OUT/kstats_$lib.csv \;
  echo "== $lib"; cut -d, -f1-4 $OUT/kstats_$lib.csv | sed 's/(.*)//' | grep -E "vit_" | head -8
  python3 - "$OUT/pmc_$lib" <<'EOF'
import csv, glob, sys, collections, re
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f[0])):
    m = re.search(r"::(k_vit_[a-z0-9_]+)", r["Kernel_Name"])
    if not m: continue
    k = m.group(1)
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    c, a = d.get("SQ_LDS_BANK_CONFLICT", 0), d.get("SQ_LDS_IDX_ACTIVE", 0)
    print(f"{k[:40]:40s} conflict/active {c:.3g}/{a:.3g} = {c / max(a, 1):.3f}  valu/wave {d.get('SQ_INSTS_VALU', 0) / max(d.get('SQ_WAVES', 1), 1):.0f}  lds/wave {d.get('SQ_INSTS_LDS', 0) / max(d.get('SQ_WAVES', 1), 1):.0f}")
EOF
done
