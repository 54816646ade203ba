#!/bin/bash
# Round 4: the whole GPU suite on the working tree's library, then A/B timings against the
# previous build (build/abl/libcpg_head.so): the training pass (count_hbm.py --train) and the
# decode alone (decode_c3.py) at 46 Mbp and 3.1 Gbp, alternating; the serial bench phases;
# kernel statistics and the LDS bank-conflict counters of the decode at 46 Mbp.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04_ab}; mkdir -p $OUT
L=$R/cpgisland_amd/libcpg.so; H=$R/build/abl/libcpg_head.so
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
hbm() {   # name lib bases
  CPG_LIB_OVERRIDE=$2 timeout -k 10 200 python -u tools/count_hbm.py --bases $3 --no-sweep --reps 10 --train > $OUT/$1.json 2> $OUT/$1.err || { tail -5 $OUT/$1.err; return 1; }
  echo "$1 train_pass_ms $(python3 -c "import json; d=json.load(open('$OUT/$1.json')); print(d.get('train_pass_ms_median'))")"
}
dec() {   # name lib bases
  CPG_LIB_OVERRIDE=$2 BASES=$3 REPS=9 timeout -k 10 200 python -u tools/decode_c3.py > $OUT/$1.json 2> $OUT/$1.err || { tail -5 $OUT/$1.err; return 1; }
  echo "$1 decode_ms $(python3 -c "import json; d=json.load(open('$OUT/$1.json')); print(round(d['ms_median'],4), d['islands'])")"
}
for i in 1 2; do
  hbm tnew46_$i $L 46000000 || exit 1; hbm thead46_$i $H 46000000 || exit 1
  dec dnew46_$i $L 46000000 || exit 1; dec dhead46_$i $H 46000000 || exit 1
done
hbm tnew3g $L 3100000000 || exit 1; hbm thead3g $H 3100000000 || exit 1
dec dnew3g $L 3100000000 || exit 1; dec dhead3g $H 3100000000 || exit 1
P4=$R/build/abl/libcpg_frontp4.so   # the front kernel with K3's 4-step table instead of lane-private rows
if [ -f $P4 ]; then
  dec dp4_46_1 $P4 46000000 || exit 1; dec dnew46_3 $L 46000000 || exit 1; dec dp4_46_2 $P4 46000000 || exit 1
  dec dp4_3g $P4 3100000000 || exit 1
fi
for lib in new head; do
  LL=$L; [ $lib = head ] && LL=$H
  CPG_LIB_OVERRIDE=$LL timeout -k 10 300 python -u bench.py --serial --steps 100 --warmup 20 --c3-steps 0 --no-cpu-baseline --cold-steps 0 > $OUT/serial_$lib.json 2> $OUT/serial_$lib.err || { tail -5 $OUT/serial_$lib.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/serial_$lib.json')); print('serial $lib', d['value'], d['phases_ms'])"
done
cd /tmp && export TMPDIR=/tmp
for lib in new head; do
  LL=$L; [ $lib = head ] && LL=$H
  CPG_LIB_OVERRIDE=$LL BASES=46000000 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$lib -o prof \
    -- python $R/tools/decode_c3.py > $OUT/prof_$lib.json 2> $OUT/prof_$lib.err || { tail -5 $OUT/prof_$lib.err; exit 1; }
  CPG_LIB_OVERRIDE=$LL BASES=46000000 timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS \
    --kernel-trace --output-format csv -d $OUT/pmc_$lib -o pmc -- python $R/tools/decode_c3.py > $OUT/pmc_$lib.json 2> $OUT/pmc_$lib.err || { tail -5 $OUT/pmc_$lib.err; exit 1; }
done
for p in "p1 SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD" "p2 FETCH_SIZE" "p3 WRITE_SIZE"; do
  set -- $p; name=$1; shift
  BASES=46000000 timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/dq/$name -o $name \
    -- python $R/tools/decode_c3.py > $OUT/dq_$name.json 2> $OUT/dq_$name.err || { tail -5 $OUT/dq_$name.err; exit 1; }
done
cd $R
python tools/pmc_summary.py $OUT/dq $OUT/pmc_decode46.json 46000000 "tools/decode_c3.py BASES=46000000 (decode alone)" > $OUT/pmc_decode46.txt 2>&1 && cut -c1-200 $OUT/pmc_decode46.txt | head -30
for lib in new head; do
  find $OUT/prof_$lib -name '*kernel_stats.csv' -exec cp {} $OUT/kstats_$lib.csv \;
  echo "== $lib"; cut -d, -f1-4 $OUT/kstats_$lib.csv | sed 's/(.*)//' | grep -E "vit_|estep" | head -10
  python3 - "$OUT/pmc_$lib" <<'EOF'
import csv, glob, sys, collections, re
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f[0])):
    m = re.search(r"::(k_vit_[a-z0-9_]+)", r["Kernel_Name"])
    if not m: continue
    acc[m.group(1)][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    c, a = d.get("SQ_LDS_BANK_CONFLICT", 0), d.get("SQ_LDS_IDX_ACTIVE", 0)
    w = max(d.get("SQ_WAVES", 1), 1)
    print(f"{k[:28]:28s} conflict/active {c:.3g}/{a:.3g} = {c / max(a, 1):.3f}  valu/wave {d.get('SQ_INSTS_VALU', 0) / w:.0f}  lds/wave {d.get('SQ_INSTS_LDS', 0) / w:.0f}")
EOF
done
