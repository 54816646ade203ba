#!/bin/bash
# Round 4: the front kernel (k_vit_front: K1-K4 in one launch) — decode parity, then the
# decode alone against the previous build (build/abl/libcpg_head.so) and the 4-step-table
# variant (build/abl/libcpg_frontp4.so) at 46 Mbp and 3.1 Gbp, alternating; kernel statistics
# and PMC of the front kernel at 46 Mbp.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04_front}; mkdir -p $OUT
L=$R/cpgisland_amd/libcpg.so; H=$R/build/abl/libcpg_head.so; P4=$R/build/abl/libcpg_frontp4.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c3.py tests/test_gpu_contigs.py tests/test_gpu_c5.py tests/test_gpu_halo.py \
  -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
dec() {   # name lib bases
  CPG_LIB_OVERRIDE=$2 BASES=$3 REPS=9 timeout -k 10 200 python -u tools/decode_c3.py > $OUT/$1.json 2> $OUT/$1.err || { tail -5 $OUT/$1.err; return 1; }
  echo "$1 decode_ms $(python3 -c "import json; d=json.load(open('$OUT/$1.json')); print(round(d['ms_median'],4), d['islands'])")"
}
for i in 1 2; do
  dec new46_$i $L 46000000 || exit 1; dec p4_46_$i $P4 46000000 || exit 1; dec head46_$i $H 46000000 || exit 1
done
dec new3g $L 3100000000 || exit 1; dec p4_3g $P4 3100000000 || exit 1; dec head3g $H 3100000000 || exit 1
cd /tmp && export TMPDIR=/tmp
for lib in new p4; do
  LL=$L; [ $lib = p4 ] && LL=$P4
  CPG_LIB_OVERRIDE=$LL BASES=46000000 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$lib -o prof \
    -- python $R/tools/decode_c3.py > $OUT/prof_$lib.json 2> $OUT/prof_$lib.err || { tail -5 $OUT/prof_$lib.err; exit 1; }
done
for p in "p1 SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD" "p2 FETCH_SIZE" "p3 WRITE_SIZE" "p4 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES"; do
  set -- $p; name=$1; shift
  BASES=46000000 timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/dq/$name -o $name \
    -- python $R/tools/decode_c3.py > $OUT/dq_$name.json 2> $OUT/dq_$name.err || { tail -5 $OUT/dq_$name.err; exit 1; }
done
cd $R
python tools/pmc_summary.py $OUT/dq $OUT/pmc_decode46.json 46000000 "tools/decode_c3.py BASES=46000000 (decode alone)" > $OUT/pmc_decode46.txt 2>&1 && cut -c1-330 $OUT/pmc_decode46.txt | head -12
python3 - $OUT <<'EOF'
import csv, re, sys, glob
for lib in ("new", "p4"):
    f = glob.glob(f"{sys.argv[1]}/prof_{lib}/**/*kernel_stats.csv", recursive=True)
    for r in csv.DictReader(open(f[0])):
        m = re.search(r'::(k_[a-z0-9_]+)', r['Name'])
        if m: print(f"{lib:4s} {m.group(1):22s} calls {r['Calls']:>4s} avg_us {float(r['AverageNs'])/1e3:8.1f}")
EOF
