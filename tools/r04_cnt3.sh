#!/bin/bash
# Round 4: count kernel defaults (batch 2, grid 2048) — parity, 3.1 Gbp timing, PMC
# (VALU / SALU / VMEM instruction counts, wave states), and the integer-op issue microbenchmark.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04_cnt3}; mkdir -p $OUT
timeout -k 10 60 ./build/ubench_bits > $OUT/ubench_bits.txt 2>&1 || { cat $OUT/ubench_bits.txt; exit 1; }
cat $OUT/ubench_bits.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 200 \
  --timeout-method thread -k "count or train_pass or golden or estep" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python -u tools/count_hbm.py --bases 3100000000 --train > $OUT/count_hbm.json 2> $OUT/count_hbm.err || { tail -5 $OUT/count_hbm.err; exit 1; }
cat $OUT/count_hbm.json
cd /tmp && export TMPDIR=/tmp
i=0
for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_SCA SQ_INSTS_LDS" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc/p$i -o p$i \
    -- python $R/tools/count_hbm.py --bases 3100000000 --no-sweep --reps 3 > /dev/null 2> $OUT/p$i.err || { tail -3 $OUT/p$i.err; exit 1; }
done
cd $R && python tools/pmc_summary.py $OUT/pmc > $OUT/pmc_summary.txt && cat $OUT/pmc_summary.txt
python3 - <<PY
import csv, glob, collections
v = collections.defaultdict(list)
for f in glob.glob("$OUT/pmc/p*/p*_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "k_count_main" in r["Kernel_Name"]:
            v[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, x in sorted(v.items()):
    print(k, sum(x) / len(x))
PY
