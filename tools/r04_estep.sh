#!/bin/bash
# Round 4: E-step normalisation by integer exponent + multiply (no v_ldexp / v_frexp in the
# loops) — parity, then the training pass against the previous build (build/abl/libcpg_head.so)
# at 46 Mbp and 3.1 Gbp, alternating, and the serial bench's phase times.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04_estep}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_contigs.py -x -q -p no:cacheprovider --timeout 200 \
  --timeout-method thread -k "estep or train_pass or golden or count" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
hbm() {
  CPG_LIB_OVERRIDE=$2 timeout -k 10 200 python -u tools/count_hbm.py --bases $3 --no-sweep --reps 10 --train > $OUT/$1.json 2> $OUT/$1.err || { tail -5 $OUT/$1.err; return 1; }
  echo "$1 $(python3 -c "import json; d=json.load(open('$OUT/$1.json')); print(round(d['count_ms_median'],4), d.get('train_pass_ms_median'))")"
}
L=$R/cpgisland_amd/libcpg.so; H=$R/build/abl/libcpg_head.so
for i in 1 2; do
  hbm new46_$i $L 46000000 || exit 1; hbm head46_$i $H 46000000 || exit 1
done
hbm new3g $L 3100000000 || exit 1; hbm head3g $H 3100000000 || exit 1
for lib in new head; do
  LL=$L; [ $lib = head ] && LL=$H
  CPG_LIB_OVERRIDE=$LL timeout -k 10 300 python -u bench.py --serial --steps 100 --warmup 20 --c3-steps 0 --no-cpu-baseline --cold-steps 0 > $OUT/serial_$lib.json 2> $OUT/serial_$lib.err || { tail -5 $OUT/serial_$lib.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/serial_$lib.json')); print('serial $lib', d['phases_ms'])"
done
# the decode alone at the C3 size, event-timed and under rocprofv3 (kernel statistics)
timeout -k 10 200 python -u tools/decode_c3.py > $OUT/decode_c3.json 2> $OUT/decode_c3.err || { tail -5 $OUT/decode_c3.err; exit 1; }
cat $OUT/decode_c3.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_dec -o prof \
  -- python $R/tools/decode_c3.py > $OUT/prof_dec.json 2> $OUT/prof_dec.err || { tail -5 $OUT/prof_dec.err; exit 1; }
cd $R && find $OUT/prof_dec -name '*kernel_stats.csv' -exec cp {} $OUT/decode_c3_kernel_stats.csv \; && cut -d, -f1-4 $OUT/decode_c3_kernel_stats.csv | sed 's/(.*)//' | head -12
