mkdir -p gpurun_out/sw2
for r in 1 2; do
for cfg in "base 192" "repb 160" "repb 176" "repb 184" "repb 192" "repb 208"; do
  set -- $cfg
  CPG_LIB_OVERRIDE=build/abl/libcpg_$1.so timeout -k 10 120 python bench.py --no-cpu-baseline --train-cus $2 > gpurun_out/sw2/$1_$2_$r.json 2> gpurun_out/sw2/$1_$2_$r.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/sw2/$1_$2_$r.json')); print('$1', $2, $r, round(d['value']/1e9,1), d['phases_ms'])"
done; done
