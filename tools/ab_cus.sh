# bench A/B over training-stream CU counts (alternating, 2 rounds; STEPS per run)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; rm -f gpurun_out/ab_cus.log
for rep in 1 2; do for cu in ${CUS:-224 234}; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --cold-steps 0 --steps ${STEPS:-40} --train-cus $cu ${EXTRA:-} > gpurun_out/ab_$cu.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_$cu.json'));print('cus',$cu,'value %.1f'%(d['value']/1e9),'ms %.4f'%d['ms_per_step'],d['phases_ms'])" >> gpurun_out/ab_cus.log
done; done
cat gpurun_out/ab_cus.log
