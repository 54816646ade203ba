# bench A/B over argument sets (ARGSETS separated by '|'), alternating, 2 rounds
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; rm -f gpurun_out/ab_args.log
IFS='|' read -ra SETS <<< "${ARGSETS:-}"
for rep in 1 2; do for a in "${SETS[@]}"; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --cold-steps 0 --steps ${STEPS:-400} $a > gpurun_out/ab.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('[$a]','value %.1f'%(d['value']/1e9),'ms %.4f'%d['ms_per_step'],d['phases_ms'])" >> gpurun_out/ab_args.log
done; done
cat gpurun_out/ab_args.log
