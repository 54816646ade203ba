# bench A/B of libcpg builds (CPG_LIB_OVERRIDE; "" = the default build), alternating, REPS rounds (2)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; rm -f gpurun_out/ab_libs.log
for rep in $(seq ${REPS:-2}); do for lib in "" ${ABL_LIBS}; do
  CPG_LIB_OVERRIDE=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --cold-steps 0 --steps ${STEPS:-40} ${EXTRA:-} > gpurun_out/ab.json 2>/dev/null || exit 1
  python -c "import json,os;d=json.load(open('gpurun_out/ab.json'));print(os.path.basename('$lib') or 'default','value %.1f'%(d['value']/1e9),'ms %.4f'%d['ms_per_step'],d['phases_ms'])" >> gpurun_out/ab_libs.log
done; done
cat gpurun_out/ab_libs.log
