# E-step timing of ablation builds (build/abl/libcpg_<name>.so) against the default build
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; rm -f gpurun_out/abl.log
for rep in 1 2; do
for lib in "" ${ABL_LIBS}; do
  CPG_LIB_OVERRIDE=$lib timeout -k 10 120 python tools/estep_ablate.py >> gpurun_out/abl.log 2>&1 || exit 1
done; done
grep -v amdgpu.ids gpurun_out/abl.log
