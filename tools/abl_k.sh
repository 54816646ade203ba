# phase timing (tools/ktime.py) of ablation builds against the default build, 2 rounds
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do for lib in "" ${ABL_LIBS}; do
  CPG_LIB_OVERRIDE=$lib timeout -k 10 120 python tools/ktime.py 2>&1 | grep " us " || exit 1
done; done
