cd "${GRAFT_REPO_ROOT:-/root/repo}"
for lib in "" ${ABL_LIBS}; do CPG_LIB_OVERRIDE=$lib CHUNKS="${CHUNKS:-256 702}" timeout -k 10 120 python tools/estep_scale.py 2>&1 | grep chunks || exit 1; done
