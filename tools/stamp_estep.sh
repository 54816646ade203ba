cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in ${STAMP_LIBS:-st4}; do CPG_LIB_OVERRIDE=build/abl/libcpg_$v.so timeout -k 10 120 python tools/estep_debug.py 2>&1 | grep "stamp c300 w\(0\|15\)" | sed "s/^/$v /" | head -2; done
[ -n "$ABL_LIBS" ] && bash tools/abl_estep.sh | grep "estep ms"
