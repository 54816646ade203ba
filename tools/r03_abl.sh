#!/bin/bash
# E-step main-loop ablations (dev-only builds, wrong results by design): the kernel time
# without the LDS atomics / the backward row loads / the forward LDS reads / half the loop.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for lib in "" build/abl/libcpg_noatom.so build/abl/libcpg_nobload.so build/abl/libcpg_noflds.so build/abl/libcpg_half.so; do
  CPG_LIB_OVERRIDE=$lib PHASES="estep estep" timeout -k 10 200 python tools/ktime.py 2>&1 | grep -v amdgpu.ids || exit 1
done
