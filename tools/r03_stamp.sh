#!/bin/bash
# Per-phase wall-clock stamps (100 MHz) of the E-step workgroups (dev-only build ABL_STAMP).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
CPG_LIB_OVERRIDE=build/abl/libcpg_stamp.so PHASES="estep" timeout -k 10 200 python tools/ktime.py > gpurun_out/stamp.log 2>&1 || exit 1
grep stamp gpurun_out/stamp.log | tail -15; grep estep gpurun_out/stamp.log | tail -2
