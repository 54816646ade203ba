#!/bin/bash
# A/B of build/abl/libcpg_$B.so against the default build: E-step / training-pass time alone
# (tools/ktime.py, after a warm-up) and the 400-step bench, alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/ab
for lib in "" build/abl/libcpg_${B}.so; do
  CPG_LIB_OVERRIDE=$lib PHASES="estep train estep train" timeout -k 10 200 python tools/ktime.py 2>&1 | grep -v amdgpu.ids || exit 1
done
for i in 1 2; do
  for lib in "" build/abl/libcpg_${B}.so; do
    tag=$(basename "${lib:-default}" .so)
    CPG_LIB_OVERRIDE=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --cold-steps 0 \
        > gpurun_out/ab/${tag}_$i.json 2> gpurun_out/ab/${tag}_$i.err || { echo "$tag failed"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab/${tag}_$i.json'));print('$tag', $i, round(d['value']/1e9,1), d['phases_ms'])"
  done
done
