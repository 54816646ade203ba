#!/bin/bash
# bench.py alternating between the default build and build/abl/libcpg_$B.so (dev A/B).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/ab
for i in 1 2 3; do
  for lib in "" build/abl/libcpg_${B}.so; do
    tag=$(basename "${lib:-default}" .so)
    CPG_LIB_OVERRIDE=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS_N:-40} \
        > gpurun_out/ab/${tag}_$i.json 2> gpurun_out/ab/${tag}_$i.err || { echo "$tag failed"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab/${tag}_$i.json'));print('$tag', $i, round(d['value']/1e9,1), d['phases_ms'])"
  done
done
