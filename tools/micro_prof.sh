#!/bin/bash
# rocprofv3 kernel stats of tools/vit_micro.py for the default build and each ablation build.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out/micro; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for lib in "" $R/build/abl/*.so; do
  tag=$(basename "${lib:-default}" .so)
  CPG_LIB_OVERRIDE=$lib REPS=${REPS:-3} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$tag -o run \
     --output-format csv -- python $R/${MICRO:-tools/vit_micro.py} > $OUT/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $OUT/$tag.log; exit 1; }
  echo "$tag ok"
done
