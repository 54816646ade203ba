#!/bin/bash
# Round-end check: the gpu suite + smoke + driver bench (tools/gpu_check.sh), then the 2-rank gloo
# rehearsal on this one GPU (bench.py's own launcher, both ranks' decodes concurrent) whose
# C3 fingerprints must equal the N = 1 leg's.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-final}; mkdir -p $OUT
bash tools/gpu_check.sh || exit 1
CPG_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --settle-ms 0 \
    > $OUT/c3_gloo2.out 2> $OUT/c3_gloo2.err || { tail -20 $OUT/c3_gloo2.err; exit 1; }
grep '^{' $OUT/c3_gloo2.out > $OUT/c3_gloo2.json
python3 - <<PY
import json
a = json.load(open("$OUT/c3_gloo2.json")); b = json.load(open("$OUT/bench_driver.json"))["c3_single_gpu"]
print("gloo2", a["n_gpus"], round(a["value"] / 1e9, 1), a["fingerprint"])
print("n1   ", b["fingerprint"])
keys = ("records_sha256", "counts_sha256", "islands", "oracle_match")
print("fingerprints equal:", all(a["fingerprint"][k] == b["fingerprint"][k] for k in keys),
      "oracle_match:", a["fingerprint"]["oracle_match"], b["fingerprint"]["oracle_match"])
print("bw", a["bw_iteration"]["ms_per_iteration"], b["bw_iteration"]["ms_per_iteration"])
PY
