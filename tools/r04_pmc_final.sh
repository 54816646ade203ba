#!/bin/bash
# Round 4 final tree: the PMC profiles bench.py reads (C2, C3, count kernel) regenerated.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; R=$(pwd); OUT=$R/gpurun_out/${TAG:-r04_pmcfinal}; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/pmc_round.sh > $OUT/pmc_round.log 2>&1 || { tail -20 $OUT/pmc_round.log; exit 1; }
cp gpurun_out/pmc_latest.json gpurun_out/pmc_c3.json gpurun_out/pmc_count.json gpurun_out/pmc_summary.txt gpurun_out/pmc_c3_summary.txt gpurun_out/pmc_count_summary.txt $OUT/
cut -c1-220 $OUT/pmc_c3_summary.txt | head -12
