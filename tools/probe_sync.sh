#!/bin/bash
# Round 3 probe: does the serial step ramp too (clocks) or only the overlapped one?
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd); OUT=$R/gpurun_out/sync5; mkdir -p $OUT
export CPG_BENCH_TIMELINE=1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --cold-steps 0 --steps 300 --warmup 5 --serial > $OUT/s300.json 2> $OUT/s300.err || exit $?
grep -A4 timeline $OUT/s300.err | python3 -c "
import sys,ast
for l in sys.stdin:
    if l.startswith('phase'):
        k,v=l.split(':',1); v=ast.literal_eval(v.strip())
        if v: print(k, [round(sum(v[i:i+20])/len(v[i:i+20]),4) for i in range(0,len(v),20)])
    else: print(l.strip())"
