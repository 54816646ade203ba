#!/bin/bash
# A/B of the untimed warm-up floor (bench.py --settle-ms) at the driver's command
# (--steps 20 --warmup 5), alternating, against the 400-step default.
set -o pipefail
mkdir -p gpurun_out/settle
O=gpurun_out/settle
for r in 1 2; do
  for s in 0 50 100 200; do
    timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --settle-ms $s --no-cpu-baseline --cold-steps 0 \
      > $O/s${s}_r${r}.json 2> $O/s${s}_r${r}.err || exit 1
    python3 -c "import json;d=json.load(open('$O/s${s}_r${r}.json'));print('settle',$s,'rep',$r,round(d['value']/1e9,1),'Gb/s',round(d['ms_per_step'],4),'ms warm',d['warmup_steps_run'])"
  done
done
timeout -k 10 150 python3 bench.py --no-cpu-baseline --cold-steps 0 --settle-ms 0 > $O/d400.json 2> $O/d400.err || exit 1
python3 -c "import json;d=json.load(open('$O/d400.json'));print('400 steps',round(d['value']/1e9,1),'Gb/s',round(d['ms_per_step'],4),'ms')"
