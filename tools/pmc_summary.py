"""Summarise rocprofv3 counter_collection CSVs per kernel (mean over dispatches).

usage: python tools/pmc_summary.py gpurun_out/pmc [out.json]

Counters are rocprofv3's per-dispatch values (summed over XCDs/SEs).  SQ_*CYCLES and SQ_WAIT_*
count quad-cycles (MI355X_MICROARCH.md, PMC slots).  HBM traffic per dispatch follows the
guide's HBM section: FETCH_SIZE (KB) is doubled on gfx950 for 16-B/lane streaming reads,
WRITE_SIZE (KB) taken as is.  With a second argument, a JSON of per-kernel traffic bytes and
durations is written (bench.py reads it for roofline.traffic).
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

base = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in glob.glob(f"{base}/p*/p*_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        m = re.search(r'::(k_[a-z0-9_]+)', r['Kernel_Name'])
        if not m:
            continue
        vals[m.group(1)][r['Counter_Name']].append(float(r['Counter_Value']))
for f in glob.glob(f"{base}/p1/p1_kernel_trace.csv"):
    for r in csv.DictReader(open(f)):
        m = re.search(r'::(k_[a-z0-9_]+)', r['Kernel_Name'])
        if m:
            dur[m.group(1)].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)

out = {}
for k in sorted(vals, key=lambda k: -sum(dur.get(k, [0]))):
    v = {c: sum(x) / len(x) for c, x in vals[k].items()}
    d = sum(dur.get(k, [0])) / max(1, len(dur.get(k, [1])))
    wc = v.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    frac = lambda c: v.get(c, 0.0) / wc
    fetch = 2 * v.get("FETCH_SIZE", 0.0) * 1024
    write = v.get("WRITE_SIZE", 0.0) * 1024
    waves = v.get("SQ_WAVES", 0.0) or 1.0
    print(f"{k:20s} dur_us={d:7.1f} waves={waves:7.0f} valu/wave={v.get('SQ_INSTS_VALU', 0) / waves:7.0f} "
          f"lds/wave={v.get('SQ_INSTS_LDS', 0) / waves:6.0f} | active={frac('SQ_ACTIVE_INST_ANY'):.2f} "
          f"wait={frac('SQ_WAIT_ANY'):.2f} issue-stall={frac('SQ_WAIT_INST_ANY'):.2f} "
          f"(lds-issue {frac('SQ_WAIT_INST_LDS'):.2f}) valu-active={frac('SQ_ACTIVE_INST_VALU'):.2f} "
          f"lds-active={frac('SQ_ACTIVE_INST_LDS'):.2f} | LDS_IDX_ACTIVE={v.get('SQ_LDS_IDX_ACTIVE', 0):.3g} "
          f"BANK_CONFLICT={v.get('SQ_LDS_BANK_CONFLICT', 0):.3g} | HBM read={fetch / 1e6:.2f} MB "
          f"write={write / 1e6:.2f} MB")
    out[k] = {"dur_us": d, "fetch_bytes": fetch, "write_bytes": write,
              "traffic_bytes": fetch + write, **{c: v[c] for c in v}}
if len(sys.argv) > 2:
    import time
    what = sys.argv[4] if len(sys.argv) > 4 else "bench.py --serial"
    json.dump({"bases": int(sys.argv[3]) if len(sys.argv) > 3 else None,
               "collected": time.strftime("%Y-%m-%d") + " tools/pmc_round.sh (" + what + ")",
               "kernels": out}, open(sys.argv[2], "w"), indent=1, sort_keys=True)
