"""Summarise rocprofv3 counter_collection CSVs per kernel (mean over dispatches)."""
import csv, glob, re, sys
from collections import defaultdict
base = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in glob.glob(f"{base}/p*/p*_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        m = re.search(r'::(k_[a-z0-9_]+)', r['Kernel_Name'])
        if not m: continue
        vals[m.group(1)][r['Counter_Name']].append(float(r['Counter_Value']))
for f in glob.glob(f"{base}/p1/p1_kernel_trace.csv"):
    for r in csv.DictReader(open(f)):
        m = re.search(r'::(k_[a-z0-9_]+)', r['Kernel_Name'])
        if m: dur[m.group(1)].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
keys = ["SQ_WAVES","SQ_INSTS_VALU","SQ_INSTS_LDS","SQ_WAVE_CYCLES","SQ_BUSY_CYCLES","SQ_WAIT_INST_LDS",
        "SQ_LDS_BANK_CONFLICT","GRBM_GUI_ACTIVE","SQ_WAIT_ANY","SQ_ACTIVE_INST_ANY","SQ_WAIT_INST_ANY",
        "FETCH_SIZE","WRITE_SIZE","SQ_INSTS_VMEM_RD"]
for k in sorted(vals, key=lambda k: -sum(dur.get(k, [0]))):
    v = {c: sum(x)/len(x) for c, x in vals[k].items()}
    d = sum(dur.get(k,[0]))/max(1,len(dur.get(k,[1])))
    s = " ".join(f"{c.replace('SQ_','')}={v[c]:.3g}" for c in keys if c in v)
    print(f"{k:22s} dur_us={d:8.1f} {s}")
