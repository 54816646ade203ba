"""Timeline of an overlapped bench run from a rocprofv3 kernel trace (tools/prof_overlap.sh).

usage: python tools/ovl_timeline.py gpurun_out/ovl

Per kernel: mean duration in the overlapped run.  Per stream (training: E-step / counts /
reduce; decode: Viterbi K1-K7 + islands): mean span per step, busy time (sum of durations)
and idle gaps between consecutive kernels of the stream (launch / dependency bubbles).
"""
import csv
import glob
import re
import sys
from collections import defaultdict

base = sys.argv[1]
rows = []
for f in glob.glob(f"{base}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r'(k_[a-z0-9_]+)', r['Kernel_Name'])
        if not m:
            continue
        rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), m.group(1)))
rows.sort()
if not rows:
    sys.exit("no kernels")
train = lambda k: k.startswith(("k_estep", "k_count", "k_bw", "k_reduce"))
dur = defaultdict(list)
for s, e, k in rows:
    dur[k].append((e - s) / 1e3)
print("kernel                 n    mean_us   min_us")
for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:20s} {len(v):4d} {sum(v) / len(v):9.1f} {min(v):8.1f}")
# steps: a decode step starts at each k_vit_approx
for name, sel, first in (("decode", lambda k: not train(k), "k_vit_approx"),
                         ("train", train, "k_estep_chunk")):
    ks = [r for r in rows if sel(r[2])]
    starts = [i for i, r in enumerate(ks) if r[2] == first]
    spans, busy, gaps = [], [], defaultdict(list)
    for a, b in zip(starts, starts[1:]):
        seg = ks[a:b]
        spans.append((seg[-1][1] - seg[0][0]) / 1e3)
        busy.append(sum(e - s for s, e, _ in seg) / 1e3)
        for (s0, e0, k0), (s1, e1, k1) in zip(seg, seg[1:]):
            gaps[f"{k0}->{k1}"].append((s1 - e0) / 1e3)
    if not spans:
        continue
    n = len(spans)
    print(f"\n{name}: {n} steps  span {sum(spans) / n:.1f} us  busy {sum(busy) / n:.1f} us")
    for g, v in gaps.items():
        print(f"  gap {g:40s} {sum(v) / len(v):7.2f} us")
    if len(starts) > 1:
        per = (ks[starts[-1]][0] - ks[starts[0]][0]) / 1e3 / (len(starts) - 1)
        print(f"  step period (start to start) {per:.1f} us")
