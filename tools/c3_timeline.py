"""Per-kernel timeline of the last steps of a C3 bench run from a rocprofv3 kernel trace
(dev tool): start / end relative to the first printed kernel, queue, duration (µs).
usage: python tools/c3_timeline.py <trace dir> [n_kernels]"""
import csv
import glob
import re
import sys

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r'(k_[a-z0-9_]+)', r['Kernel_Name'])
        rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']),
                     m.group(1) if m else r['Kernel_Name'][:30], r['Queue_Id'], r['Grid_Size_X']))
rows.sort()
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
seg = rows[-n:]
t0 = seg[0][0]
for s, e, k, q, g in seg:
    print(f"{k:24s} q={q:>3s} grid={g:>9s} {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}")
