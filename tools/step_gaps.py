"""Per-step timeline of a short bench run from a rocprofv3 kernel trace.

usage: python tools/step_gaps.py gpurun_out/tr20

Prints every training-pass and decode step (start, end relative to the first kernel of the
run, µs) so a fixed cost at the start of the timed region shows up as a gap or as slow
early steps.
"""
import csv
import glob
import re
import sys

base = sys.argv[1]
rows = []
for f in glob.glob(f"{base}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r'(k_[a-z0-9_]+)', r['Kernel_Name'])
        name = m.group(1) if m else r['Kernel_Name'][:40]
        rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), name))
rows.sort()
t0 = rows[0][0]
prev_end = t0
print(f"{'kernel':28s} {'start':>10s} {'end':>10s} {'dur':>8s} {'gap':>8s}")
for s, e, k in rows:
    print(f"{k:28s} {(s - t0) / 1e3:10.1f} {(e - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f} "
          f"{(s - prev_end) / 1e3:8.1f}")
    prev_end = max(prev_end, e)
