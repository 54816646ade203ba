"""Print a rocprofv3 kernel_stats.csv compactly (dev tool)."""
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    m = re.search(r'::(k_[a-z0-9_]+)', r['Name'])
    n = m.group(1) if m else r['Name'][:40]
    print(f"{n:26s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1e3:8.2f} min_us={float(r['MinNs'])/1e3:8.2f} tot%={float(r['Percentage']):6.2f}")
