"""Compact per-kernel summary of a rocprofv3 kernel_stats.csv (avg us, calls)."""
import csv
import re
import sys

for path in sys.argv[1:]:
    print(path)
    for x in csv.DictReader(open(path)):
        m = re.search(r'(k_\w+|__amd\w+|vectorized\w*|elementwise\w*)', x['Name'])
        n = m.group(1) if m else x['Name'][:30]
        print(f"  {n:28s} {x['Calls']:>4} {float(x['AverageNs'])/1e3:8.1f} us")
