"""Print the headline numbers of a bench.py JSON line (one line per leg)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", round(d["value"] / 1e9, 1), "Gbase/s", "ms/step", round(d["ms_per_step"], 4),
      "phases", d.get("phases_ms"))
print("fingerprint", d.get("fingerprint"))
print("cold_cache", d.get("cold_cache"))
for k in ("c3_single_gpu", "bw_iteration"):
    if isinstance(d.get(k), dict):
        v = d[k]
        print(k, {x: v[x] for x in ("value", "ms_per_step", "phases_ms", "ms_per_iteration",
                                      "decode_ms", "fingerprint") if x in v})
for k in ("roofline", "roofline_count", "roofline_decode"):
    if isinstance(d.get(k), dict):
        v = d[k]
        print(k, {x: v[x] for x in ("achieved", "frac", "ms_median") if x in v})
