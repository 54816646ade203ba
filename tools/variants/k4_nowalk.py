"""Ablation (timing only, wrong results): K4 segment path without lane 0's walk over the
staged stream (staging, exits and the rest unchanged)."""
import sys
p = sys.argv[1]
s = open(p).read()
old = "        if (t == 0) {\n            double P = init.x, M = init.y;"
assert s.count(old) == 1
s = s.replace(old, "        if (t == 0 && nbar < 0) {\n            double P = init.x, M = init.y;")
open(p, 'w').write(s)
