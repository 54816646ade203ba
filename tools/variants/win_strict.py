"""Variant (development only): K3b's window rule as before round 6's relaxation — every
candidate of every step inside the binade (the window then also covers the steps where only
a clearly losing candidate has left it)."""
import sys
p = sys.argv[1]
s = open(p).read()
old = """            const bool regA = okA && vmax <= HA && vmin > LA && (lP > LA || wP - lP > MA) &&
                              (lM > LA || wM - lM > MA);
            const bool regB = okB && vmax <= HB && vmin > LB && (lP > LB || wP - lP > MB) &&
                              (lM > LB || wM - lM > MB);"""
assert s.count(old) == 1
s = s.replace(old, """            const int64_t vlo = min(vmin, min(lP, lM));
            const bool regA = okA && vmax <= HA && vlo > LA;
            const bool regB = okB && vmax <= HB && vlo > LB;""")
open(p, 'w').write(s)
