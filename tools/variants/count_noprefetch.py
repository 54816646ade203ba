"""Variant edit of k_count.hip: full rounds without the ping-pong prefetch (each wave loads a
round, then counts it: one round of loads in flight per wave)."""
import sys
p = sys.argv[1]
s = open(p).read()
a = s.index('    Round A, B;\n    if (g <= gfull) load_round(A,')
b = s.index('    // the grid\'s last, partial round')
s = s[:a] + '''    Round A;
    while (g <= gfull) {
        load_round(A, packed4, sign2, packed, sign, g, lane, zv);
        count_round(A, g, true);
        g += step;
    }
''' + s[b:]
open(p, 'w').write(s)
