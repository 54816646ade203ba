"""Variant edit of k_count.hip: before each prefetch, wait for the round in flight (vmcnt(0)),
so that a wave has exactly one round of loads in flight while it counts (never two)."""
import sys
p = sys.argv[1]
s = open(p).read()
for r in ("B", "A"):
    old = f"        if (g + step <= gfull) load_round({r}, "
    assert old in s
    s = s.replace(old, "        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)\n" + old)
open(p, 'w').write(s)
