"""Experiment (development only): K4 (k_vit_chain_seg) with ~8.5 KB more LDS, touched once."""
import sys
p = sys.argv[1]
s = open(p).read()
i0 = s.index("k_vit_chain_seg(")
h = "    const int t = threadIdx.x;\n"
j = s.index(h, i0) + len(h)
s = s[:j] + "    __shared__ double sPad[1088];\n    for (int i = t; i < 1088; i += kSegT) sPad[i] = (double)i;\n" + s[j:]
e = "        if (t < nseg) went[s0 + t] = E;\n        else ent[g.nsb] = E;\n"
j = s.index(e, i0)
s = s[:j] + "        if (t == 9999) E.x += sPad[t & 1023];\n" + s[j:]
open(p, 'w').write(s)
