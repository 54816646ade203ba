"""Diagnostic (development only): K4 (k_vit_chain_seg) prints, for the first 256 chunks, its
barrier count, staged window steps, SEQ/SPLIT counts and the clock64 ticks (2.4 GHz) of
phases A-B, phase C's staging, its walk, and phases D-E, from thread 0."""
import sys
p = sys.argv[1]
s = open(p).read()
i0 = s.index("k_vit_chain_seg(")
h = "    const int t = threadIdx.x;\n"
j = s.index(h, i0) + len(h)
s = s[:j] + "    const long long tcS = clock64(), wS = wall_clock64();\n" + s[j:]
a = "    // C. the serial chain over the barriers (k_vit_chain's phase 3)\n"
assert s.count(a) == 1
s = s.replace(a, "    const long long tcA = clock64();\n" + a)
w = "    if (all_staged) {\n"
j = s.index(w, i0)
s = s[:j] + "    const long long tcB = clock64();\n" + s[j:]
b = "    __syncthreads();\n    // D. anchor values by block id"
assert s.count(b) == 1
s = s.replace(b, "    __syncthreads();\n    const long long tcC = clock64();\n    // D. anchor values by block id")
e = "        if (t < nseg) went[s0 + t] = E;\n        else ent[g.nsb] = E;\n    }\n"
j = s.index(e, i0) + len(e)
s = s[:j] + """    __syncthreads();
    if (t == 0 && c < 256) {
        int nseq = 0, nspl = 0, wmax = 0;
        for (int i = 0; i < nst; ++i) {
            nseq += sPt[i] == PLAN_SEQ;
            nspl += sPt[i] == PLAN_SPLIT;
            wmax = max(wmax, sWb[i] - sWa[i]);
        }
        printf("K4DIAG c=%d nbar=%d nst=%d steps=%d seq=%d split=%d wmax=%d staged=%d ab=%lld stage=%lld walk=%lld de=%lld w0=%lld w1=%lld\\n",
               (int)c, nbar, nst, sWoff[nst], nseq, nspl, wmax, (int)all_staged,
               tcA - tcS, tcB - tcA, tcC - tcB, clock64() - tcC, wS, wall_clock64());
    }
""" + s[j:]
open(p, 'w').write(s)
