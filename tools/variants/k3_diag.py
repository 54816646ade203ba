"""Diagnostic (development only): every K3 (k_vit_exact) workgroup prints its role and its
wall_clock64 (100 MHz) start and end."""
import sys
p = sys.argv[1]
s = open(p).read()
i0 = s.index("__global__ __launch_bounds__(kThreads) void k_vit_exact(")
h = "    __shared__ int s_emin, s_emax, s_part;\n"
j = s.index(h, i0) + len(h)
s = s[:j] + """    const long long wS = wall_clock64();
    struct K3Diag {
        long long w;
        ~K3Diag() {}
    };
""" + s[j:]
# end of K3b branch
old = """                      seg ? (int)(ib % nseg) : -1, sA, sB, comp1, segprod);
        return;"""
assert s.count(old) == 1
s = s.replace(old, """                      seg ? (int)(ib % nseg) : -1, sA, sB, comp1, segprod);
        __syncthreads();
        if (threadIdx.x == 0) printf("K3DIAG irr %u %lld %lld\\n", blockIdx.x, wS, wall_clock64());
        return;""")
# end of main path: after the SegSum writes (end of kernel body)
old = """    if (threadIdx.x < kThreads / 64) sg.mask[threadIdx.x] = sMask[threadIdx.x];
}"""
assert s.count(old) == 1
s = s.replace(old, """    if (threadIdx.x < kThreads / 64) sg.mask[threadIdx.x] = sMask[threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0) printf("K3DIAG main %u %lld %lld\\n", blockIdx.x, wS, wall_clock64());
}""")
open(p, 'w').write(s)
