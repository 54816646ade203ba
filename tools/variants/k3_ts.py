"""Diagnostic (development only): every K3 (k_vit_exact) workgroup records its role, its
wall_clock64 (100 MHz) start, (K3b) the end of its classification, and its end in a device
table read back by cpg_dbg_k3ts (exported by this variant only)."""
import sys
p = sys.argv[1]
s = open(p).read()
i0 = s.index("__global__ __launch_bounds__(kThreads) void k_vit_exact(")
s = s[:i0] + "__device__ long long g_k3ts[16384][4];\n" + s[i0:]
i0 = s.index("__global__ __launch_bounds__(kThreads) void k_vit_exact(")
h = "    __shared__ int s_emin, s_emax, s_part;\n"
j = s.index(h, i0) + len(h)
s = s[:j] + "    const long long wS = wall_clock64();\n" + s[j:]
old = """                      seg ? (int)(ib % nseg) : -1, sA, sB, comp1, segprod);
        return;"""
assert s.count(old) == 1
s = s.replace(old, """                      seg ? (int)(ib % nseg) : -1, sA, sB, comp1, segprod);
        __syncthreads();
        if (threadIdx.x == 0 && blockIdx.x < 16384) {
            g_k3ts[blockIdx.x][0] = 1; g_k3ts[blockIdx.x][1] = wS; g_k3ts[blockIdx.x][3] = wall_clock64();
        }
        return;""")
old = """    if (threadIdx.x < kThreads / 64) sg.mask[threadIdx.x] = sMask[threadIdx.x];
}"""
assert s.count(old) == 1
s = s.replace(old, """    if (threadIdx.x < kThreads / 64) sg.mask[threadIdx.x] = sMask[threadIdx.x];
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x < 16384) {
        g_k3ts[blockIdx.x][0] = 2; g_k3ts[blockIdx.x][1] = wS; g_k3ts[blockIdx.x][3] = wall_clock64();
    }
}""")
# K3b: end of the classification
old = """        __syncthreads();   // (the list and the entries: global writes of this workgroup)
"""
assert s.count(old) == 1
s = s.replace(old, old + """        if (threadIdx.x == 0 && blockIdx.x < 16384) g_k3ts[blockIdx.x][2] = wall_clock64();
""")
s += """
extern "C" int cpg_dbg_k3ts(long long* host, int n) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(cpg::g_k3ts), (size_t)n * 4 * sizeof(long long));
}
"""
open(p, 'w').write(s)
