"""Dev tool: build/abl/libcpg_stamp.so — the library with per-phase wall-clock stamps
(s_memrealtime, 100 MHz) in the fused training pass, inserted into a COPY of the sources at
anchor lines (the product sources carry no instrumentation).  Read them with
tools/stamp_estep.py (CPG_DEV_PKG=build/abl/pkg_stamp)."""
import os
import shutil
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(R, "cpgisland_amd", "csrc")
TREE = os.path.join(R, "build", "abl", "stamp_tree")        # csrc + include, same relative layout
DST = os.path.join(TREE, "cpgisland_amd", "csrc")
HEAD = '''__device__ unsigned long long g_stamp[2048 * 12];
#define STAMP(i) do { if (threadIdx.x == 0 && blockIdx.x < 2048) g_stamp[blockIdx.x * 12 + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)
'''
TAIL = '''
namespace cpg {
extern "C" int cpg_dbg_stamps(unsigned long long* h, int n) {
    return (int)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_stamp), (size_t)n * 8);
}
}
'''
# (anchor, stamp index, before|after): the phase boundaries of k_estep_chunk
ANCHORS = [
    ("    const uint32_t* pk = packed + c * (C / 16);\n", 0, "after"),
    ("    // the lane's 64 bases = one count block", 1, "before"),
    ("    // 4-step products: window (b0..b4)", 2, "before"),
    ("    constexpr int L = kLanePos;            // 64 positions per lane", 3, "before"),
    ("    // 2. ", 4, "before"),
    ("    STAMP_ROWS", 5, "before"),
    ("    // every lane is past its 4-step table reads", 6, "before"),
    ("    // 3a. ", 7, "before"),
    ("    // the epilogue's indices from an opaque copy", 9, "before"),
    ("    // done != nullptr: the last workgroup", 10, "before"),
]


def main():
    shutil.rmtree(TREE, ignore_errors=True)
    shutil.copytree(SRC, DST)
    shutil.copytree(os.path.join(R, "include"), os.path.join(TREE, "include"))
    p = os.path.join(DST, "k_estep.hip")
    s = open(p).read()
    s = s.replace("namespace cpg {\nnamespace {\n", "namespace cpg {\nnamespace {\n" + HEAD, 1)
    for a, i, where in ANCHORS:
        if a == "    STAMP_ROWS":   # the barrier after the row / wave scans' shuffles
            a = "    __syncthreads();\n    if (t < 64) {"
        assert s.count(a) >= 1, a
        ins = f"    STAMP({i});\n"
        s = s.replace(a, ins + a if where == "before" else a + ins, 1)
    s = s.replace("        reset_done(done);\n    }\n}", "        reset_done(done);\n    }\n    STAMP(11);\n}", 1)
    s = s.replace("    STAMP(7);\n", "    STAMP(7);\n    STAMP(8);\n", 1)
    s += TAIL
    open(p, "w").write(s)
    base = ("-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function "
            "-Wno-unused-variable --offload-arch=gfx950 -munsafe-fp-atomics " + os.environ.get("STAMP_FLAGS", ""))
    subprocess.run(["make", "-s", "-j8", "-C", DST, "OBJDIR=../../obj",
                    f"OUT={os.path.join(R, 'build', 'abl', os.environ.get('STAMP_OUT', 'libcpg_stamp.so'))}", f"CXXFLAGS={base}", os.path.join(R, 'build', 'abl', os.environ.get('STAMP_OUT', 'libcpg_stamp.so'))],
                   check=True)
    # the package tree that loads it (CPG_DEV_PKG=build/abl/pkg_stamp)
    pkg = os.path.join(R, "build", "abl", "pkg_" + os.environ.get("STAMP_OUT", "libcpg_stamp.so")[7:-3], "cpgisland_amd")
    shutil.rmtree(pkg, ignore_errors=True)
    os.makedirs(pkg)
    for f in os.listdir(os.path.join(R, "cpgisland_amd")):
        if f.endswith(".py"):
            shutil.copy(os.path.join(R, "cpgisland_amd", f), pkg)
    shutil.copy(os.path.join(R, "build", "abl", os.environ.get("STAMP_OUT", "libcpg_stamp.so")),
                os.path.join(pkg, "libcpg.so"))


if __name__ == "__main__":
    sys.exit(main())
