"""Time the E-step kernel of one libcpg build (CPG_DEV_PKG: a tree made by tools/build_variant.sh) on 46 Mbp (dev tool)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("CPG_DEV_PKG"):   # a variant tree from tools/build_variant.sh
    sys.path.insert(0, os.environ["CPG_DEV_PKG"])
import torch
from cpgisland_amd import Context, HmmModel
from cpgisland_amd import device as D
N = 46_000_000
dev = torch.device("cuda:0")
p, s = D.synth_host(1, 0, N)
dp = D.to_device(p, dev)
ctx = Context(0); ctx.reserve(N)
m = HmmModel.initial()
out = torch.empty(105, dtype=torch.float64, device=dev)
for _ in range(3): D.bw_estep(ctx, m, dp, N, 65536, out=out)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
for _ in range(10):
    a.record(); D.bw_estep(ctx, m, dp, N, 65536, out=out); b.record(); torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
print(os.environ.get("CPG_DEV_PKG", "default"), "estep ms median %.4f min %.4f" % (sorted(ts)[5], min(ts)))
# accuracy of this build on 32 chunks vs the oracle (max relative error over non-zero counts)
import numpy as np
from oracle import coracle as co, pyref as pr
n = 32 * 65536
got = D.bw_estep(ctx, m, dp, n, 65536).cpu().numpy()
ref = co.estep(m.to_struct(), pr.unpack(p, n), 65536)
nz = ref != 0
print("   max rel err vs oracle %.3e" % np.max(np.abs(got[nz] - ref[nz]) / np.abs(ref[nz])))
