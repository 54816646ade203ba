"""E-step time vs number of 64 Ki chunks (dev tool): shows the per-round workgroup time and
the grid's round quantisation on 256 CUs."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("CPG_DEV_PKG"):   # a variant tree from tools/build_variant.sh
    sys.path.insert(0, os.environ["CPG_DEV_PKG"])
import torch
from cpgisland_amd import Context, HmmModel
from cpgisland_amd import device as D
dev = torch.device("cuda:0")
NMAX = 1024 * 65536
p, s = D.synth_host(1, 0, NMAX)
dp = D.to_device(p, dev)
ctx = Context(0); ctx.reserve(NMAX)
m = HmmModel.initial()
out = torch.empty(105, dtype=torch.float64, device=dev)
for k in [int(x) for x in os.environ.get("CHUNKS", "64 128 256 384 512 640 702 768 1024").split()]:
    N = k * 65536
    for _ in range(2): D.bw_estep(ctx, m, dp, N, 65536, out=out)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(7):
        a.record(); D.bw_estep(ctx, m, dp, N, 65536, out=out); b.record(); torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    t = sorted(ts)[3]
    print(f"{os.path.basename(os.environ.get('CPG_DEV_PKG', 'default'))} chunks {k:5d} ms {t:.4f} per-chunk-us {t*1e3/k:.3f}", flush=True)
