"""E-step kernel time on 46 Mbp at several chunk lengths (dev probe): C = 65536 runs one
1024-lane workgroup per CU (104.5 KB LDS), C = 32768 two 512-lane workgroups per CU (72.5 KB
each), C = 16384 four 256-lane ones.  Same per-position work, so the difference is what
co-resident workgroups (one's prologue / barriers beside another's main loop) buy.
Warmed up for ~40 ms first (the clock ramp, profiles/r03_v1/startup_probe.txt)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("CPG_DEV_PKG"):   # a variant tree from tools/build_variant.sh
    sys.path.insert(0, os.environ["CPG_DEV_PKG"])
import torch  # noqa: E402
from cpgisland_amd import Context, HmmModel  # noqa: E402
from cpgisland_amd import device as D  # noqa: E402
N = int(os.environ.get("N", "46000000"))
dev = torch.device("cuda:0")
p, s = D.synth_host(20251016, 0, N)
dp, ds = D.to_device(p, dev), D.to_device(s, dev)
ctx = Context(0)
ctx.reserve(N)
m = HmmModel.initial()
ec = torch.empty(105, dtype=torch.float64, device=dev)
lc = torch.empty(124, dtype=torch.int64, device=dev)
for _ in range(300):
    D.bw_estep(ctx, m, dp, N, 65536, out=ec)
torch.cuda.synchronize()
for C in (65536, 32768, 16384, 65536, 32768):
    for kind in ("estep", "train"):
        f = (lambda: D.bw_estep(ctx, m, dp, N, C, out=ec)) if kind == "estep" else \
            (lambda: D.train_pass(ctx, m, dp, ds, N, C, estep_out=ec, counts_out=lc))
        for _ in range(5):
            f()
        ts = []
        for _ in range(31):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(); f(); b.record()
            ts.append((a, b))
        torch.cuda.synchronize()
        t = sorted(a.elapsed_time(b) * 1e3 for a, b in ts)
        print(f"C {C:6d} {kind:6s} median {t[15]:7.1f} us  min {t[0]:7.1f}", flush=True)
