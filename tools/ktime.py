"""Median time (HIP events) of one hot-path phase on 46 Mbp for the libcpg build named by
CPG_DEV_PKG (dev tool).  PHASE = estep | counts | train | viterbi | islands."""
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
so = torch.empty(D.words32(N) + 4, dtype=torch.int32, device=dev)
lc = torch.empty(124, dtype=torch.int64, device=dev)
ec = torch.empty(105, dtype=torch.float64, device=dev)
iout = torch.empty((1 << 20, 32), dtype=torch.uint8, device=dev)
icnt = torch.zeros(1, dtype=torch.int64, device=dev)
D.viterbi(ctx, m, dp, N, 1 << 20, sign_out=so)
ph = {"estep": lambda: D.bw_estep(ctx, m, dp, N, 65536, out=ec),
      "counts": lambda: D.count_labelled(ctx, dp, ds, N, 65536, out=lc),
      "train": lambda: D.train_pass(ctx, m, dp, ds, N, 65536, estep_out=ec, counts_out=lc),
      "viterbi": lambda: D.viterbi(ctx, m, dp, N, 1 << 20, sign_out=so),
      "islands": lambda: D.islands(ctx, dp, so, N, 1 << 20, cap=1 << 20, out=iout, count=icnt)}
name = os.path.basename(os.environ.get("CPG_DEV_PKG", "") or "default")
for phase in os.environ.get("PHASES", "counts").split():
    f = ph[phase]
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(15):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); f(); b.record(); torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    extra = ""
    if phase == "counts":
        import numpy as np
        from oracle import coracle as co, pyref as pr
        n2 = 4 * (1 << 20) + 12345
        got = D.count_labelled(ctx, dp, ds, n2, 65536).cpu().numpy()
        ref = co.count_labelled(pr.unpack(p, n2), pr.unpack_bits(s, n2), 65536)
        extra = "exact" if np.array_equal(got, ref) else "MISMATCH"
    print(f"{name:22s} {phase:8s} median {ts[7]:7.1f} us  min {ts[0]:7.1f} {extra}", flush=True)
