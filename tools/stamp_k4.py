"""Per-phase wall-clock stamps of K4 (k_vit_chain_seg) workgroups from the stamp build
(dev tool: CPG_LIB_OVERRIDE=build/abl/libcpg_stamp.so, tools/stamp_build.py)."""
import ctypes
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from cpgisland_amd import Context, HmmModel  # noqa: E402
from cpgisland_amd import device as D  # noqa: E402
from cpgisland_amd import _lib  # noqa: E402
N = int(os.environ.get("N", "46000000"))
dev = torch.device("cuda:0")
p, s = D.synth_host(20251016, 0, N)
dp = D.to_device(p, dev)
ctx = Context(0)
ctx.reserve(N)
m = HmmModel.initial()
so = torch.empty(D.words32(N) + 4, dtype=torch.int32, device=dev)
for _ in range(20):
    D.viterbi(ctx, m, dp, N, 1 << 20, sign_out=so)
torch.cuda.synchronize()
nch = N >> 20
h = np.zeros(1024 * 8, np.uint64)
lib = ctypes.CDLL(_lib.LIB_PATH)
assert lib.cpg_dbg_stamps4(h.ctypes.data_as(ctypes.c_void_p), len(h)) == 0
st = h.reshape(1024, 8)[:nch, :6].astype(np.int64)
names = ["A:list", "B1:loads", "B2+stage", "chain", "D+E"]
d = np.diff(st, axis=1)
print("K4 median ticks (10 ns):", " ".join(f"{n} {np.median(d[:, i]):.0f}" for i, n in enumerate(names)))
print("K4 max ticks    (10 ns):", " ".join(f"{n} {np.max(d[:, i]):.0f}" for i, n in enumerate(names)))
t0 = st[:, 0].min()
print("K4 start spread", int(st[:, 0].max() - t0), "end", int(st[:, 5].max() - t0))
