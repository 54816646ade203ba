"""Per-phase wall-clock stamps (s_memrealtime, 100 MHz) of the fused training pass's
workgroups, from an ABL_STAMP build (dev tool: CPG_DEV_PKG=build/abl/pkg_stamp)."""
import ctypes
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("CPG_DEV_PKG"):   # a variant tree from tools/build_variant.sh
    sys.path.insert(0, os.environ["CPG_DEV_PKG"])
import numpy as np  # noqa: E402
import torch  # noqa: E402
from cpgisland_amd import Context, HmmModel  # noqa: E402
from cpgisland_amd import device as D  # noqa: E402
from cpgisland_amd import _lib  # noqa: E402
N = int(os.environ.get("N", "46000000"))
dev = torch.device("cuda:0")
p, s = D.synth_host(20251016, 0, N)
dp, ds = D.to_device(p, dev), D.to_device(s, dev)
ctx = Context(0)
ctx.reserve(N)
m = HmmModel.initial()
lc = torch.empty(124, dtype=torch.int64, device=dev)
ec = torch.empty(105, dtype=torch.float64, device=dev)
for _ in range(20):
    D.train_pass(ctx, m, dp, ds, N, 65536, estep_out=ec, counts_out=lc)
torch.cuda.synchronize()
nwg = N // 65536
if nwg >= 2048:   # the long-launch form: four chunks per workgroup (stamps: its last chunk)
    nwg = (nwg + 3) // 4
h = np.zeros(2048 * 12, np.uint64)
lib = ctypes.CDLL(_lib.LIB_PATH)
assert lib.cpg_dbg_stamps(h.ctypes.data_as(ctypes.c_void_p), len(h)) == 0
st = h.reshape(2048, 12)[:nwg].astype(np.int64)
names = ["codes+bar", "counts", "tables+bar", "phase1", "rowscans", "wavescan", "ckpt+bar",
         "zero+bar", "main+bar", "epilogue", "final/end"]
d = np.diff(st, axis=1)
print("median ticks (10 ns):", " ".join(f"{n} {np.median(d[:, i]):.0f}" for i, n in enumerate(names)))
print("mean ticks   (10 ns):", " ".join(f"{n} {np.mean(d[:, i]):.0f}" for i, n in enumerate(names)))
t0 = st[:, 0].min()
print("wg lifetime median", np.median(st[:, 11] - st[:, 0]), "kernel span", st[:, 11].max() - t0)
# workgroups resident at once per CU: lifetime x workgroups / span / CUs
print("mean resident workgroups", float(np.sum(st[:, 11] - st[:, 0]) / (st[:, 11].max() - t0)))
starts = np.sort(st[:, 0] - t0)
print("start quantiles", [int(x) for x in np.quantile(starts, [0, .1, .3, .36, .37, .5, .7, .73, .74, .9, 1])])
