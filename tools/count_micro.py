"""Labelled counts of one libcpg build (CPG_DEV_PKG: a tree made by tools/build_variant.sh) repeated on 46 Mbp, for rocprofv3
kernel statistics of ablation variants (dev tool; results not checked)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("CPG_DEV_PKG"):   # a variant tree from tools/build_variant.sh
    sys.path.insert(0, os.environ["CPG_DEV_PKG"])
import torch  # noqa: E402
from cpgisland_amd import Context  # noqa: E402
from cpgisland_amd import device as D  # noqa: E402
N = 46_000_000
dev = torch.device("cuda:0")
p, s = D.synth_host(20251016, 0, N)
dp, ds = D.to_device(p, dev), D.to_device(s, dev)
ctx = Context(0)
ctx.reserve(N)
for _ in range(int(os.environ.get("REPS", "5"))):
    D.count_labelled(ctx, dp, ds, N)
torch.cuda.synchronize()
print("ok", os.environ.get("CPG_DEV_PKG", "default"))
