"""Run the E-step of a debug libcpg build (CPG_LIB_OVERRIDE, -DCPG_DEBUG_ESTEP) once on
46 Mbp: the kernel prints per-phase wall-clock ticks for a few chunks (dev tool)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from cpgisland_amd import Context, HmmModel  # noqa: E402
from cpgisland_amd import device as D  # noqa: E402
N = 46_000_000
p, _ = D.synth_host(1, 0, N)
dp = D.to_device(p, torch.device("cuda:0"))
ctx = Context(0)
ctx.reserve(N)
for _ in range(2):
    D.bw_estep(ctx, HmmModel.initial(), dp, N, 65536)
torch.cuda.synchronize()
