import sys; sys.path.insert(0, '.')
import numpy as np, torch
from cpgisland_amd import HmmModel, Context
from cpgisland_amd import device as D
dev = torch.device("cuda:0"); ctx = Context(0)
m = HmmModel.initial()
for N in [41 * 65536, 41 * 65536 + 77, 9 * 65536 + 77, 2 * 65536]:
    p, s = D.synth_host(77, 0, N)
    dp = D.to_device(p, dev)
    e = D.bw_estep(ctx, m, dp, N).cpu().numpy()
    print(N, e[:4], e[8:10], e[-1])
