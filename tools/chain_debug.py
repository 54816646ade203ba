import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from cpgisland_amd import Context, HmmModel
from cpgisland_amd import device as D
N = 2 << 20
p, s = D.synth_host(20251016, 0, N)
ctx = Context(0)
so, sc = D.viterbi(ctx, HmmModel.initial(), D.to_device(p, torch.device("cuda:0")), N)
torch.cuda.synchronize()
