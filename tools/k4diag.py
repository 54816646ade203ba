"""Development only: one C2 decode through a variant package (CPG_DEV_PKG) built with
tools/variants/k4_diag.py; the device printf lines go to stdout."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.abspath(os.environ["CPG_DEV_PKG"]))
sys.path.insert(1, ROOT)
import numpy as np
import torch
from cpgisland_amd import Context, HmmModel
from cpgisland_amd import device as D
from cpgisland_amd import fingerprint as F
fx = F.load(os.path.join(ROOT, "tests", "golden", "fingerprints.json"))["C2"]
n = fx["nbases"]
m = HmmModel.from_struct(F.hex_to_f64(fx["decode"]["model_hex"]))
p, _ = D.synth_host(fx["seed"], fx["start"], n)
dev = torch.device("cuda:0")
dp = D.to_device(np.concatenate([p, np.zeros(8, np.uint32)]), dev)
ctx = Context(0)
D.decode(ctx, m, dp, n, 1 << 20)
torch.cuda.synchronize()
ctx.sync()
ctx.close()
print("done", flush=True)
