"""Development only: one C2 decode through a variant package (CPG_DEV_PKG) built with
tools/variants/k3_ts.py; prints the K3 workgroups' timing summary as JSON."""
import ctypes as C
import json
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.abspath(os.environ["CPG_DEV_PKG"]))
sys.path.insert(1, ROOT)
import numpy as np
import torch
from cpgisland_amd import Context, HmmModel, _lib
from cpgisland_amd import device as D
from cpgisland_amd import fingerprint as F
fx = F.load(os.path.join(ROOT, "tests", "golden", "fingerprints.json"))["C2"]
n = fx["nbases"]
m = HmmModel.from_struct(F.hex_to_f64(fx["decode"]["model_hex"]))
p, _ = D.synth_host(fx["seed"], fx["start"], n)
dev = torch.device("cuda:0")
dp = D.to_device(np.concatenate([p, np.zeros(8, np.uint32)]), dev)
ctx = Context(0)
for _ in range(3):
    D.decode(ctx, m, dp, n, 1 << 20)
torch.cuda.synchronize()
ctx.sync()
ts = np.zeros((16384, 4), np.int64)
assert _lib.lib.cpg_dbg_k3ts(ts.ctypes.data_as(C.c_void_p), 16384) == 0
ctx.close()
ts = ts[ts[:, 0] > 0]
t0 = ts[:, 1].min()
out = {}
for role, name in ((1, "irr"), (2, "main")):
    r = ts[ts[:, 0] == role]
    d = (r[:, 3] - r[:, 1]) / 100.0
    out[name] = {"n": int(len(r)), "start_max_us": float((r[:, 1].max() - t0) / 100),
                 "end_max_us": float((r[:, 3].max() - t0) / 100),
                 "dur_p50_us": float(np.median(d)), "dur_max_us": float(d.max())}
    if role == 1:
        cl = r[r[:, 2] > 0]
        out[name]["scanned"] = int(len(cl))
        if len(cl):
            out[name]["classify_max_us"] = float(((cl[:, 2] - cl[:, 1]) / 100).max())
            out[name]["scanned_dur_max_us"] = float(((cl[:, 3] - cl[:, 1]) / 100).max())
print(json.dumps(out))
