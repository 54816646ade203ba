"""The decode alone (cpg_decode_d: exact Viterbi + island scan) over the whole
HBM-resident 3.1 Gbp C3 genome on one GPU, event-timed, for rocprofv3 kernel statistics of
the decode kernels at scale (dev tool).  Prints one JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.environ.get("CPG_DEV_PKG"):   # a variant tree from tools/build_variant.sh
    sys.path.insert(0, os.environ["CPG_DEV_PKG"])
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
import torch  # noqa: E402

from cpgisland_amd import Context, HmmModel, baumwelch  # noqa: E402
from cpgisland_amd import device as D  # noqa: E402

N = int(os.environ.get("BASES", "3100000000"))
REPS = int(os.environ.get("REPS", "5"))
SEP = os.environ.get("SEPARATE", "") == "1"   # Viterbi and island scan as two calls
IGN = os.environ.get("IGNORE_STATUS", "") == "1"   # ablation builds: time only
DEC = 1 << 20
dev = torch.device("cuda:0")
t0 = time.time()
p, s = D.synth_host(20251015 + 2, 0, N)
dp = D.to_device(p, dev)
del p, s
ctx = Context(0)
ctx.reserve(N)
e0 = D.bw_estep(ctx, HmmModel.initial(), dp, N, 65536)
m1 = baumwelch.normalize(e0.cpu().numpy())
nd = N // DEC
so = torch.empty(D.words32(N) + 4, dtype=torch.int32, device=dev)
sc = torch.empty(nd, dtype=torch.float64, device=dev)
cap = nd * 64
iout = torch.empty((cap, 32), dtype=torch.uint8, device=dev)
icnt = torch.zeros(1, dtype=torch.int64, device=dev)


def sync():
    try:
        ctx.sync()
    except Exception:   # ablation builds produce wrong paths by construction
        if not IGN:
            raise


def run():
    if SEP:
        D.viterbi(ctx, m1, dp, N, DEC, sign_out=so, score=sc)
        D.islands(ctx, dp, so, N, DEC, cap=cap, out=iout, count=icnt)
    else:
        D.decode(ctx, m1, dp, N, DEC, cap=cap, sign_out=so, score=sc, out=iout, count=icnt)


for _ in range(2):
    run()
torch.cuda.synchronize()
sync()
ev = []
for _ in range(REPS):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    run()
    b.record()
    ev.append((a, b))
torch.cuda.synchronize()
sync()
ms = sorted(a.elapsed_time(b) for a, b in ev)[REPS // 2]
print(json.dumps({"tool": "decode_c3", "separate": SEP, "bases": N, "decode_chunks": nd, "ms_median": ms,
                  "Gbase_s": N / ms / 1e6, "islands": int(icnt.item()),
                  "setup_s": round(time.time() - t0, 1)}), flush=True)
ctx.close()
