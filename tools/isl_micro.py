"""Island-scan phase alone, repeated on one decoded path of the bench genome (46 Mbp, the
one-iteration model), for rocprofv3 kernel statistics (dev tool).  Prints the run count and
the mean phase time from HIP events."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("CPG_DEV_PKG"):   # a variant tree from tools/build_variant.sh
    sys.path.insert(0, os.environ["CPG_DEV_PKG"])
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cpgisland_amd import Context, HmmModel, baumwelch  # noqa: E402
from cpgisland_amd import device as D  # noqa: E402

N = int(os.environ.get("BASES", "46000000"))
TRAIN, DECODE = 65536, 1 << 20
dev = torch.device("cuda:0")
p, _ = D.synth_host(20251016, 0, N)
dp = D.to_device(p, dev)
ctx = Context(0)
ctx.reserve(N)
ecnt = torch.empty(105, dtype=torch.float64, device=dev)
D.bw_estep(ctx, HmmModel.initial(), dp, N, TRAIN, out=ecnt)
m1 = baumwelch.normalize(ecnt.cpu().numpy())
so = torch.empty(D.words32(N) + 4, dtype=torch.int32, device=dev)
D.viterbi(ctx, m1, dp, N, DECODE, sign_out=so)
icap = 1 << 20
iout = torch.empty((icap, 32), dtype=torch.uint8, device=dev)
icnt = torch.zeros(1, dtype=torch.int64, device=dev)
reps = int(os.environ.get("REPS", "20"))
D.islands(ctx, dp, so, N, DECODE, cap=icap, out=iout, count=icnt)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    D.islands(ctx, dp, so, N, DECODE, cap=icap, out=iout, count=icnt)
e1.record()
torch.cuda.synchronize()
ndec = N // DECODE
s = so[: ndec * DECODE // 32].cpu().numpy().view(np.uint32).reshape(ndec, -1)
bits = np.unpackbits(s.view(np.uint8), bitorder="little").reshape(ndec, -1).astype(np.int8)
starts = int((np.diff(bits, axis=1, prepend=0) == 1).sum())
print(json.dumps({"islands_ms": e0.elapsed_time(e1) / reps, "runs": starts,
                  "runs_per_chunk": starts / ndec, "islands": int(icnt.item())}))
