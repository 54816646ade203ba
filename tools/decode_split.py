"""Probe (dev tool): does the C3 decode gain from running two halves of the genome on two
streams, offset so that one half's LDS-bound kernels (K3) overlap the other's VALU-bound ones
(K1, K5)?  Two contexts (separate workspaces), the halves' chunks contiguous; a torch sleep
kernel delays the second half.  Prints one JSON line of median times (ms)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
import torch  # noqa: E402

from cpgisland_amd import Context, HmmModel, baumwelch  # noqa: E402
from cpgisland_amd import device as D  # noqa: E402

DEC = 1 << 20
ND = int(os.environ.get("CHUNKS", "2956"))
REPS = int(os.environ.get("REPS", "5"))
N = ND * DEC
dev = torch.device("cuda:0")
p, s = D.synth_host(20251015 + 2, 0, N)
dp = D.to_device(p, dev)
del p, s
ctxs = [Context(0), Context(0)]
for c in ctxs:
    c.reserve(N)
e0 = D.bw_estep(ctxs[0], HmmModel.initial(), dp, N, 65536)
m1 = baumwelch.normalize(e0.cpu().numpy())
h = ND // 2
parts = [(0, h), (h, ND - h)]
bufs = []
for c0, n in parts:
    so = torch.empty(D.words32(n * DEC) + 4, dtype=torch.int32, device=dev)
    sc = torch.empty(n, dtype=torch.float64, device=dev)
    io = torch.empty((n * 64, 32), dtype=torch.uint8, device=dev)
    ic = torch.zeros(1, dtype=torch.int64, device=dev)
    bufs.append((so, sc, io, ic))
sos = torch.empty(D.words32(N) + 4, dtype=torch.int32, device=dev)
scs = torch.empty(ND, dtype=torch.float64, device=dev)
ios = torch.empty((ND * 64, 32), dtype=torch.uint8, device=dev)
ics = torch.zeros(1, dtype=torch.int64, device=dev)
streams = [torch.cuda.Stream(), torch.cuda.Stream()]


def half(i):
    c0, n = parts[i]
    so, sc, io, ic = bufs[i]
    D.decode(ctxs[i], m1, dp[c0 * DEC // 16:], n * DEC, DEC, cap=n * 64, first_chunk=c0,
             sign_out=so, score=sc, out=io, count=ic)


def whole():
    D.decode(ctxs[0], m1, dp, N, DEC, cap=ND * 64, sign_out=sos, score=scs, out=ios, count=ics)


# sleep calibration: ms per 1e6 cycles
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda._sleep(1000)
a.record()
torch.cuda._sleep(1_000_000)
b.record()
torch.cuda.synchronize()
ms_per_mcyc = a.elapsed_time(b)


def split(delay_ms):
    main = torch.cuda.current_stream()
    for st in streams:
        st.wait_stream(main)
    with torch.cuda.stream(streams[0]):
        half(0)
    with torch.cuda.stream(streams[1]):
        if delay_ms > 0:
            torch.cuda._sleep(int(delay_ms / ms_per_mcyc * 1e6))
        half(1)
    for st in streams:
        main.wait_stream(st)


def timed(fn):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    ev = []
    for _ in range(REPS):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        ev.append((a, b))
    torch.cuda.synchronize()
    for c in ctxs:
        c.sync()
    return round(sorted(x.elapsed_time(y) for x, y in ev)[REPS // 2], 4)


MODE = os.environ.get("MODE", "")   # "whole" / "halves": only that form (for rocprofv3 stats)
out = {"tool": "decode_split", "chunks": ND, "ms_per_Mcycle_sleep": ms_per_mcyc}
if MODE in ("", "whole"):
    out["whole"] = timed(whole)
if MODE in ("", "halves"):
    out["halves_serial"] = timed(lambda: (half(0), half(1)))
if MODE == "":
    for d in (0.0, 0.3):
        out[f"split_delay_{d}"] = timed(lambda: split(d))
out["islands_whole"] = int(ics.item())
out["islands_halves"] = int(bufs[0][3].item()) + int(bufs[1][3].item())
print(json.dumps(out), flush=True)
for c in ctxs:
    c.close()
