"""Debug: the C3 shard's decode through the direct path at several chunk counts and through
the streamed pipeline; reports which calls fail their self-check (dev tool)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from cpgisland_amd import Context, HmmModel  # noqa: E402
from cpgisland_amd import device as D  # noqa: E402
from cpgisland_amd.dist import shard_bounds  # noqa: E402
from oracle import coracle as co, pyref as pr  # noqa: E402
DEC, TR = 1 << 20, 65536
start, n = shard_bounds(3_100_000_000, 8, 6)
packed, sign = D.synth_host(20251015 + 2, start, n)
m0 = HmmModel.initial()
m1 = HmmModel.from_struct(co.normalize(co.estep(m0.to_struct(), pr.unpack(packed, 8 * TR), TR)))
dev = torch.device("cuda:0")
dp = D.to_device(np.concatenate([packed, np.zeros(8, np.uint32)]), dev)
ctx = Context(0)
for rep in range(2):   # first on a fresh context, as tests/test_gpu_c3.py
    try:
        got = D.genome_run(ctx, m0, m1, packed, sign, n, first_chunk=start // DEC)
        print("fresh genome_run", rep, "ok", flush=True)
    except Exception as e:
        print("fresh genome_run", rep, "FAIL", e, flush=True)
for nch in [1, 16, 43, 64, 65, 128, n // DEC]:
    try:
        for off in [0, 64]:
            if off + nch > n // DEC:
                continue
            so, sc = D.viterbi(ctx, m1, dp[off * DEC // 16:], nch * DEC, DEC)
            torch.cuda.synchronize()
            ctx.sync()
        print("direct", nch, "ok", flush=True)
    except Exception as e:
        print("direct", nch, "FAIL", e, flush=True)
for tm in [None, m0]:
    try:
        got = D.genome_run(ctx, tm, m1, packed, sign if tm else None, n, first_chunk=start // DEC)
        print("genome_run train" if tm else "genome_run decode-only", "ok", flush=True)
    except Exception as e:
        print("genome_run", "train" if tm else "decode-only", "FAIL", e, flush=True)
