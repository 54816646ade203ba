"""Island scan over many short chunks: cpg_islands_d accepts any chunk length that
is a multiple of 32, so a call can carry hundreds of thousands of chunks.  Each chunk's first
record is found from a scan of the per-chunk kept counts between the two resolve passes
(k_isl_base / k_isl_bscan, k_islands.hip), not by summing every earlier chunk per chunk.
Records against the oracle's :262-339 scan chunk by chunk (CpGIslandFinder.java:262-339; the
coordinates of :287 with the call's chunk length as the stride, int32), and the call's run time
bounded."""
import time

import numpy as np
import pytest

from oracle import coracle as co
from oracle import pyref as pr

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("chunk_len,nch", [(256, 250_000), (1024, 4097), (4096, 4096)])
def test_islands_many_short_chunks(gpu_ctx, chunk_len, nch):
    import torch
    from cpgisland_amd import device as D
    n = chunk_len * nch
    packed, _ = D.synth_host(20251015 + 7, 0, n)
    # short random '+' runs (the planted islands are longer than these chunks): many islands
    # open and close inside every chunk
    rng = np.random.default_rng(chunk_len)
    sign = (rng.integers(0, 2**32, D.words32(n) + 4, dtype=np.uint64) &
            rng.integers(0, 2**32, D.words32(n) + 4, dtype=np.uint64)).astype(np.uint32)
    dev = torch.device("cuda:0")
    dp, ds = D.to_device(packed, dev), D.to_device(sign, dev)
    cap = n // 8
    out, cnt = D.islands(gpu_ctx, dp, ds, n, chunk_len, cap=cap)      # warm (workspace)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out, cnt = D.islands(gpu_ctx, dp, ds, n, chunk_len, cap=cap)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    gpu_ctx.sync()
    got = D.islands_to_numpy(out, cnt)
    assert dt < 0.5, f"{nch} chunks of {chunk_len}: {dt:.3f} s"
    obs = pr.unpack(packed, n).astype(np.int32)
    st = obs + np.where(pr.unpack_bits(sign, n) != 0, 0, 4).astype(np.int32)
    ref = [co.islands(st[c * chunk_len:(c + 1) * chunk_len], c) for c in range(nch)]
    ref = np.concatenate([r for r in ref if len(r)] or [np.zeros(0, co.ISLAND_DTYPE)])
    assert len(got) == len(ref) > 1000
    assert np.array_equal(got, ref)
