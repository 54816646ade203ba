"""Config C3 (3.1 Gbp hg38-sized genome over 8 GPUs) at its per-GPU shard size on one GPU:
the shard of rank 6 (387.5 Mbp starting past chunk 2048, where the reference's int32 island
coordinates wrap).  The streamed pipeline and the per-call device path agree bitwise; the
decoded path's log-probability equals the reported score on sampled chunks; two chunks are
checked against the oracle (8-state Mahout-order Viterbi + the :262-339 scan with the global
chunk index, so the coordinate wrap is exercised); count identities of the chunk geometry."""
import numpy as np
import pytest

from oracle import coracle as co
from oracle import pyref as pr

pytestmark = pytest.mark.gpu
DECODE = 1 << 20
TRAIN = 65536
G = 3_100_000_000


@pytest.fixture(scope="module")
def shard():
    from cpgisland_amd import device as D
    from cpgisland_amd.dist import shard_bounds
    start, n = shard_bounds(G, 8, 6)
    assert start // DECODE > 2048           # past the int32 coordinate wrap
    packed, sign = D.synth_host(20251015 + 2, start, n)
    return start, n, packed, sign


def test_c3_shard_stream_equals_calls_and_oracle(gpu_ctx, shard):
    import torch
    from cpgisland_amd import HmmModel
    from cpgisland_amd import device as D
    start, n, packed, sign = shard
    dev = torch.device("cuda:0")
    m0 = HmmModel.initial()
    m1 = HmmModel.from_struct(co.normalize(co.estep(m0.to_struct(), pr.unpack(packed, 8 * TRAIN),
                                                    TRAIN)))
    fc = start // DECODE
    got = D.genome_run(gpu_ctx, m0, m1, packed, sign, n, first_chunk=fc)
    pad = np.zeros(8, np.uint32)
    dp = D.to_device(np.concatenate([packed, pad]), dev)
    ds = D.to_device(np.concatenate([sign, pad]), dev)
    est = D.bw_estep(gpu_ctx, m0, dp, n, TRAIN).cpu().numpy()
    cnt = D.count_labelled(gpu_ctx, dp, ds, n, TRAIN).cpu().numpy()
    so, sc = D.viterbi(gpu_ctx, m1, dp, n, DECODE)
    out, c = D.islands(gpu_ctx, dp, so, n, DECODE, first_chunk=fc)
    torch.cuda.synchronize()
    gpu_ctx.sync()                        # every Viterbi block's exactness self-check
    isl = D.islands_to_numpy(out, c)
    nd = n // DECODE
    assert np.array_equal(got["estep"], est) and np.array_equal(got["counts"], cnt)
    assert np.array_equal(got["scores"], sc.cpu().numpy()[:nd])
    assert np.array_equal(got["islands"], isl)
    sw = so.cpu().numpy().view(np.uint32)
    assert np.array_equal(got["sign_out"][: D.words32(n)], sw[: D.words32(n)])
    assert (isl["beg1"] < 0).any()        # coordinates wrapped as Java ints
    # count identities of the chunk geometry
    nch = n // TRAIN
    assert cnt[:8].sum() == nch and cnt[8:72].sum() == nch * (TRAIN - 1)
    assert abs(est[:8].sum() - nch) < 1e-6 * nch
    # path score == reported score on sampled chunks
    obs = pr.unpack(packed, n)
    sg = pr.unpack_bits(sw, n)
    m = m1.to_struct()
    L = np.log(m[8:72].reshape(8, 8))
    scs = sc.cpu().numpy()
    for k in range(0, nd, 37):
        if scs[k] == -np.inf:             # degenerate chunk: compared with the oracle below
            continue
        o = obs[k * DECODE:(k + 1) * DECODE].astype(np.int64)
        s = o + np.where(sg[k * DECODE:(k + 1) * DECODE] != 0, 0, 4)
        v = np.log(m[s[0]]) + L[s[:-1], s[1:]].sum()
        assert abs(v - scs[k]) <= 1e-9 * abs(scs[k])
    # two chunks against the oracle, with their global chunk index, and one degenerate chunk
    # (pi = 0 for both live states of its first base under the 8-chunk-trained model: Mahout's
    # loop keeps every delta at -inf and decodes the all-state-0 path, SURVEY A.2 — parity
    # unpinned, the A.2 start being recalled, not vendored): its sign bits are all '+'
    # (state 0 < 4), its score -inf and its island records none (the whole-chunk run is still
    # open at the chunk end)
    degen = [k for k in range(nd) if scs[k] == -np.inf]
    assert degen, "no degenerate chunk under the 8-chunk model"
    for k in (0, nd - 1, degen[len(degen) // 2]):
        o = obs[k * DECODE:(k + 1) * DECODE]
        st, best = co.viterbi8(m, o)
        assert np.array_equal(sg[k * DECODE:(k + 1) * DECODE], (st < 4).astype(np.uint8))
        assert scs[k] == best
        ref = co.islands(st, fc + k)
        mine = isl[isl["chunk"] == fc + k]
        assert np.array_equal(mine, ref)
