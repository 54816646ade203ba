"""Config C5 at its size: one 3.1 Gbp (hg38-sized) synthetic genome in PINNED host DRAM,
streamed through cpg_genome_run (the multi-genome batch runs one such genome per GPU).

Checks: the streamed E-step, labelled counts, decoded path, per-chunk
scores and island records equal the unstreamed "_d" calls over the same genome resident in
HBM (counts bitwise: fixed-point accumulators finalized once); count identities of the chunk
geometry; the decoded path's log-probability equals the reported score on sampled chunks;
the first and the last decode chunk against the oracle (8-state Mahout-order Viterbi + the
:262-339 scan with the global chunk index: the last chunk, 2956, is past the int32 coordinate
wrap at chunk 2048, :287).  Every call goes through the C-ABI (libcpg.so)."""
import numpy as np
import pytest

from oracle import coracle as co
from oracle import pyref as pr

pytestmark = pytest.mark.gpu
DECODE = 1 << 20
TRAIN = 65536
G = 3_100_000_000


def _pinned_copy(a):
    import torch
    t = torch.from_numpy(a.view(np.int32)).pin_memory()
    return t, t.numpy().view(np.uint32)


def test_c5_one_genome_streamed_from_pinned_host(gpu_ctx):
    import torch
    from cpgisland_amd import HmmModel
    from cpgisland_amd import device as D
    dev = torch.device("cuda:0")
    p0, s0 = D.synth_host(20251015 + 4, 0, G)
    tp, packed = _pinned_copy(p0)
    ts, sign = _pinned_copy(s0)
    del p0, s0
    m0 = HmmModel.initial()
    m1 = HmmModel.from_struct(co.normalize(co.estep(m0.to_struct(), pr.unpack(packed, 8 * TRAIN),
                                                    TRAIN)))
    got = D.genome_run(gpu_ctx, m0, m1, packed, sign, G, island_cap=1 << 21)
    nd, nt = G // DECODE, G // TRAIN
    # the same genome resident in HBM, through the per-call entry points
    pad = np.zeros(8, np.uint32)
    dp = D.to_device(np.concatenate([packed, pad]), dev)
    ds = D.to_device(np.concatenate([sign, pad]), dev)
    est = D.bw_estep(gpu_ctx, m0, dp, G, TRAIN).cpu().numpy()
    cnt = D.count_labelled(gpu_ctx, dp, ds, G, TRAIN).cpu().numpy()
    del ds
    so, sc, out, c = D.decode(gpu_ctx, m1, dp, G, DECODE, cap=1 << 21)
    torch.cuda.synchronize()
    gpu_ctx.sync()                        # every Viterbi block's exactness self-check
    isl = D.islands_to_numpy(out, c)
    scs = sc.cpu().numpy()[:nd]
    sw = so.cpu().numpy().view(np.uint32)
    del dp, so
    assert np.array_equal(got["estep"], est) and np.array_equal(got["counts"], cnt)
    assert np.array_equal(got["scores"], scs)
    assert got["island_count"] == len(isl) and np.array_equal(got["islands"], isl)
    assert np.array_equal(got["sign_out"][: D.words32(G)], sw[: D.words32(G)])
    assert (isl["beg1"] < 0).any()        # coordinates wrapped as Java ints (:287)
    # count identities of the chunk geometry
    assert cnt[:8].sum() == nt and cnt[8:72].sum() == nt * (TRAIN - 1)
    assert abs(est[:8].sum() - nt) < 1e-6 * nt
    assert abs(est[8:72].sum() - nt * (TRAIN - 1)) < 1e-6 * nt * TRAIN
    # the undecoded tail (G mod 2^20 bases) reads '-'
    tail = pr.unpack_bits(sw[nd * DECODE // 32: D.words32(G)], G - nd * DECODE)
    assert not tail.any()
    # path score == reported score on sampled chunks
    m = m1.to_struct()
    L = np.log(m[8:72].reshape(8, 8))
    for k in list(range(0, nd, 211)) + [nd - 1]:
        o = pr.unpack(packed[k * DECODE // 16:(k + 1) * DECODE // 16], DECODE).astype(np.int64)
        sg = pr.unpack_bits(sw[k * DECODE // 32:(k + 1) * DECODE // 32], DECODE)
        s = o + np.where(sg != 0, 0, 4)
        v = np.log(m[s[0]]) + L[s[:-1], s[1:]].sum()
        assert abs(v - scs[k]) <= 1e-9 * abs(scs[k]), k
    # the first and the last chunk against the oracle, with their global chunk index
    for k in (0, nd - 1):
        o = pr.unpack(packed[k * DECODE // 16:(k + 1) * DECODE // 16], DECODE)
        st, best = co.viterbi8(m, o)
        sg = pr.unpack_bits(sw[k * DECODE // 32:(k + 1) * DECODE // 32], DECODE)
        assert np.array_equal(sg, (st < 4).astype(np.uint8))
        assert scs[k] == best
        assert np.array_equal(isl[isl["chunk"] == k], co.islands(st, k))
