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


ESTEP_RTOL = 1e-9        # north_star: fp64 within 1e-9 relative
KREP_MIN_CHUNKS = 2048   # k_estep.hip: launches of >= 2,048 chunks take k_estep_chunk<*, true>


def test_c3_train_pass_production_kernel(gpu_ctx, shard):
    """The training pass every C3 shard runs (cpg_train_pass_d at >= 2,048 chunks: the fused
    k_estep_chunk<true, true>, lane-private 2-step rows): bitwise equal to the separate
    cpg_bw_estep_d + cpg_count_labelled_d over the shard's 5,912 chunks (which the test above
    ties bitwise to the windowed pipeline's non-kRep kernels), and against the oracle: three
    sampled chunks, each repeated 2,048 times so the same production kernel runs — the
    fixed-point sums are exact, so the total is 2,048 x the chunk's result (counts: exactly;
    E-step: within 1e-9 relative plus the derived grid bound, tests/test_gpu_parity.py)."""
    import torch
    from cpgisland_amd import HmmModel
    from cpgisland_amd import device as D
    start, n, packed, sign = shard
    assert n // TRAIN >= KREP_MIN_CHUNKS
    dev = torch.device("cuda:0")
    m0 = HmmModel.initial()
    pad = np.zeros(8, np.uint32)
    dp = D.to_device(np.concatenate([packed, pad]), dev)
    ds = D.to_device(np.concatenate([sign, pad]), dev)
    et, ct = D.train_pass(gpu_ctx, m0, dp, ds, n, TRAIN)
    est = D.bw_estep(gpu_ctx, m0, dp, n, TRAIN)
    cnt = D.count_labelled(gpu_ctx, dp, ds, n, TRAIN)
    torch.cuda.synchronize()
    assert np.array_equal(et.cpu().numpy(), est.cpu().numpy())
    assert np.array_equal(ct.cpu().numpy(), cnt.cpu().numpy())
    et2, ct2 = D.train_pass(gpu_ctx, m0, dp, ds, n, TRAIN)      # deterministic
    assert np.array_equal(et2.cpu().numpy(), et.cpu().numpy())
    del dp, ds
    m = m0.to_struct()
    obs = pr.unpack(packed, n)
    truth = pr.unpack_bits(sign, n)
    wpc, spc = TRAIN // 16, TRAIN // 32
    rep = KREP_MIN_CHUNKS
    nch = n // TRAIN
    for k in (0, nch // 2, nch - 1):
        rp = np.concatenate([np.tile(packed[k * wpc:(k + 1) * wpc], rep), pad])
        rs = np.concatenate([np.tile(sign[k * spc:(k + 1) * spc], rep), pad])
        e, c = D.train_pass(gpu_ctx, m0, D.to_device(rp, dev), D.to_device(rs, dev),
                            rep * TRAIN, TRAIN)
        e, c = e.cpu().numpy(), c.cpu().numpy()
        o1 = obs[k * TRAIN:(k + 1) * TRAIN]
        assert np.array_equal(c, rep * co.count_labelled(o1, truth[k * TRAIN:(k + 1) * TRAIN],
                                                         TRAIN))
        ref = rep * co.estep(m, o1, TRAIN)                          # x 2^11: exact
        d = (o1[:-1].astype(np.int64) | (o1[1:].astype(np.int64) << 2))
        nd = np.bincount(d, minlength=16).astype(np.float64) * rep
        b = np.zeros(105)
        b[:8] = rep * 2.0 ** -63
        for i in range(8):
            for j in range(8):
                b[8 + 8 * i + j] = nd[(i & 3) | ((j & 3) << 2)] * 2.0 ** -47
        for j in range(8):
            b[72 + 4 * j + (j & 3)] = b[j] + sum(b[8 + 8 * i + j] for i in range(8))
        b[104] = rep * 2.0 ** -25
        assert np.array_equal(e == 0, ref == 0)
        err = np.abs(e - ref)
        ok = err <= b + ESTEP_RTOL * np.abs(ref)
        assert ok.all(), (k, np.flatnonzero(~ok), err[~ok], b[~ok])


def test_c3_fused_decode_past_the_tail_fusion(gpu_ctx, shard):
    """cpg_decode_d at the shard's 369 decode chunks (> 256: the separate K6 launch and the
    separate island tile + resolve kernels, cpg_internal.h tail_fusion_pays): bitwise equal
    to cpg_viterbi_d + cpg_islands_at_d, and two sampled chunks (global chunk index past the
    int32 coordinate wrap) against the oracle's 8-state Mahout-order Viterbi + :262-339 scan."""
    import torch
    from cpgisland_amd import HmmModel
    from cpgisland_amd import device as D
    start, n, packed, sign = shard
    nd = n // DECODE
    assert nd > 256
    dev = torch.device("cuda:0")
    m1 = HmmModel.from_struct(co.normalize(co.estep(HmmModel.initial().to_struct(),
                                                    pr.unpack(packed, 64 * TRAIN), TRAIN)))
    fc = start // DECODE
    dp = D.to_device(np.concatenate([packed, np.zeros(8, np.uint32)]), dev)
    sg, sc, out, c = D.decode(gpu_ctx, m1, dp, n, DECODE, cap=1 << 20, first_chunk=fc)
    so, sc2 = D.viterbi(gpu_ctx, m1, dp, n, DECODE)
    out2, c2 = D.islands(gpu_ctx, dp, so, n, DECODE, first_chunk=fc)
    torch.cuda.synchronize()
    gpu_ctx.sync()
    isl = D.islands_to_numpy(out, c)
    w = D.words32(n)
    assert np.array_equal(sg.cpu().numpy()[:w], so.cpu().numpy()[:w])
    assert np.array_equal(sc.cpu().numpy()[:nd], sc2.cpu().numpy()[:nd])
    assert np.array_equal(isl, D.islands_to_numpy(out2, c2))
    assert len(isl) > 1000 and (isl["beg1"] < 0).any()
    bits = pr.unpack_bits(sg.cpu().numpy().view(np.uint32), n)
    m = m1.to_struct()
    scs = sc.cpu().numpy()
    for k in (nd // 3, nd - 2):
        o = pr.unpack(packed[k * DECODE // 16:(k + 1) * DECODE // 16], DECODE)
        st, best = co.viterbi8(m, o)
        assert np.array_equal(bits[k * DECODE:(k + 1) * DECODE], (st < 4).astype(np.uint8))
        assert scs[k] == best
        assert np.array_equal(isl[isl["chunk"] == fc + k], co.islands(st, fc + k))
