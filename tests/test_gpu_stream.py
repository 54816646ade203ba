"""Streamed whole-genome pass (cpg_genome_run, BASELINE config C5) == the unstreamed "_d"
calls over the whole genome: E-step and labelled counts BITWISE (fixed-point accumulators
finalized once), decoded path, per-chunk scores and island records identical, for several
window sizes, buffer counts, ragged tails, and pageable (registered on the fly) host input."""
import numpy as np
import pytest

from oracle import coracle as co
from oracle import pyref as pr

pytestmark = pytest.mark.gpu
DECODE = 1 << 20
TRAIN = 65536


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _unstreamed(ctx, dev, m0, m1, packed, sign, n):
    import torch
    from cpgisland_amd import device as D
    dp = D.to_device(np.concatenate([packed, np.zeros(8, np.uint32)]), dev)
    ds = D.to_device(np.concatenate([sign, np.zeros(8, np.uint32)]), dev)
    est = D.bw_estep(ctx, m0, dp, n, TRAIN).cpu().numpy()
    cnt = D.count_labelled(ctx, dp, ds, n, TRAIN).cpu().numpy()
    so, sc = D.viterbi(ctx, m1, dp, n, DECODE)
    out, c = D.islands(ctx, dp, so, n, DECODE)
    torch.cuda.synchronize()
    ctx.sync()
    return {"estep": est, "counts": cnt, "sign": so.cpu().numpy().view(np.uint32),
            "scores": sc.cpu().numpy()[: n // DECODE], "islands": D.islands_to_numpy(out, c)}


@pytest.mark.parametrize("n,window,nbuf", [
    (37 * DECODE + 12345, 8 * DECODE, 3),
    (37 * DECODE + 12345, 4 * DECODE, 2),
    (37 * DECODE + 12345, 64 * DECODE, 0),     # one window
    (5 * DECODE - 1, 1 * DECODE, 8),           # ragged tail window
    (700000, 0, 0),                            # no decode chunk, 10 train chunks
])
def test_stream_equals_unstreamed(gpu_ctx, torch_dev, n, window, nbuf):
    from cpgisland_amd import HmmModel
    from cpgisland_amd import device as D
    packed, sign = D.synth_host(4242, 0, n)
    m0 = HmmModel.initial()
    m1 = HmmModel.from_struct(co.normalize(co.estep(m0.to_struct(),
                                                    pr.unpack(packed, 4 * TRAIN), TRAIN)))
    ref = _unstreamed(gpu_ctx, torch_dev, m0, m1, packed, sign, n)
    got = D.genome_run(gpu_ctx, m0, m1, packed, sign, n, window_bases=window, nbuf=nbuf)
    assert np.array_equal(got["estep"], ref["estep"])          # bitwise, not 1e-9
    assert np.array_equal(got["counts"], ref["counts"])
    nw = D.words32(n)
    assert np.array_equal(got["sign_out"][:nw], ref["sign"][:nw])
    assert np.array_equal(got["scores"], ref["scores"])
    assert np.array_equal(got["islands"], ref["islands"])


def test_stream_train_only_and_decode_only(gpu_ctx, torch_dev):
    from cpgisland_amd import HmmModel
    from cpgisland_amd import device as D
    n = 9 * DECODE + 3
    packed, sign = D.synth_host(11, 0, n)
    m = HmmModel.initial()
    ref = _unstreamed(gpu_ctx, torch_dev, m, m, packed, sign, n)
    a = D.genome_run(gpu_ctx, m, None, packed, None, n, window_bases=2 * DECODE)
    assert np.array_equal(a["estep"], ref["estep"]) and a["counts"] is None
    b = D.genome_run(gpu_ctx, None, m, packed, None, n, window_bases=2 * DECODE,
                     want_sign_out=False)
    assert b["estep"] is None and np.array_equal(b["islands"], ref["islands"])
    assert np.array_equal(b["scores"], ref["scores"])
