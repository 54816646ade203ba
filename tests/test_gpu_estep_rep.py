"""The E-step's long-launch form (k_estep_chunk_rep: >= 2,048 chunks, lane-private rows, four
chunks per workgroup with the model's tables built once) at every chunk length the entry points
accept, and with a chunk count that the four-chunk runs do not divide.

* One chunk repeated 2,048 times: the fixed-point sums are exact integers, so the total is
  2^11 x the single chunk's (a one-chunk launch: the other form) — bitwise, since scaling by a
  power of two commutes with every rounding of the finalize.  Chunks of 4,096 bases run the
  form with a single wave per workgroup (its own row copy).
* 2,049 chunks of 64 Ki: cpg_bw_estep_d / cpg_train_pass_d against the windowed pipeline
  (cpg_genome_run, windows of 1,024 chunks: the other form, the same accumulators) — bitwise.
(k_estep.hip; reference: the BW mapper behind CpGIslandFinder.java:200.)"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
KREP = 2048   # k_estep.hip kEstRepMinChunks


@pytest.mark.parametrize("chunk", [4096, 8192, 65536])
def test_rep_form_repeated_chunk_is_exact_multiple(gpu_ctx, chunk):
    import torch
    from cpgisland_amd import HmmModel
    from cpgisland_amd import device as D
    dev = torch.device("cuda:0")
    packed, sign = D.synth_host(20251015 + 5, 3 * chunk, chunk)
    packed = np.ascontiguousarray(packed[:chunk // 16])   # exactly one chunk's words
    pad = np.zeros(8, np.uint32)
    m0 = HmmModel.initial()
    one = D.bw_estep(gpu_ctx, m0, D.to_device(np.concatenate([packed, pad]), dev), chunk, chunk)
    rp = np.concatenate([np.tile(packed, KREP), pad])
    many = D.bw_estep(gpu_ctx, m0, D.to_device(rp, dev), KREP * chunk, chunk)
    again = D.bw_estep(gpu_ctx, m0, D.to_device(rp, dev), KREP * chunk, chunk)
    torch.cuda.synchronize()
    gpu_ctx.sync()
    one, many = one.cpu().numpy(), many.cpu().numpy()
    assert np.isfinite(one).all() and one[8:72].sum() > 0
    assert np.array_equal(many, one * KREP)
    assert np.array_equal(again.cpu().numpy(), many)   # deterministic


def test_rep_form_ragged_run_equals_windowed_pipeline(gpu_ctx):
    import torch
    from cpgisland_amd import HmmModel
    from cpgisland_amd import device as D
    T = 65536
    nch = KREP + 1   # 2,049: four-chunk runs over a grid of 513 workgroups, the last short
    n = nch * T
    dev = torch.device("cuda:0")
    packed, sign = D.synth_host(20251015 + 6, 0, n)
    pad = np.zeros(8, np.uint32)
    m0 = HmmModel.initial()
    dp = D.to_device(np.concatenate([packed, pad]), dev)
    ds = D.to_device(np.concatenate([sign, pad]), dev)
    est = D.bw_estep(gpu_ctx, m0, dp, n, T)
    et, ct = D.train_pass(gpu_ctx, m0, dp, ds, n, T)
    torch.cuda.synchronize()
    gpu_ctx.sync()
    got = D.genome_run(gpu_ctx, m0, None, packed, sign, n, window_bases=1024 * T,
                       want_sign_out=False)
    assert np.array_equal(est.cpu().numpy(), got["estep"])
    assert np.array_equal(et.cpu().numpy(), got["estep"])
    assert np.array_equal(ct.cpu().numpy(), got["counts"])
