"""The WHOLE bench workloads against the oracle — every chunk, not samples.

tests/golden/fingerprints.json holds the oracle's results (oracle/cpg_oracle.c, written by
tests/golden/make_fingerprints.py) over every training and decode chunk of:
  C2  46 Mbp chr21-sized (seed 20251016):   701 training chunks, 43 decode chunks, 527 islands
  C3  3.1 Gbp hg38-sized (seed 20251017): 47,302 training chunks, 2,956 decode chunks; chunks
      2,048.. carry the int32-wrapped island coordinates of CpGIslandFinder.java:287
The GPU tests run the production entry points the bench runs — cpg_train_pass_d (E-step +
labelled counts in one launch; at C3 the >= 2,048-chunk k_estep_chunk_rep form) and
cpg_decode_d (exact Viterbi + island scan; at C3 the > 256-chunk form) — over the whole genome
on one GPU, and compare: labelled int64 counts, sign path, per-chunk scores and island records
bitwise; the E-step within 1e-9 relative plus the fixed-point grid bound per entry.

The CPU tests check the fixture itself: the genome digests against cpg_synth, the decode model
against the reducer of the committed E-step, and sampled chunks against a fresh oracle run.
PARITY UNPINNED: the oracle restates the reference."""
import numpy as np
import pytest

from cpgisland_amd import fingerprint as F

TRAIN = 65536
DECODE = 1 << 20


@pytest.fixture(scope="module")
def fx():
    return F.load()


def _genome(cfg):
    from cpgisland_amd import device as D
    p, s = D.synth_host(cfg["seed"], cfg["start"], cfg["nbases"])
    return p, s


def test_fixture_c2_genome_model_and_sampled_chunks(fx):
    """C2 entry: cpg_synth reproduces the digested genome; the decode model is the oracle's
    reducer applied to the committed E-step; three decode chunks and eight training chunks
    recomputed by the oracle match the per-chunk digests / the chunk geometry."""
    from cpgisland_amd import device as D
    from oracle import coracle as co
    from oracle import pyref as pr
    c = fx["C2"]
    n = c["nbases"]
    p, s = _genome(c)
    assert F.sha256(p[: D.words16(n)]) == c["genome"]["packed_sha256"]
    assert F.sha256(s[: D.words32(n)]) == c["genome"]["sign_sha256"]
    est = F.hex_to_f64(c["train"]["estep_hex"])
    m1 = F.hex_to_f64(c["decode"]["model_hex"])
    assert np.array_equal(co.normalize(est), m1)
    ntr = n // TRAIN
    cnt = np.asarray(c["train"]["counts"], np.int64)
    assert c["train"]["chunks"] == ntr and cnt[:8].sum() == ntr
    assert cnt[8:72].sum() == ntr * (TRAIN - 1) and cnt[120:].sum() == ntr * TRAIN
    dd = c["decode"]
    assert dd["chunks"] == n // DECODE == len(dd["chunk_path_digests"]) == len(dd["scores_hex"])
    sc = F.hex_to_f64(dd["scores_hex"])
    for k in (0, 21, dd["chunks"] - 1):
        o = pr.unpack(p[k * DECODE // 16:(k + 1) * DECODE // 16], DECODE)
        st, best = co.viterbi8(m1, o)
        w = np.packbits((st < 4).astype(np.uint8), bitorder="little").view(np.uint32)
        assert F.chunk_digests(w, 1, DECODE)[0] == dd["chunk_path_digests"][k]
        assert best == sc[k]


def test_fixture_has_both_configs(fx):
    for name, nb, ntr, nde in (("C2", 46_000_000, 701, 43), ("C3", 3_100_000_000, 47302, 2956)):
        c = fx[name]
        assert c["nbases"] == nb and c["train"]["chunks"] == ntr and c["decode"]["chunks"] == nde
        assert len(c["train"]["estep_hex"]) == 105 and len(c["train"]["counts"]) == 124
        assert len(c["decode"]["model_hex"]) == 104
        assert len(c["decode"]["chunk_path_digests"]) == nde
    assert fx["C3"]["decode"]["islands"] > 30000


def _run_whole(ctx, c, p, s):
    """cpg_train_pass_d + cpg_decode_d over the whole genome, as the bench calls them."""
    import torch
    from cpgisland_amd import HmmModel
    from cpgisland_amd import device as D
    dev = torch.device("cuda:0")
    n = c["nbases"]
    pad = np.zeros(8, np.uint32)
    dp = D.to_device(np.concatenate([p[: D.words16(n)], pad]), dev)
    ds = D.to_device(np.concatenate([s[: D.words32(n)], pad]), dev)
    ctx.reserve(n)
    est, cnt = D.train_pass(ctx, HmmModel.initial(), dp, ds, n, TRAIN)
    m1 = HmmModel.from_struct(F.hex_to_f64(c["decode"]["model_hex"]))
    nd = n // DECODE
    sg, sc, out, icnt = D.decode(ctx, m1, dp, nd * DECODE, DECODE, cap=1 << 20,
                                 first_chunk=c["start"] // DECODE)
    torch.cuda.synchronize()
    ctx.sync()                      # every Viterbi block's exactness self-check
    dd = F.decode_digest(sg.cpu().numpy(), sc.cpu().numpy(), D.islands_to_numpy(out, icnt), nd,
                         DECODE, per_chunk=True)
    return est.cpu().numpy(), cnt.cpu().numpy(), dd


def _check(c, est, cnt, dd):
    r = F.compare(c, estep=est, counts=cnt, decode=dd)
    assert r["counts"], "labelled int64 counts differ from the oracle's"
    assert r["estep"], f"E-step outside 1e-9 + grid bound (max rel {r['estep_max_rel_err']})"
    assert r["path"], f"sign path differs in chunks {r.get('path_chunks_differing')}"
    assert r["scores"], [k for k, (a, b) in enumerate(zip(dd["scores_hex"],
                                                          c["decode"]["scores_hex"])) if a != b][:8]
    assert r["records"], (dd["islands"], c["decode"]["islands"])
    assert r["oracle_match"]


@pytest.mark.gpu
def test_c2_whole_genome_equals_oracle(gpu_ctx, fx):
    c = fx["C2"]
    p, s = _genome(c)
    _check(c, *_run_whole(gpu_ctx, c, p, s))


@pytest.mark.gpu
def test_c3_whole_genome_equals_oracle(fx):
    """3.1 Gbp on one GPU: 47,302 training chunks through the k_estep_chunk_rep training pass,
    2,956 decode chunks through the > 256-chunk decode, every one against the oracle."""
    import torch
    from cpgisland_amd import Context
    from cpgisland_amd import device as D
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = fx["C3"]
    p, s = _genome(c)
    assert F.sha256(p[: D.words16(c["nbases"])]) == c["genome"]["packed_sha256"]
    ctx = Context(0)
    try:
        res = _run_whole(ctx, c, p, s)
    finally:
        ctx.close()
    del p, s
    _check(c, *res)
