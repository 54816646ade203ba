"""Config C4 at its full size (BASELINE.json configs[3]: 10M ragged contigs of 150 bp - 50 kbp,
~86 Gbases resident in HBM) through the contig entry points (k_contigs.hip), one call each:
  * labelled counts: exact identities of the batch geometry (one init per contig, len - 1
    transitions per contig, every base once in the mononucleotide counts);
  * E-step: the init posteriors sum to one per contig, the transitions to len - 1;
  * Viterbi: the reported score of sampled contigs equals the log-probability of the decoded
    path re-evaluated on the host (1e-9 relative), and 32 contigs (with the longest and the
    shortest) are bitwise the oracle's 8-state Mahout-order Viterbi, path and score;
  * islands: the records of those 32 contigs equal the oracle's :262-339 scan of the oracle's
    states, and every record of the batch satisfies the reference's filter (cg > 0.5,
    oe > 0.6) inside its contig.
The bases are a 2^30-base synthetic genome tiled over the batch span (device copies), as in
tools/bench_contigs.py.  PARITY UNPINNED (see oracle/cpg_oracle.h)."""
import numpy as np
import pytest

from oracle import coracle as co
from oracle import pyref as pr

pytestmark = pytest.mark.gpu
NCONTIG = 10_000_000


@pytest.fixture(scope="module")
def big():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cpgisland_amd import device as D
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(20251019)
    lens = np.exp(rng.uniform(np.log(150), np.log(50000), NCONTIG)).astype(np.int64)
    offs, span = D.contig_layout(lens)
    tile = 1 << 30
    p1, s1 = D.synth_host(20251019, 0, tile)
    wp, ws = tile // 16, tile // 32
    words_p, words_s = D.words16(span) + 8, D.words32(span) + 8
    dp = torch.empty(words_p, dtype=torch.int32, device=dev)
    ds = torch.empty(words_s, dtype=torch.int32, device=dev)
    tp, tsg = D.to_device(p1[:wp], dev), D.to_device(s1[:ws], dev)
    for i in range(0, words_p, wp):
        k = min(wp, words_p - i)
        dp[i:i + k].copy_(tp[:k])
    for i in range(0, words_s, ws):
        k = min(ws, words_s - i)
        ds[i:i + k].copy_(tsg[:k])
    del tp, tsg
    yield {"lens": lens, "offs": offs, "span": span, "dp": dp, "ds": ds, "dev": dev,
           "d_offs": torch.from_numpy(offs).to(dev),
           "d_lens": torch.from_numpy(lens.astype(np.int32)).to(dev)}
    del dp, ds
    torch.cuda.empty_cache()


def _bases(b, c, plane="dp"):
    """Contig c's bases (plane dp) or bits (a sign buffer) from the device buffers."""
    from cpgisland_amd import device as D
    o, L = int(b["offs"][c]), int(b["lens"][c])
    if plane == "dp":
        w = b["dp"][o // 16: o // 16 + D.words16(L)].cpu().numpy().view(np.uint32)
        return pr.unpack(w, L)
    w = plane[o // 32: o // 32 + D.words32(L)].cpu().numpy().view(np.uint32)
    return pr.unpack_bits(w, L)


def test_c4_full_size(gpu_ctx, big):
    import torch
    from cpgisland_amd import HmmModel
    from cpgisland_amd import device as D
    b = big
    n, span, lens = NCONTIG, b["span"], b["lens"]
    m = co.initial_model()
    order = D.contigs_order(gpu_ctx, b["d_lens"], n)
    cnt = D.contigs_count_labelled(gpu_ctx, b["dp"], b["ds"], span, b["d_offs"], b["d_lens"],
                                   order, n).cpu().numpy()
    est = D.contigs_estep(gpu_ctx, HmmModel.from_struct(m), b["dp"], span, b["d_offs"],
                          b["d_lens"], order, n).cpu().numpy()
    so = torch.zeros(D.words32(span) + 8, dtype=torch.int32, device=b["dev"])
    so, sc = D.contigs_viterbi(gpu_ctx, HmmModel.from_struct(m), b["dp"], span, b["d_offs"],
                               b["d_lens"], order, n, sign_out=so)
    out, ic = D.contigs_islands(gpu_ctx, b["dp"], so, span, b["d_offs"], b["d_lens"], order, n,
                                cap=1 << 24)
    torch.cuda.synchronize()
    gpu_ctx.sync()
    total = int(lens.sum())
    assert total > 8e10
    # counts: geometry identities
    assert cnt[:8].sum() == n
    assert cnt[8:72].sum() == total - n
    assert cnt[120:124].sum() == total and cnt[104:120].sum() == total - n
    assert np.array_equal(cnt[72:104].reshape(8, 4).sum(1), cnt[:8] + cnt[8:72].reshape(8, 8).sum(0))
    # E-step: posteriors sum to one per position
    assert abs(est[:8].sum() - n) < 1e-6 * n
    assert abs(est[8:72].sum() - (total - n)) < 1e-6 * total
    sc = sc.cpu().numpy()
    assert np.all(np.isfinite(sc)) and np.all(sc < 0)
    isl = D.islands_to_numpy(out, ic)
    assert len(isl) > 1000
    assert np.all(np.diff(isl["chunk"]) >= 0)
    assert np.all(isl["cg"] > 0.5) and np.all(isl["oe"] > 0.6)
    assert np.all((isl["beg1"] >= 1) & (isl["beg1"] <= isl["end1"]) &
                  (isl["end1"] <= lens[isl["chunk"]]))
    assert np.array_equal(isl["len"], isl["end1"] - isl["beg1"] + 1)
    # sampled contigs: score == the decoded path's log-probability; 32 against the oracle
    rng = np.random.default_rng(4)
    L = np.log(m[8:72].reshape(8, 8))
    for c in rng.choice(n, 200, replace=False):
        o = _bases(b, c).astype(np.int64)
        s = o + np.where(_bases(b, c, so) != 0, 0, 4)
        v = np.log(m[s[0]]) + L[s[:-1], s[1:]].sum()
        assert abs(v - sc[c]) <= 1e-9 * abs(sc[c]), c
    pick = list(rng.choice(n, 30, replace=False)) + [int(np.argmax(lens)), int(np.argmin(lens))]
    for c in pick:
        o = _bases(b, c)
        st, best = co.viterbi8(m, o)
        assert np.array_equal(_bases(b, c, so), (st < 4).astype(np.uint8)), c
        assert sc[c] == best, c
        ref = co.islands(st.astype(np.int32), 0)
        ref["chunk"] = c
        assert np.array_equal(isl[isl["chunk"] == c], ref), c
