"""Ragged contig batches (BASELINE config C4) on the GPU vs the oracle applied per contig:
every contig is one observation sequence with the reference's per-chunk semantics.
Viterbi paths and scores, labelled counts and island records bit-exact; E-step within 1e-9
relative.  Edge lengths (1, 2, 15..17, 63..65, 127..129, 255, 256), log-uniform 150 bp -
50 kbp lengths, padding garbage between contigs, with and without the length schedule.
PARITY UNPINNED (see oracle/cpg_oracle.h)."""
import numpy as np
import pytest

from oracle import coracle as co
from oracle import pyref as pr

pytestmark = pytest.mark.gpu
ESTEP_RTOL = 1e-9


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


EDGE = [1, 2, 3, 15, 16, 17, 63, 64, 65, 127, 128, 129, 255, 256, 1000, 4097]


def make_batch(seed, n_random, gap=17):
    from cpgisland_amd import device as D
    rng = np.random.default_rng(seed)
    lens = np.exp(rng.uniform(np.log(150), np.log(50000), n_random)).astype(np.int64)
    lens = np.concatenate([EDGE, lens])
    rng.shuffle(lens)
    offs, span = D.contig_layout(lens, gap=gap)
    packed, sign = D.synth_host(seed, 0, span + 64)
    return lens, offs, span, packed, sign


@pytest.fixture(scope="module")
def batch(torch_dev):
    from cpgisland_amd import device as D
    lens, offs, span, packed, sign = make_batch(7, 240)
    obs = pr.unpack(packed, span)
    truth = pr.unpack_bits(sign, span)
    pad = np.zeros(8, np.uint32)
    dev = {"packed": D.to_device(np.concatenate([packed, pad]), torch_dev),
           "sign": D.to_device(np.concatenate([sign, pad]), torch_dev),
           "offs": __import__("torch").from_numpy(offs).to(torch_dev),
           "lens": __import__("torch").from_numpy(lens.astype(np.int32)).to(torch_dev)}
    return {"lens": lens, "offs": offs, "span": span, "obs": obs, "truth": truth, "dev": dev}


def _order(ctx, b, use):
    from cpgisland_amd import device as D
    if not use:
        return None
    o = D.contigs_order(ctx, b["dev"]["lens"], len(b["lens"]))
    oo = o.cpu().numpy()
    L = b["lens"][oo]
    assert np.all(L[:-1] >= L[1:]) and np.array_equal(np.sort(oo), np.arange(len(L)))
    return o


@pytest.mark.parametrize("use_order", [True, False])
def test_contig_viterbi_exact(gpu_ctx, batch, use_order):
    import torch
    from cpgisland_amd import HmmModel
    from cpgisland_amd import device as D
    m = co.initial_model()
    d = batch["dev"]
    n = len(batch["lens"])
    so, sc = D.contigs_viterbi(gpu_ctx, HmmModel.from_struct(m), d["packed"], batch["span"],
                               d["offs"], d["lens"], _order(gpu_ctx, batch, use_order), n)
    torch.cuda.synchronize()
    gpu_ctx.sync()
    sg = D.sign_to_numpy(so, batch["span"] + 64)
    sc = sc.cpu().numpy()
    for c in range(n):
        o, L = int(batch["offs"][c]), int(batch["lens"][c])
        st, best = co.viterbi8(m, batch["obs"][o:o + L])
        assert np.array_equal(sg[o:o + L], (st < 4).astype(np.uint8)), c
        assert sc[c] == best, (c, sc[c], best)
        assert not sg[o + L: o + ((L + 63) // 64) * 64].any()     # padding bits are '-'


def test_contig_labelled_counts_exact(gpu_ctx, batch):
    import torch
    from cpgisland_amd import device as D
    d = batch["dev"]
    n = len(batch["lens"])
    got = D.contigs_count_labelled(gpu_ctx, d["packed"], d["sign"], batch["span"], d["offs"],
                                   d["lens"], _order(gpu_ctx, batch, True), n).cpu().numpy()
    torch.cuda.synchronize()
    ref = np.zeros(124, np.int64)
    for c in range(n):
        o, L = int(batch["offs"][c]), int(batch["lens"][c])
        ref += co.count_labelled(batch["obs"][o:o + L], batch["truth"][o:o + L], L)
    assert np.array_equal(got, ref)


def test_contig_estep_tolerance(gpu_ctx, batch):
    import torch
    from cpgisland_amd import HmmModel
    from cpgisland_amd import device as D
    m = co.initial_model()
    d = batch["dev"]
    n = len(batch["lens"])
    e1 = D.contigs_estep(gpu_ctx, HmmModel.from_struct(m), d["packed"], batch["span"], d["offs"],
                         d["lens"], _order(gpu_ctx, batch, True), n).cpu().numpy()
    e2 = D.contigs_estep(gpu_ctx, HmmModel.from_struct(m), d["packed"], batch["span"], d["offs"],
                         d["lens"], None, n).cpu().numpy()
    torch.cuda.synchronize()
    gpu_ctx.sync()
    assert np.array_equal(e1, e2)        # fixed-point sums: independent of the schedule
    ref = np.zeros(105)
    for c in range(n):
        o, L = int(batch["offs"][c]), int(batch["lens"][c])
        ref += co.estep(m, batch["obs"][o:o + L], L)
    nz = ref != 0
    assert np.all(e1[~nz] == 0)
    assert np.max(np.abs(e1[nz] - ref[nz]) / np.abs(ref[nz])) < ESTEP_RTOL


def test_contig_islands_exact(gpu_ctx, batch):
    import torch
    from cpgisland_amd import device as D
    d = batch["dev"]
    n = len(batch["lens"])
    out, cnt = D.contigs_islands(gpu_ctx, d["packed"], d["sign"], batch["span"], d["offs"],
                                 d["lens"], _order(gpu_ctx, batch, True), n)
    torch.cuda.synchronize()
    got = D.islands_to_numpy(out, cnt)
    recs = []
    for c in range(n):
        o, L = int(batch["offs"][c]), int(batch["lens"][c])
        states = batch["obs"][o:o + L].astype(np.int32) + np.where(batch["truth"][o:o + L], 0, 4)
        r = co.islands(states, 0)
        r["chunk"] = c
        recs.append(r)
    ref = np.concatenate(recs)
    assert len(ref) > 20
    assert np.array_equal(got, ref)


def test_contig_layout_violation_reported(gpu_ctx, torch_dev):
    import torch
    from cpgisland_amd import CpgInvalid, HmmModel
    from cpgisland_amd import device as D
    packed, _ = D.synth_host(1, 0, 4096)
    dp = D.to_device(packed, torch_dev)
    offs = torch.tensor([0, 100], dtype=torch.int64, device=torch_dev)     # 100 % 64 != 0
    lens = torch.tensor([50, 50], dtype=torch.int32, device=torch_dev)
    D.contigs_viterbi(gpu_ctx, HmmModel.initial(), dp, 4096, offs, lens, None, 2)
    torch.cuda.synchronize()
    with pytest.raises(CpgInvalid):
        gpu_ctx.sync()


@pytest.mark.parametrize("kind", ["trained", "degenerate_pi"])
def test_contig_viterbi_other_models(gpu_ctx, batch, kind):
    """Trained model (one BW iteration) and a model with pi = 0 for some states: contigs whose
    first base has pi = 0 for both live states decode as the reference does (all '+',
    score -inf: SURVEY.md A.2), the others exactly."""
    import torch
    from cpgisland_amd import HmmModel
    from cpgisland_amd import device as D
    m = co.initial_model()
    if kind == "trained":
        o = batch["obs"][: 8 * 65536]
        m = co.normalize(co.estep(m, o, 65536))
    else:
        m = m.copy()
        m[[0, 4]] = 0.0          # pi(A+) = pi(A-) = 0
        m[:8] /= m[:8].sum()
    d = batch["dev"]
    n = len(batch["lens"])
    so, sc = D.contigs_viterbi(gpu_ctx, HmmModel.from_struct(m), d["packed"], batch["span"],
                               d["offs"], d["lens"], _order(gpu_ctx, batch, True), n)
    torch.cuda.synchronize()
    gpu_ctx.sync()
    sg = D.sign_to_numpy(so, batch["span"] + 64)
    sc = sc.cpu().numpy()
    for c in range(n):
        o, L = int(batch["offs"][c]), int(batch["lens"][c])
        st, best = co.viterbi8(m, batch["obs"][o:o + L])
        assert np.array_equal(sg[o:o + L], (st < 4).astype(np.uint8)), c
        assert sc[c] == best, (c, sc[c], best)
