"""Decode of every model the reference accepts (VERDICT r02 missing #5): Mahout's loop takes
log(0) = -inf without complaint (HmmAlgorithms.viterbiAlgorithm, called through
HmmEvaluator.decode at CpGIslandFinder.java:260), so models with zero transitions, emission rows
that are not deterministic and pi with zeros must decode exactly too.  They run through the
general-model path (k_vit_general.hip: Mahout's 8-state recurrence, chunks in parallel),
checked bitwise against the oracle's 8-state Viterbi (oracle/cpg_oracle.c orc_viterbi8) and
island scan (:262-339 over the states themselves).  Every call goes through the C-ABI."""
import numpy as np
import pytest

from oracle import coracle as co
from oracle import pyref as pr

pytestmark = pytest.mark.gpu


def _rand_model(rng, zero_frac=0.2, det_b=False):
    pi = rng.random(8) * (rng.random(8) > zero_frac)
    pi[rng.integers(0, 8)] += 0.1
    a = rng.random((8, 8)) * (rng.random((8, 8)) > zero_frac)
    a[np.arange(8), rng.integers(0, 8, 8)] += 0.05          # no all-zero row
    if det_b:
        b = np.zeros((8, 4))
        b[np.arange(8), np.arange(8) % 4] = 1.0
    else:
        b = rng.random((8, 4)) * (rng.random((8, 4)) > zero_frac)
        b[np.arange(8), np.arange(8) % 4] += 0.05
    return co.model_flat(pi / pi.sum(), a / a.sum(1, keepdims=True), b / b.sum(1, keepdims=True))


def _dev(packed, dev):
    from cpgisland_amd import device as D
    return D.to_device(np.concatenate([packed.astype(np.uint32), np.zeros(8, np.uint32)]), dev)


@pytest.fixture(scope="module")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.mark.parametrize("seed", range(6))
def test_decode_states_any_model(gpu_ctx, dev, seed):
    """HmmEvaluator.decode on models outside the exact scan's contract: zeros in pi / A,
    emission rows that are not deterministic — the states bitwise the oracle's."""
    from cpgisland_amd import HmmEvaluator, HmmModel
    rng = np.random.default_rng(seed)
    m = _rand_model(rng, det_b=(seed % 3 == 0))
    for T in (1, 2, 37, 5000):
        obs = rng.integers(0, 4, T).astype(np.int32)
        st = HmmEvaluator.decode(HmmModel.from_struct(m), obs, ctx=gpu_ctx)
        ref, _ = co.viterbi8(m, obs.astype(np.uint8))
        assert np.array_equal(st, ref), (seed, T)


def test_viterbi_states_multi_chunk_and_scores(gpu_ctx, dev):
    import torch
    from cpgisland_amd import HmmModel
    from cpgisland_amd import device as D
    rng = np.random.default_rng(11)
    m = _rand_model(rng)
    C, nch = 4096, 11                       # 11 chunks: one wave's 8 + a partial second wave
    n = nch * C + 777
    obs = rng.integers(0, 4, n).astype(np.uint8)
    st, sc = D.viterbi_states(gpu_ctx, HmmModel.from_struct(m), _dev(pr.pack(obs), dev), n, C)
    torch.cuda.synchronize()
    gpu_ctx.sync()
    st, sc = st.cpu().numpy(), sc.cpu().numpy()
    for c in range(nch):
        ref, best = co.viterbi8(m, obs[c * C:(c + 1) * C])
        assert np.array_equal(st[c * C:(c + 1) * C], ref), c
        assert sc[c] == best or (np.isnan(best) and np.isnan(sc[c])), c


def test_viterbi_d_zero_transitions(gpu_ctx, dev):
    """Deterministic emissions with zero transitions: cpg_viterbi_d's sign bits and scores
    equal the oracle's; a dead end (every candidate -inf after a C->G step) leaves the bases'
    states, which sign bits cannot carry: cpg_sync says CPG_E_UNSUPPORTED and
    cpg_viterbi_states_d gives the exact states."""
    import torch
    from cpgisland_amd import CpgError, HmmModel
    from cpgisland_amd import device as D
    rng = np.random.default_rng(3)
    pi, a, b = co.model_split(co.initial_model())
    a2 = a.copy()
    a2[0, 5] = 0.0                          # A+ -> C- impossible
    a2[7, 2] = 0.0                          # T- -> G+ impossible
    a2 /= a2.sum(1, keepdims=True)
    m = co.model_flat(pi, a2, b)
    C, nch = 4096, 3
    obs = rng.integers(0, 4, nch * C).astype(np.uint8)
    sg, sc = D.viterbi(gpu_ctx, HmmModel.from_struct(m), _dev(pr.pack(obs), dev), nch * C, C)
    torch.cuda.synchronize()
    gpu_ctx.sync()
    bits = D.sign_to_numpy(sg, nch * C)
    scs = sc.cpu().numpy()
    for c in range(nch):
        ref, best = co.viterbi8(m, obs[c * C:(c + 1) * C])
        assert np.array_equal(bits[c * C:(c + 1) * C], (ref < 4).astype(np.uint8)), c
        assert scs[c] == best
    # dead end: C+/C- -> G+/G- all impossible; a 'CG' in the chunk kills every candidate
    a3 = a.copy()
    a3[np.ix_([1, 5], [2, 6])] = 0.0
    a3 /= a3.sum(1, keepdims=True)
    m3 = co.model_flat(pi, a3, b)
    o3 = rng.integers(0, 4, C).astype(np.uint8)
    o3[100:102] = [1, 2]
    dp3 = _dev(pr.pack(o3), dev)
    D.viterbi(gpu_ctx, HmmModel.from_struct(m3), dp3, C, C)
    torch.cuda.synchronize()
    with pytest.raises(CpgError, match="UNSUPPORTED"):
        gpu_ctx.sync()
    st, _ = D.viterbi_states(gpu_ctx, HmmModel.from_struct(m3), dp3, C, C)
    torch.cuda.synchronize()
    gpu_ctx.sync()
    ref, best = co.viterbi8(m3, o3)
    assert best == -np.inf and np.array_equal(st.cpu().numpy(), ref)


def test_decode_d_non_deterministic_emissions(gpu_ctx, dev):
    """cpg_decode_d (Viterbi + islands in one call) with emission rows that are not
    deterministic: the island records are the :262-339 scan over the decoded STATES (the
    reference counts C+ / G+ states, not bases), equal to the oracle's testModel loop."""
    import torch
    from cpgisland_amd import HmmModel
    from cpgisland_amd import device as D
    rng = np.random.default_rng(21)
    pi, a, b = co.model_split(co.initial_model())
    b2 = 0.9 * b + 0.025                    # every symbol possible from every state
    m = co.model_flat(pi, a, b2 / b2.sum(1, keepdims=True))
    C = 65536
    n = 3 * C + 999
    packed, _ = D.synth_host(77, 0, n)
    obs = pr.unpack(packed, n)
    so, sc, out, cnt = D.decode(gpu_ctx, HmmModel.from_struct(m), _dev(packed, dev), n, C,
                                first_chunk=5)
    torch.cuda.synchronize()
    gpu_ctx.sync()
    isl = D.islands_to_numpy(out, cnt)
    states, ref_isl, ref_sc = co.decode_chunks(m, obs, C)
    assert np.array_equal(sc.cpu().numpy()[:3], ref_sc)
    assert np.array_equal(D.sign_to_numpy(so, n)[:3 * C], (states < 4).astype(np.uint8))
    assert not D.sign_to_numpy(so, n)[3 * C:].any()          # the undecoded tail reads '-'
    ref_isl = ref_isl.copy()
    ref_isl["chunk"] += 5
    ref_isl["beg1"] += 5 * C
    ref_isl["end1"] += 5 * C
    assert len(ref_isl) > 0 and np.array_equal(isl, ref_isl)


def test_reserved_general_path_does_not_allocate(dev):
    """ cpg_reserve_ex(CPG_RESERVE_GENERAL) sizes the general-model Viterbi's
    workspace: after it, decodes that take the general path (zero transitions, several chunk
    lengths, the whole input as one chunk) and the exact-scan path (a non-power-of-two chunk
    length) leave the context's workspace unchanged — no allocation, no device-wide sync, so
    the calls are safe to capture in a hipGraph.  Results still equal the oracle's."""
    import torch
    from cpgisland_amd import Context, HmmModel
    from cpgisland_amd import device as D
    rng = np.random.default_rng(5)
    pi, a, b = co.model_split(co.initial_model())
    a2 = a.copy()
    a2[0, 5] = 0.0
    a2 /= a2.sum(1, keepdims=True)
    mg = co.model_flat(pi, a2, b)
    n = 5 * 65536 + 333
    obs = rng.integers(0, 4, n).astype(np.uint8)
    dp = _dev(pr.pack(obs), dev)
    ctx = Context(0)
    try:
        ctx.reserve(n, general=True)
        before = ctx.workspace_bytes()
        for C in (4096, 65536, 12288, 768, 12544):   # (multiples of 256 too)
            D.viterbi(ctx, HmmModel.from_struct(mg), dp, n, C)
            D.viterbi(ctx, HmmModel.initial(), dp, n, C)
            D.decode(ctx, HmmModel.initial(), dp, n, C)
        st, sc = D.viterbi_states(ctx, HmmModel.from_struct(mg), dp, n, n)   # one chunk
        torch.cuda.synchronize()
        ctx.sync()
        assert ctx.workspace_bytes() == before
        ref, best = co.viterbi8(mg, obs)
        assert np.array_equal(st.cpu().numpy()[:n], ref) and sc.cpu().numpy()[0] == best
    finally:
        ctx.close()
