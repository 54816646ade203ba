"""GPU parity: libcpg's HIP path vs the CPU oracle on the same seeded inputs.

Bit-exact for everything integer/index (labelled counts, Viterbi paths, island records) and
for the Viterbi best score (the kernels reproduce the sequential fp64 recurrence exactly);
Baum-Welch expected counts within a stated relative tolerance (fp64, re-associated sums).
Every call goes through the C-ABI (libcpg.so).  PARITY UNPINNED (see oracle/cpg_oracle.h).
"""
import numpy as np
import pytest

from oracle import coracle as co
from oracle import pyref as pr

pytestmark = pytest.mark.gpu

ESTEP_RTOL = 1e-9        # north_star: fp64 within 1e-9 relative
TRAIN = 65536
DECODE = 1 << 20


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def golden():
    import os
    return np.load(os.path.join(os.path.dirname(__file__), "golden", "golden.npz"))


def _model(m):
    from cpgisland_amd import HmmModel
    return HmmModel.from_struct(m)


def _dev_genome(packed, sign, dev):
    from cpgisland_amd import device as D
    pad = np.zeros(8, np.uint32)
    dp = D.to_device(np.concatenate([packed.astype(np.uint32), pad]), dev)
    ds = D.to_device(np.concatenate([sign.astype(np.uint32), pad]), dev)
    return dp, ds


def _viterbi(ctx, m, dp, n, C):
    import torch
    from cpgisland_amd import device as D
    so, sc = D.viterbi(ctx, _model(m), dp, n, C)
    torch.cuda.synchronize()
    ctx.sync()
    return D.sign_to_numpy(so, n), sc.cpu().numpy()[: n // C]


def _trained_model(m0, obs):
    return co.normalize(co.estep(m0, obs, TRAIN))


# ---------------------------------------------------------------- golden vectors
def test_golden_viterbi_islands_counts(gpu_ctx, torch_dev, golden):
    import torch
    from cpgisland_amd import device as D
    N = DECODE
    dp, ds = _dev_genome(golden["synth_packed"], golden["synth_truth"], torch_dev)
    m = golden["model_initial"]
    sg, sc = _viterbi(gpu_ctx, m, dp, N, N)
    assert np.array_equal(pr.pack_bits(sg), golden["viterbi_sign"])
    assert np.array_equal(sc, golden["viterbi_score"])          # exact, not 1e-9
    so = D.to_device(pr.pack_bits(sg), torch_dev)
    out, cnt = D.islands(gpu_ctx, dp, so, N, N)
    isl = D.islands_to_numpy(out, cnt)
    assert np.array_equal(isl, golden["islands"])
    assert "".join(co.format_island(r) for r in isl) == str(golden["islands_txt"])
    c = D.count_labelled(gpu_ctx, dp, ds, N, TRAIN)
    assert np.array_equal(c.cpu().numpy(), golden["counts_labelled"])
    e = D.bw_estep(gpu_ctx, _model(m), dp, N, TRAIN)
    torch.cuda.synchronize()
    ref = golden["estep_counts"]
    got = e.cpu().numpy()
    nz = ref != 0
    assert np.all(got[~nz] == 0)
    assert np.max(np.abs(got[nz] - ref[nz]) / np.abs(ref[nz])) < ESTEP_RTOL
    sg1, sc1 = _viterbi(gpu_ctx, golden["model_trained1"], dp, N, N)
    assert np.array_equal(pr.pack_bits(sg1), golden["viterbi_sign_trained1"])
    assert np.array_equal(sc1, golden["viterbi_score_trained1"])


# ---------------------------------------------------------------- Viterbi
@pytest.mark.parametrize("T", [1, 2, 3, 16, 17, 255, 256, 257, 511, 512, 513, 1000, 4097,
                               65536, 100003])
def test_decode_states_vs_mahout_order(gpu_ctx, T):
    from cpgisland_amd import HmmEvaluator, HmmModel
    rng = np.random.default_rng(T)
    obs = rng.integers(0, 4, T).astype(np.int32)
    m = co.initial_model()
    st = HmmEvaluator.decode(HmmModel.from_struct(m), obs, True, ctx=gpu_ctx)
    ref, _ = co.viterbi8(m, obs.astype(np.uint8))
    assert np.array_equal(st, ref)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_viterbi_multichunk_synthetic(gpu_ctx, torch_dev, seed):
    from cpgisland_amd import device as D
    N = 6 * DECODE + 4321
    packed, sign = D.synth_host(1000 + seed, 0, N)
    obs = pr.unpack(packed, N)
    m = co.initial_model() if seed != 3 else _trained_model(co.initial_model(), obs[:16 * TRAIN])
    dp, _ = _dev_genome(packed, sign, torch_dev)
    sg, sc = _viterbi(gpu_ctx, m, dp, N, DECODE)
    states, _, score = co.decode_chunks(m, obs, DECODE)
    nd = len(states)
    assert np.array_equal(sg[:nd], (states < 4).astype(np.uint8))
    assert not sg[nd:].any()                                     # tail never decoded
    assert np.array_equal(sc, score)


@pytest.mark.parametrize("C", [256, 4096, 65536])
def test_viterbi_small_chunks(gpu_ctx, torch_dev, C):
    rng = np.random.default_rng(C)
    N = 40 * C + 100
    obs = rng.integers(0, 4, N).astype(np.uint8)
    m = co.initial_model()
    dp, _ = _dev_genome(pr.pack(obs), np.zeros(N // 32 + 1, np.uint32), torch_dev)
    sg, sc = _viterbi(gpu_ctx, m, dp, N, C)
    for c in range(N // C):
        s2, best = co.viterbi2(m, obs[c * C:(c + 1) * C])
        assert np.array_equal(sg[c * C:(c + 1) * C], s2), c
        assert sc[c] == best


@pytest.mark.parametrize("nsb,trim", [(3856, 0), (3856, 100), (3968, 0)])
def test_viterbi_partly_filled_tscan_lanes(gpu_ctx, torch_dev, nsb, trim):
    """Chunk lengths whose 256-position block count nsb is in (3840, 4096] and a multiple of
    16 take K6's 16-B path with some lanes owning no block (nsb = 3856: lanes 241-255);
    trim > 0: one chunk with a partly filled last block."""
    from cpgisland_amd import device as D
    C = nsb * 256 - trim
    nch = 1 if trim else 2
    N = nch * C + 777
    packed, sign = D.synth_host(4000 + nsb + trim, 0, N)
    obs = pr.unpack(packed, N)
    m = co.initial_model()
    dp, _ = _dev_genome(packed, sign, torch_dev)
    sg, sc = _viterbi(gpu_ctx, m, dp, N, C)
    states, _, score = co.decode_chunks(m, obs, C)
    assert len(states) == nch * C
    assert np.array_equal(sg[:nch * C], (states < 4).astype(np.uint8))
    assert not sg[nch * C:].any()
    assert np.array_equal(sc, score)


def test_viterbi_adversarial_inputs(gpu_ctx, torch_dev):
    m = co.initial_model()
    n = DECODE
    cases = {
        "cg": np.tile(np.array([1, 2], np.uint8), n // 2),
        "at": np.tile(np.array([0, 3], np.uint8), n // 2),
        "allA": np.zeros(n, np.uint8),
        "allC": np.ones(n, np.uint8),
        "blocks": np.repeat(np.random.default_rng(0).integers(0, 4, n // 4096), 4096)
                  .astype(np.uint8),
    }
    for name, obs in cases.items():
        dp, _ = _dev_genome(pr.pack(obs), np.zeros(n // 32, np.uint32), torch_dev)
        sg, sc = _viterbi(gpu_ctx, m, dp, n, n)
        s2, best = co.viterbi2(m, obs)
        assert np.array_equal(sg, s2), name
        assert sc[0] == best, name


def test_viterbi_extreme_models(gpu_ctx, torch_dev):
    """Tiny transition probabilities (large |log a|: other fixed-point scale and binade
    range), pi with zeros, and the degenerate pi = 0 for both live states."""
    from cpgisland_amd import HmmEvaluator, HmmModel
    rng = np.random.default_rng(4)
    n = 3 * 4096
    obs = rng.integers(0, 4, n).astype(np.uint8)
    pi, a, b = co.model_split(co.initial_model())
    a2 = a.copy()
    a2[:4, 4:] = 1e-12
    a2[4:, :4] = 1e-9
    a2 /= a2.sum(axis=1, keepdims=True)
    for m in (co.model_flat(pi, a2, b),
              co.model_flat(np.array([0, .25, .25, .25, 0, .1, .1, .05]), a, b)):
        dp, _ = _dev_genome(pr.pack(obs), np.zeros(n // 32 + 1, np.uint32), torch_dev)
        sg, sc = _viterbi(gpu_ctx, m, dp, n, 4096)
        for c in range(3):
            st, best = co.viterbi8(m, obs[c * 4096:(c + 1) * 4096])
            assert np.array_equal(sg[c * 4096:(c + 1) * 4096], (st < 4).astype(np.uint8))
            assert sc[c] == best
    # degenerate: pi[o0+] = pi[o0-] = 0
    mdeg = co.model_flat(np.array([0, .25, .25, .25, 0, .1, .1, .05]), a, b)
    o = obs[:5000].astype(np.int32)
    o[0] = 0
    st = HmmEvaluator.decode(HmmModel.from_struct(mdeg), o, ctx=gpu_ctx)
    ref, _ = co.viterbi8(mdeg, o.astype(np.uint8))
    assert np.array_equal(st, ref)
    st1 = HmmEvaluator.decode(HmmModel.from_struct(mdeg), o[:1], ctx=gpu_ctx)
    ref1, _ = co.viterbi8(mdeg, o[:1].astype(np.uint8))
    assert np.array_equal(st1, ref1)


def test_viterbi_score_is_path_score_full_size(gpu_ctx, torch_dev):
    """Size-independent property at the C2 size (46 Mbp, 43 chunks): the reported best
    score equals the log-probability of the decoded path (within 1e-9 relative), and every
    chunk's kernel self-check (block exit == next block entry, bitwise) passed."""
    from cpgisland_amd import device as D
    N = 46_000_000
    packed, sign = D.synth_host(20251016, 0, N)
    m = co.initial_model()
    dp, _ = _dev_genome(packed, sign, torch_dev)
    sg, sc = _viterbi(gpu_ctx, m, dp, N, DECODE)
    obs = pr.unpack(packed, N)
    L = np.log(m[8:72].reshape(8, 8))
    for c in range(0, N // DECODE, 7):
        o = obs[c * DECODE:(c + 1) * DECODE].astype(np.int64)
        s = o + np.where(sg[c * DECODE:(c + 1) * DECODE] != 0, 0, 4)
        v = np.log(m[s[0]]) + L[s[:-1], s[1:]].sum()
        assert abs(v - sc[c]) <= 1e-9 * abs(sc[c])
    # one full chunk bitwise against the oracle
    c = 21
    s2, best = co.viterbi2(m, obs[c * DECODE:(c + 1) * DECODE])
    assert np.array_equal(sg[c * DECODE:(c + 1) * DECODE], s2) and sc[c] == best


def test_decode_errors(gpu_ctx):
    from cpgisland_amd import CpgError, CpgInvalid, HmmEvaluator, HmmModel
    from cpgisland_amd import _lib
    m = HmmModel.initial()
    with pytest.raises(CpgInvalid):
        HmmEvaluator.decode(m, np.array([0, 1, 4], np.int32), ctx=gpu_ctx)
    with pytest.raises(CpgInvalid):
        HmmEvaluator.decode(m, np.array([], np.int32), ctx=gpu_ctx)
    # a non-deterministic emission row: HmmEvaluator.decode takes it (the general-model path,
    # tests/test_gpu_general.py) and matches the oracle; sign bits cannot carry such a path,
    # so cpg_viterbi_d refuses it
    nd = HmmModel.initial()
    nd.b[0] = [0.9, 0.1, 0, 0]
    obs = np.array([0, 1, 2], np.int32)
    ref, _ = co.viterbi8(nd.to_struct(), obs.astype(np.uint8))
    assert np.array_equal(HmmEvaluator.decode(nd, obs, ctx=gpu_ctx), ref)
    import torch
    from cpgisland_amd import device as D
    dp = D.to_device(np.zeros(4096 // 16 + 8, np.uint32), torch.device("cuda:0"))
    with pytest.raises(CpgError) as e:
        D.viterbi(gpu_ctx, nd, dp, 4096, 4096)
    assert e.value.code == _lib.CPG_E_UNSUPPORTED


# ---------------------------------------------------------------- labelled counts
def _labelled(kind, N, seed):
    """(bases, signs) of a labelled-count case; "alternating" and "runs" put a sign change
    at every / many positions (the counters' one-by-one border path, count_dev.h)."""
    from cpgisland_amd import device as D
    rng = np.random.default_rng(seed)
    if kind == "synth":
        packed, sign = D.synth_host(77 + seed, 0, N)
        return pr.unpack(packed, N), pr.unpack_bits(sign, N)
    obs = rng.integers(0, 4, N).astype(np.uint8)
    if kind == "runs":
        sg = np.repeat(np.arange(N) % 2, rng.integers(1, 9, N))[:N]
    else:
        sg = {"random": (rng.random(N) < 0.5), "plus": np.ones(N), "minus": np.zeros(N),
              "alternating": np.arange(N) % 2}[kind]
    return obs, sg.astype(np.uint8)


@pytest.mark.parametrize("C", [256, 768, 4096, 12288, 65536])   # 768 / 12288: k_count_main<false>
@pytest.mark.parametrize("kind", ["random", "synth", "plus", "minus", "alternating", "runs"])
def test_counts_bit_exact(gpu_ctx, torch_dev, C, kind):
    from cpgisland_amd import device as D
    N = 37 * C + 123
    obs, sg = _labelled(kind, N, C)
    dp, ds = _dev_genome(pr.pack(obs), pr.pack_bits(sg), torch_dev)
    got = D.count_labelled(gpu_ctx, dp, ds, N, C).cpu().numpy()
    assert np.array_equal(got, co.count_labelled(obs, sg, C))


@pytest.mark.parametrize("kind", ["synth", "plus"])
def test_counts_many_batches_vs_oracle(gpu_ctx, torch_dev, kind):
    """160 Mbp: ~19 blocks per lane of the count grid, several batches per lane; all-A /
    all-'+' puts 63 transitions of one class in every block, so every lane's 32-bit moment
    registers and the island moments' LDS replicas take their largest per-block increments."""
    from cpgisland_amd import device as D
    N = 160_000_000 + 4321
    if kind == "synth":
        packed, sign = D.synth_host(8, 0, N)
        obs, sg = pr.unpack(packed, N), pr.unpack_bits(sign, N)
    else:
        obs, sg = np.zeros(N, np.uint8), np.ones(N, np.uint8)
        packed, sign = pr.pack(obs), pr.pack_bits(sg)
    dp, ds = _dev_genome(packed, sign, torch_dev)
    got = D.count_labelled(gpu_ctx, dp, ds, N, TRAIN).cpu().numpy()
    assert np.array_equal(got, co.count_labelled(obs, sg, TRAIN))


@pytest.mark.parametrize("C", [4096, 16384, 65536])
@pytest.mark.parametrize("kind", ["synth", "random", "alternating"])
def test_train_pass_equals_separate_calls(gpu_ctx, torch_dev, C, kind):
    """cpg_train_pass_d (one launch for C >= 16 Ki: each E-step lane also counts its 64
    bases) == cpg_bw_estep_d + cpg_count_labelled_d: E-step bitwise, counts bit-exact vs
    the oracle."""
    from cpgisland_amd import device as D
    N = 11 * C + 321
    obs, sg = _labelled(kind, N, C + 1)
    dp, ds = _dev_genome(pr.pack(obs), pr.pack_bits(sg), torch_dev)
    m = co.initial_model()
    e, c = D.train_pass(gpu_ctx, _model(m), dp, ds, N, C)
    e, c = e.cpu().numpy(), c.cpu().numpy()
    assert np.array_equal(c, co.count_labelled(obs, sg, C))
    assert np.array_equal(e, D.bw_estep(gpu_ctx, _model(m), dp, N, C).cpu().numpy())
    ref = co.estep(m, obs, C)
    nz = ref != 0
    assert np.max(np.abs(e[nz] - ref[nz]) / np.abs(ref[nz])) < ESTEP_RTOL


def test_train_pass_interleaved_with_single_calls(gpu_ctx, torch_dev):
    """The fused pass shares the count / E-step accumulators and the E-step's done counters
    with the single calls: any interleaving and grid size leaves them re-zeroed."""
    from cpgisland_amd import device as D
    m = co.initial_model()
    packed, sign = D.synth_host(321, 0, 41 * TRAIN)
    obs, truth = pr.unpack(packed, 41 * TRAIN), pr.unpack_bits(sign, 41 * TRAIN)
    dp, ds = _dev_genome(packed, sign, torch_dev)
    for i, nch in enumerate([2, 41, 1, 17, 41, 3]):
        n = nch * TRAIN + 50
        cref = co.count_labelled(obs[:n], truth[:n], TRAIN)
        eref = co.estep(m, obs[:n], TRAIN)
        nz = eref != 0
        e, c = D.train_pass(gpu_ctx, _model(m), dp, ds, n, TRAIN)
        assert np.array_equal(c.cpu().numpy(), cref), nch
        e = e.cpu().numpy()
        assert np.max(np.abs(e[nz] - eref[nz]) / np.abs(eref[nz])) < ESTEP_RTOL, nch
        if i % 2:
            assert np.array_equal(D.count_labelled(gpu_ctx, dp, ds, n, TRAIN).cpu().numpy(), cref)
        else:
            assert np.array_equal(D.bw_estep(gpu_ctx, _model(m), dp, n, TRAIN).cpu().numpy(), e)


def test_counts_full_size_properties(gpu_ctx, torch_dev):
    """C2 size: totals are exact identities of the chunk geometry; invariant under sharding."""
    from cpgisland_amd import device as D
    N = 46_000_000
    packed, sign = D.synth_host(5, 0, N)
    dp, ds = _dev_genome(packed, sign, torch_dev)
    full = D.count_labelled(gpu_ctx, dp, ds, N, TRAIN).cpu().numpy()
    nch = N // TRAIN
    assert full[:8].sum() == nch and full[8:72].sum() == nch * (TRAIN - 1)
    assert full[120:124].sum() == nch * TRAIN and full[104:120].sum() == nch * (TRAIN - 1)
    # sharded in 4 contiguous pieces of whole chunks: the sum is identical
    per = (nch // 4) * TRAIN
    acc = np.zeros(124, np.int64)
    for r in range(4):
        n_r = per if r < 3 else (nch - 3 * nch // 4) * TRAIN
        acc += D.count_labelled(gpu_ctx, dp[r * per // 16:], ds[r * per // 32:], n_r,
                                TRAIN).cpu().numpy()
    assert np.array_equal(acc, full)


# ---------------------------------------------------------------- islands
def test_islands_random_states_vs_oracle(gpu_ctx, torch_dev):
    from cpgisland_amd import device as D
    rng = np.random.default_rng(12)
    C = 4096
    nch = 64
    N = nch * C
    states = np.concatenate([np.resize(_rand_states(rng), C) for _ in range(nch)])
    obs = (states % 4).astype(np.uint8)
    sg = (states < 4).astype(np.uint8)
    dp, ds = _dev_genome(pr.pack(obs), pr.pack_bits(sg), torch_dev)
    for first in (0, 2048 * 256 - 3):      # the second crosses chunk*C = 2^31 (int wrap)
        out, cnt = D.islands(gpu_ctx, dp, ds, N, C, first_chunk=first)
        got = D.islands_to_numpy(out, cnt)
        exp = np.concatenate([co.islands(states[c * C:(c + 1) * C], first + c)
                              for c in range(nch)])
        assert len(exp) > 100
        assert np.array_equal(got, exp)


@pytest.mark.parametrize("C", [1 << 17, 1 << 20])
def test_islands_multi_tile_vs_oracle(gpu_ctx, torch_dev, C):
    """Chunks of several 131,072-position tiles with runs across tile borders: 2^17 has
    ~4k runs per chunk (several per lane, register-cached), 2^20 ~35k (re-read path)."""
    from cpgisland_amd import device as D
    rng = np.random.default_rng(C)
    nch = 3
    states = np.resize(_rand_states(rng, nch * C), nch * C)
    obs = (states % 4).astype(np.uint8)
    sg = (states < 4).astype(np.uint8)
    dp, ds = _dev_genome(pr.pack(obs), pr.pack_bits(sg), torch_dev)
    out, cnt = D.islands(gpu_ctx, dp, ds, nch * C, C, cap=1 << 16)
    got = D.islands_to_numpy(out, cnt)
    exp = np.concatenate([co.islands(states[c * C:(c + 1) * C], c) for c in range(nch)])
    assert len(exp) > 1000
    assert np.array_equal(got, exp)


def test_islands_huge_chunk_vs_oracle(gpu_ctx, torch_dev):
    """One chunk of 1,025 tiles: the tile offsets live in global memory, not LDS."""
    from cpgisland_amd import device as D
    C = (1 << 27) + (1 << 17)
    st = np.full(C, 6, np.int32)
    rng = np.random.default_rng(5)
    for b in np.sort(rng.choice(C - 4000, 300, replace=False)):
        L = int(rng.integers(2, 3000))
        st[b:b + L] = np.resize(np.array([1, 2, 1, 2, 0, 3], np.int32), L)
    st[(1 << 27) - 50:(1 << 27) + 50] = np.resize(np.array([1, 2], np.int32), 100)   # across
    st[C - 200:C - 100] = 1                          # the last tile border; no G: dropped
    dp, ds = _dev_genome(pr.pack((st % 4).astype(np.uint8)),
                         pr.pack_bits((st < 4).astype(np.uint8)), torch_dev)
    out, cnt = D.islands(gpu_ctx, dp, ds, C, C)
    exp = co.islands(st, 0)
    assert len(exp) > 100
    assert np.array_equal(D.islands_to_numpy(out, cnt), exp)


def _rand_states(rng, n=4096):
    out = []
    while len(out) < n:
        plus = rng.random() < 0.4
        L = int(rng.integers(1, 60))
        b = rng.choice(4, L, p=[0.15, 0.35, 0.35, 0.15] if plus else [0.3, 0.2, 0.2, 0.3])
        out += [int(x) + (0 if plus else 4) for x in b]
    return np.array(out, np.int32)


def test_islands_long_overflow_island(gpu_ctx, torch_dev):
    from cpgisland_amd import device as D
    C = 1 << 17
    st = np.full(C, 6, np.int32)
    st[10:10 + 70000] = np.resize(np.array([1, 2], np.int32), 70000)   # cg*len overflows
    st[80000:81000] = np.resize(np.array([1, 2, 0], np.int32), 1000)
    st[90000:90010] = [3, 3, 3, 1, 4, 2, 2, 1, 2, 2]                     # stale atC
    st[90010:90020] = [4, 4, 4, 0, 2, 4, 4, 4, 4, 4]
    dp, ds = _dev_genome(pr.pack((st % 4).astype(np.uint8)),
                         pr.pack_bits((st < 4).astype(np.uint8)), torch_dev)
    out, cnt = D.islands(gpu_ctx, dp, ds, C, C)
    assert np.array_equal(D.islands_to_numpy(out, cnt), co.islands(st, 0))


def test_decode_on_two_cus_equals_full_gpu(gpu_ctx):
    """No kernel of cpg_decode_d waits for another workgroup: K1 stores its segments' products
    and the next launch (k_vit_segplan) reads the chunk's earlier ones; a fused decode's chunk
    resolve (its last traceback workgroup, a done counter) writes per-chunk counts and the
    write pass places the records.  So the decode on a stream of TWO compute units — where a
    workgroup spinning on another could hold the units that one needs — completes, and equals
    the whole GPU's decode and the two single calls bitwise (8 chunks of 1 Mi: the segment
    path, 16 segments per chunk, and the fused island resolve)."""
    import torch
    from cpgisland_amd import HmmModel
    from cpgisland_amd import device as D
    dev = torch.device("cuda:0")
    n, cl = 8 << 20, 1 << 20
    p, _ = D.synth_host(11, 0, n)
    dp = D.to_device(np.concatenate([p, np.zeros(8, np.uint32)]), dev)
    m = HmmModel.initial()
    so, sc, io, ic = D.decode(gpu_ctx, m, dp, n, cl)
    s2 = D.cu_stream(0, [0, 1])
    try:
        with torch.cuda.stream(s2):
            so2, sc2, io2, ic2 = D.decode(gpu_ctx, m, dp, n, cl)
        s2.synchronize()
    finally:
        D.cu_stream_destroy(s2)
    so3, sc3 = D.viterbi(gpu_ctx, m, dp, n, cl)
    o3, c3 = D.islands(gpu_ctx, dp, so3, n, cl)
    torch.cuda.synchronize()
    gpu_ctx.sync()
    w = D.words32(n)
    for a_, b_ in ((so2, so), (so3, so)):
        assert np.array_equal(a_.cpu().numpy()[:w], b_.cpu().numpy()[:w])
    assert np.array_equal(sc2.cpu().numpy(), sc.cpu().numpy())
    assert np.array_equal(sc3.cpu().numpy(), sc.cpu().numpy())
    isl = D.islands_to_numpy(io, ic)
    assert len(isl) > 0
    assert np.array_equal(D.islands_to_numpy(io2, ic2), isl)
    assert np.array_equal(D.islands_to_numpy(o3, c3), isl)
    st, best = co.viterbi8(m.to_struct(), pr.unpack(p[: cl // 16], cl))
    assert np.array_equal(D.sign_to_numpy(so, cl), (st < 4).astype(np.uint8))
    assert sc.cpu().numpy()[0] == best
    assert np.array_equal(isl[isl["chunk"] == 0], co.islands(st, 0))


def test_islands_capacity(gpu_ctx, torch_dev, golden):
    from cpgisland_amd import device as D
    N = DECODE
    dp, _ = _dev_genome(golden["synth_packed"], golden["synth_truth"], torch_dev)
    so = D.to_device(golden["viterbi_sign"], torch_dev)
    out, cnt = D.islands(gpu_ctx, dp, so, N, N, cap=3)
    assert int(cnt.item()) == len(golden["islands"])
    assert np.array_equal(out[:3].cpu().numpy().reshape(-1).view(co.ISLAND_DTYPE),
                          golden["islands"][:3])


# ---------------------------------------------------------------- E-step
@pytest.mark.parametrize("C", [4096, 16384, 65536])
def test_estep_tolerance_and_determinism(gpu_ctx, torch_dev, C):
    import torch
    from cpgisland_amd import device as D
    N = 9 * C + 77
    packed, sign = D.synth_host(31 + C, 0, N)
    obs = pr.unpack(packed, N)
    m = co.initial_model()
    dp, _ = _dev_genome(packed, sign, torch_dev)
    e1 = D.bw_estep(gpu_ctx, _model(m), dp, N, C).cpu().numpy()
    e2 = D.bw_estep(gpu_ctx, _model(m), dp, N, C).cpu().numpy()
    torch.cuda.synchronize()
    assert np.array_equal(e1, e2)                                 # deterministic
    ref = co.estep(m, obs, C)
    nz = ref != 0
    assert np.all(e1[~nz] == 0)
    assert np.max(np.abs(e1[nz] - ref[nz]) / np.abs(ref[nz])) < ESTEP_RTOL
    # the M-step of the GPU counts is the oracle's model to the same tolerance
    assert np.allclose(co.normalize(e1), co.normalize(ref), rtol=ESTEP_RTOL, atol=0)


def test_estep_trained_model_iteration(gpu_ctx, torch_dev):
    """Two Baum-Welch iterations on the GPU track the oracle's (model after iteration 2)."""
    from cpgisland_amd import device as D
    N = 24 * TRAIN
    packed, sign = D.synth_host(99, 0, N)
    obs = pr.unpack(packed, N)
    dp, _ = _dev_genome(packed, sign, torch_dev)
    mg = mo = co.initial_model()
    for _ in range(2):
        mg = co.normalize(D.bw_estep(gpu_ctx, _model(mg), dp, N, TRAIN).cpu().numpy())
        mo = co.normalize(co.estep(mo, obs, TRAIN))
    assert np.allclose(mg, mo, rtol=1e-8, atol=0)


def estep_grid_bound(obs, chunk_len):
    """Absolute error bound, per cpg_counts_f64 entry, of the E-step kernel's fixed-point sums
    (k_estep.hip): positions go in two-position blocks whose 4 joint posteriors Zeta(a,c) are
    each rounded to the nearest multiple of 2^-47 (error <= 2^-48) before they are summed
    exactly; each position's pair posterior xi is a convex-weighted sum of two of them
    (xi_{2j}(a,b) = sum_c f(a,b,c) Zeta(a,c), f <= 1), so a transition bin of class d (previous
    base | current base << 2) is off by at most n_d * 2^-47, n_d = the positions of class d
    over the whole chunks; an
    emission entry (init + a column of transition bins) by the sum of its terms' bounds; the
    init posteriors (2^-62 grid) by 2^-63 per chunk; the log-likelihood (2^-24 per chunk) by
    2^-25 per chunk.  The fp64 arithmetic itself (a different association than the oracle's)
    stays within ESTEP_RTOL relative: |gpu - oracle| <= bound + ESTEP_RTOL * |oracle|."""
    obs = np.asarray(obs)
    nch = len(obs) // chunk_len
    o = obs[: nch * chunk_len].reshape(nch, chunk_len).astype(np.int64)
    d = (o[:, :-1] | (o[:, 1:] << 2)).ravel()
    nd = np.bincount(d, minlength=16).astype(np.float64)
    b = np.zeros(105)
    b[:8] = nch * 2.0 ** -63
    for i in range(8):
        for j in range(8):
            b[8 + 8 * i + j] = nd[(i & 3) | ((j & 3) << 2)] * 2.0 ** -47
    for j in range(8):
        b[72 + 4 * j + (j & 3)] = b[j] + sum(b[8 + 8 * i + j] for i in range(8))
    b[104] = nch * 2.0 ** -25
    return b


def assert_estep_close(got, ref, obs, chunk_len, what=""):
    """ESTEP_RTOL relative plus the fixed-point grid's derived bound (estep_grid_bound)."""
    bound = estep_grid_bound(obs, chunk_len)
    assert np.array_equal(got == 0, ref == 0), what
    err = np.abs(got - ref)
    ok = err <= bound + ESTEP_RTOL * np.abs(ref)
    assert ok.all(), (what, np.flatnonzero(~ok), err[~ok], bound[~ok], ref[~ok])


def test_estep_single_class_chunks(gpu_ctx, torch_dev):
    """Chunks whose positions are (nearly) all one dinucleotide class: the per-chunk class
    count the kernel recovers from its raw fixed-point bin sums (k_estep.hip class_count)
    is then at its largest (65,535 for all-A) — parity with the oracle holds as elsewhere."""
    from cpgisland_amd import device as D
    n = 4 * TRAIN
    cases = {
        "allA": np.zeros(n, np.uint8),
        "cg": np.tile(np.array([1, 2], np.uint8), n // 2),
        "allT_then_random": np.concatenate(
            [np.full(2 * TRAIN, 3, np.uint8),
             np.random.default_rng(5).integers(0, 4, 2 * TRAIN).astype(np.uint8)]),
    }
    m = co.initial_model()
    for name, obs in cases.items():
        dp, _ = _dev_genome(pr.pack(obs), np.zeros(n // 32, np.uint32), torch_dev)
        got = D.bw_estep(gpu_ctx, _model(m), dp, n, TRAIN).cpu().numpy()
        ref = co.estep(m, obs, TRAIN)
        # the '+' posteriors of these chunks are far below the 2^-47 grid: their bins are
        # within the grid's derived bound (n_d * 2^-47), every other entry within 1e-9
        # relative; the init posteriors (2^-62 grid) within 1e-9 relative everywhere
        assert_estep_close(got, ref, obs, TRAIN, name)
        nz = ref[:8] != 0
        assert np.all(np.abs(got[:8][nz] - ref[:8][nz]) <= ESTEP_RTOL * np.abs(ref[:8][nz])), name


def test_fused_finalize_across_grid_sizes(gpu_ctx, torch_dev):
    """The count and E-step launches finalize in their last workgroup (two-level done
    counters, re-zeroed by the finalizer): calls of every grid size — fewer workgroups than
    counter groups, more, uneven groups — in any order each return their own sums."""
    from cpgisland_amd import device as D
    m = co.initial_model()
    packed, sign = D.synth_host(123, 0, 41 * TRAIN)
    obs, truth = pr.unpack(packed, 41 * TRAIN), pr.unpack_bits(sign, 41 * TRAIN)
    dp, ds = _dev_genome(packed, sign, torch_dev)
    for nch in [2, 17, 41, 9, 1, 41, 2, 33]:
        n = nch * TRAIN + (nch % 3) * 100
        e = D.bw_estep(gpu_ctx, _model(m), dp, n, TRAIN).cpu().numpy()
        ref = co.estep(m, obs[:n], TRAIN)
        nz = ref != 0
        assert np.max(np.abs(e[nz] - ref[nz]) / np.abs(ref[nz])) < ESTEP_RTOL, nch
        c = D.count_labelled(gpu_ctx, dp, ds, n, TRAIN).cpu().numpy()
        assert np.array_equal(c, co.count_labelled(obs[:n], truth[:n], TRAIN)), nch


def test_viterbi_islands_calls_of_changing_size(gpu_ctx, torch_dev):
    """Calls of different chunk counts back to back: the workspace layout changes between
    them, and the look-back words (Viterbi segment products, island counts) live in slots of
    their own, so no stale word of another array can pass for this call's tag.  Every chunk
    decodes as in one call over all chunks (chunks are independent)."""
    import torch
    from cpgisland_amd import device as D
    D1 = 1 << 20
    nmax = 64
    packed, _ = D.synth_host(4242, 0, nmax * D1)
    dp, _ = _dev_genome(packed, np.zeros(nmax * D1 // 32, np.uint32), torch_dev)
    m = _model(co.initial_model())
    so_all, sc_all = D.viterbi(gpu_ctx, m, dp, nmax * D1, D1)
    out_all, c_all = D.islands(gpu_ctx, dp, so_all, nmax * D1, D1)
    torch.cuda.synchronize()
    gpu_ctx.sync()
    ref = so_all.cpu().numpy().view(np.uint32)
    isl_all = D.islands_to_numpy(out_all, c_all)
    for nch in [49, 64, 17, 3, 64, 49, 1, 33]:
        so, sc = D.viterbi(gpu_ctx, m, dp, nch * D1, D1)
        out, c = D.islands(gpu_ctx, dp, so, nch * D1, D1)
        torch.cuda.synchronize()
        gpu_ctx.sync()
        w = nch * D1 // 32
        assert np.array_equal(so.cpu().numpy().view(np.uint32)[:w], ref[:w]), nch
        assert np.array_equal(sc.cpu().numpy()[:nch], sc_all.cpu().numpy()[:nch]), nch
        isl = D.islands_to_numpy(out, c)
        assert np.array_equal(isl, isl_all[isl_all["chunk"] < nch]), nch
        # the fused decode (per-chunk done counters reused across calls of other sizes)
        so2, sc2, out2, c2 = D.decode(gpu_ctx, m, dp, nch * D1, D1)
        torch.cuda.synchronize()
        gpu_ctx.sync()
        assert np.array_equal(so2.cpu().numpy().view(np.uint32)[:w], ref[:w]), nch
        assert np.array_equal(sc2.cpu().numpy()[:nch], sc_all.cpu().numpy()[:nch]), nch
        assert np.array_equal(D.islands_to_numpy(out2, c2), isl), nch


def _switchy_model(scale):
    """The reference's initial model with the +/- switches made `scale` times likelier:
    Viterbi paths of many short runs (island records across every tile border)."""
    pi, a, b = co.model_split(co.initial_model())
    a2 = a.copy()
    a2[:4, 4:] *= scale
    a2[4:, :4] *= scale
    a2 /= a2.sum(axis=1, keepdims=True)
    return co.model_flat(pi, a2, b)


@pytest.mark.parametrize("C,nch", [(1 << 16, 5), (1 << 20, 3), (1 << 17, 2), (1 << 21, 2),
                                   (1 << 15, 4), (4096, 9)])
@pytest.mark.parametrize("model", ["initial", "switchy"])
def test_decode_fused_vs_oracle_and_separate_calls(gpu_ctx, torch_dev, C, nch, model):
    """cpg_decode_d (Viterbi + islands in one call; for chunk lengths that are multiples of
    65,536 the traceback writes the island run records itself) against the oracle's decode
    loop (:256-340: states, best scores, island records) and bitwise against the two single
    calls, with a chunk offset (first_chunk) and a tail past the last whole chunk."""
    import torch
    from cpgisland_amd import device as D
    N = nch * C + 777
    packed, _ = D.synth_host(900 + C % 97, 0, N)
    obs = pr.unpack(packed, N)
    m = co.initial_model() if model == "initial" else _switchy_model(40.0)
    dp, _ = _dev_genome(packed, np.zeros(N // 32 + 1, np.uint32), torch_dev)
    hm = _model(m)
    so, sc, out, cnt = D.decode(gpu_ctx, hm, dp, N, C, cap=1 << 18)
    torch.cuda.synchronize()
    gpu_ctx.sync()
    states, isl_ref, score = co.decode_chunks(m, obs, C)
    nd = len(states)
    sg = D.sign_to_numpy(so, N)
    assert np.array_equal(sg[:nd], (states < 4).astype(np.uint8))
    assert not sg[nd:].any()
    assert np.array_equal(sc.cpu().numpy()[:nch], score)
    got = D.islands_to_numpy(out, cnt)
    assert np.array_equal(got, isl_ref)
    if model == "switchy":
        assert len(isl_ref) > 8 * nch * C // 65536, len(isl_ref)
    # bitwise the two single calls, chunk numbering from 7
    so2, sc2, out2, cnt2 = D.decode(gpu_ctx, hm, dp, N, C, cap=1 << 18, first_chunk=7)
    so3, sc3 = D.viterbi(gpu_ctx, hm, dp, N, C)
    out3, cnt3 = D.islands(gpu_ctx, dp, so3, N, C, cap=1 << 18, first_chunk=7)
    torch.cuda.synchronize()
    gpu_ctx.sync()
    w = (N + 31) // 32
    assert np.array_equal(so2.cpu().numpy()[:w], so3.cpu().numpy()[:w])
    assert np.array_equal(sc2.cpu().numpy()[:nch], sc3.cpu().numpy()[:nch])
    assert np.array_equal(D.islands_to_numpy(out2, cnt2), D.islands_to_numpy(out3, cnt3))
    assert np.array_equal(D.islands_to_numpy(out2, cnt2)["chunk"], got["chunk"] + 7)


def test_decode_fused_capacity_and_empty(gpu_ctx, torch_dev):
    """cpg_decode_d: *d_count is the full count when records exceed cap (first cap records
    written), and a call with no whole chunk writes count 0 and a '-' tail."""
    import torch
    from cpgisland_amd import device as D
    C = 1 << 16
    N = 4 * C
    packed, _ = D.synth_host(77, 0, N)
    dp, _ = _dev_genome(packed, np.zeros(N // 32 + 1, np.uint32), torch_dev)
    hm = _model(_switchy_model(40.0))
    _, _, out, cnt = D.decode(gpu_ctx, hm, dp, N, C, cap=1 << 16)
    _, _, out3, cnt3 = D.decode(gpu_ctx, hm, dp, N, C, cap=3)
    torch.cuda.synchronize()
    gpu_ctx.sync()
    full = D.islands_to_numpy(out, cnt)
    assert int(cnt3.item()) == len(full) > 3
    assert np.array_equal(out3[:3].cpu().numpy().reshape(-1).view(co.ISLAND_DTYPE), full[:3])
    so = torch.full((8,), -1, dtype=torch.int32, device=torch_dev)
    _, _, _, c0 = D.decode(gpu_ctx, hm, dp, 100, C, sign_out=so)
    torch.cuda.synchronize()
    gpu_ctx.sync()
    assert int(c0.item()) == 0
    assert so.cpu().numpy()[:4].tolist() == [0, 0, 0, 0]


@pytest.mark.parametrize("world", [1, 2, 8])
def test_merge_train_records(gpu_ctx, torch_dev, world):
    """cpg_merge_train_d (the reducer over ranks): the fp64 parts summed in rank order —
    bitwise the sequential sum — and the int64 parts exactly, from one gathered buffer."""
    import torch
    from cpgisland_amd import device as D
    from cpgisland_amd import dist as cd
    rng = np.random.default_rng(world)
    e = rng.random((world, 105)) * 10.0 ** rng.integers(-3, 9, (world, 105))
    c = rng.integers(0, 1 << 40, (world, 124), dtype=np.int64)
    g = np.concatenate([e, c.view(np.float64)], axis=1).reshape(-1)
    gd = torch.from_numpy(g.copy()).to(torch_dev)
    oe = torch.empty(105, dtype=torch.float64, device=torch_dev)
    oc = torch.empty(124, dtype=torch.int64, device=torch_dev)
    D.merge_train(gpu_ctx, gd, world, oe, oc)
    ref = e[0].copy()
    for r in range(1, world):
        ref += e[r]
    assert np.array_equal(oe.cpu().numpy(), ref)
    assert np.array_equal(oc.cpu().numpy(), c.sum(axis=0))
    # the single-process record path (world 1 without a process group) is the identity
    rec, re_, rc = cd.train_record(torch_dev)
    re_.copy_(torch.from_numpy(e[0]))
    rc.copy_(torch.from_numpy(c[0]))
    cd.merge_train_records(gpu_ctx, rec, oe, oc)
    assert np.array_equal(oe.cpu().numpy(), e[0]) and np.array_equal(oc.cpu().numpy(), c[0])
