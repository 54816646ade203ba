"""Pin the CPU oracle before trusting it (CPU only).

PARITY UNPINNED: the reference ships no tests/golden vectors and cannot run here (SURVEY.md
§8c).  The C restatement is pinned by (1) the independent Python restatement, (2) hand-derived
known-answer tests from SURVEY.md §4, (3) the committed golden vectors (tests/golden).
"""
import numpy as np
import pytest

from oracle import coracle as co
from oracle import pyref as pr

M0 = None


def m0():
    global M0
    if M0 is None:
        M0 = co.initial_model()
    return M0


def states_of(obs, sign):
    return obs.astype(np.int32) + np.where(np.asarray(sign) != 0, 0, 4)


# ---------------------------------------------------------------- model / ingest
def test_initial_model_matches_reference_constants():
    pi, a, b = co.model_split(m0())
    assert np.array_equal(pi, pr.INITIAL_PI)          # :155
    assert np.array_equal(a, pr.INITIAL_A)            # :157-164
    assert np.array_equal(b, pr.INITIAL_B)            # :166-173
    # rows 0-3 do not sum to 1 in fp64 (not renormalised by the reference)
    sums = [sum(r) for r in pr.INITIAL_A]
    assert sums[0] != 1.0 or sums[1] != 1.0


@pytest.mark.parametrize("txt", [b"", b"ACGT", b"acgtNNNNacgt\n>chr1 x\n", b"xyz" * 10])
def test_ingest_short_inputs_have_no_chunks(txt):
    assert len(co.ingest_train(txt)) == 0
    syms, crash = co.ingest_decode(txt)
    assert len(syms) == 0 and not crash


def test_ingest_train_quirk_extra_all_A_chunk():
    # :130-141 runs per character: a newline read while count sits on 65536 emits an
    # extra all-zero (all-'A') chunk
    rng = np.random.default_rng(1)
    bases = rng.choice(list(b"ACGT"), 65536).astype(np.uint8).tobytes()
    syms = co.ingest_train(bases + b"\n\n" + bases[:10])
    assert len(syms) == 3 * 65536
    assert np.array_equal(syms[:65536], pr.unpack(pr.pack(np.frombuffer(
        bases.translate(bytes.maketrans(b"ACGT", b"\0\1\2\3")), np.uint8)), 65536))
    assert not syms[65536:].any()
    chunks, crash = pr.ingest(bases + b"\n\n" + bases[:10], 0x10000)
    assert len(chunks) == 3 and not crash
    assert np.array_equal(np.concatenate(chunks).astype(np.uint8), syms)


def test_ingest_decode_crash_on_boundary_non_acgt():
    # :256-258: get(i) on an empty list throws IndexOutOfBoundsException
    bases = b"A" * 0x100000
    syms, crash = co.ingest_decode(bases + b"\n")
    assert crash and len(syms) == 0x100000
    syms, crash = co.ingest_decode(bases + b"C")
    assert not crash and len(syms) == 0x100000


def test_ingest_header_letters_count_as_bases():
    # FASTA header letters a/c/g/t are bases (:112-128): '>chr21 cat' contributes c,c,a,t
    chunks, _ = pr.ingest(b">chr21 cat\n" + b"G" * (65536 - 4), 0x10000)
    assert len(chunks) == 1 and chunks[0][:4] == [1, 1, 0, 3]


# ---------------------------------------------------------------- Viterbi
@pytest.mark.parametrize("T", [1, 2, 3, 5, 16, 17, 100, 257])
def test_viterbi_c_vs_python(T):
    rng = np.random.default_rng(T)
    obs = rng.integers(0, 4, T).astype(np.uint8)
    st, best = co.viterbi8(m0(), obs)
    seq, mp = pr.viterbi8(pr.INITIAL_PI, pr.INITIAL_A, pr.INITIAL_B, obs.tolist())
    assert list(st) == seq and best == mp
    sg, b2 = co.viterbi2(m0(), obs)
    assert np.array_equal(sg, (st < 4).astype(np.uint8)) and b2 == best


def test_viterbi_two_state_collapse_bitwise_long():
    rng = np.random.default_rng(7)
    obs = rng.integers(0, 4, 200000).astype(np.uint8)
    st, best = co.viterbi8(m0(), obs)
    sg, b2 = co.viterbi2(m0(), obs)
    assert np.array_equal(sg, (st < 4).astype(np.uint8)) and b2 == best


def test_viterbi_brute_force_small():
    """Enumerate all 2^T sign paths (T <= 12): the argmax value equals the Viterbi score."""
    import itertools
    import math
    rng = np.random.default_rng(3)
    for T in (2, 5, 9, 12):
        obs = rng.integers(0, 4, T).tolist()
        st, best = co.viterbi8(m0(), np.array(obs, np.uint8))
        bestv = -math.inf
        for signs in itertools.product((0, 1), repeat=T):
            s = [o + (0 if g else 4) for o, g in zip(obs, signs)]
            v = math.log(pr.INITIAL_PI[s[0]])
            for t in range(1, T):
                v += math.log(pr.INITIAL_A[s[t - 1]][s[t]])
            bestv = max(bestv, v)
        assert abs(bestv - best) <= 1e-12 * abs(best)
        # the decoded path scores the optimum
        v = math.log(pr.INITIAL_PI[st[0]])
        for t in range(1, T):
            v += math.log(pr.INITIAL_A[st[t - 1]][st[t]])
        assert abs(v - best) <= 1e-12 * abs(best)


def test_kat_cg_repeat_decodes_plus_and_at_repeat_minus():
    # SURVEY §4 known answers on a full 2^20 chunk
    n = 1 << 20
    cg = np.tile(np.array([1, 2], np.uint8), n // 2)
    sg, _ = co.viterbi2(m0(), cg)
    assert sg.all()
    at = np.tile(np.array([0, 3], np.uint8), n // 2)
    sg, _ = co.viterbi2(m0(), at)
    assert not sg.any()
    aa = np.zeros(n, np.uint8)                     # A-->A- 0.300 beats A+->A+ 0.170
    sg, _ = co.viterbi2(m0(), aa)
    assert not sg.any()


def test_degenerate_pi_zero_path_is_state_zero():
    """pi = 0 for both live states: every candidate is -inf, Mahout's maxProb starts at
    candidate 0, so delta stays -inf, maxState stays 0 at every step and the
    final argmax (strict '>' from -inf) leaves state 0: the path is all state 0 (A+)."""
    m = m0().copy()
    m[3] = 0.0
    m[7] = 0.0        # pi[T+] = pi[T-] = 0
    obs = np.array([3, 1, 2, 0, 3], np.uint8)
    st, best = co.viterbi8(m, obs)
    assert list(st) == [0, 0, 0, 0, 0]
    assert best == -np.inf
    sg, b2 = co.viterbi2(m, obs)          # the 2-state form: all '+', score -inf
    assert sg.all() and b2 == -np.inf
    seq, mp = pr.viterbi8(m[:8].tolist(), m[8:72].reshape(8, 8).tolist(),
                          m[72:].reshape(8, 4).tolist(), obs.tolist())
    assert seq == list(st)


# ---------------------------------------------------------------- E-step
@pytest.mark.parametrize("T", [1, 2, 9, 128, 500])
def test_estep_c_vs_python_bitwise(T):
    rng = np.random.default_rng(100 + T)
    obs = rng.integers(0, 4, T).astype(np.uint8)
    e = co.estep(m0(), obs, T)
    i, t, em, ll = pr.estep8(pr.INITIAL_PI, pr.INITIAL_A, pr.INITIAL_B, obs.tolist())
    assert np.array_equal(e, np.concatenate([i, np.ravel(t), np.ravel(em), [ll]]))


def test_estep_properties():
    rng = np.random.default_rng(11)
    T = 4096
    obs = rng.integers(0, 4, T).astype(np.uint8)
    e = co.estep(m0(), obs, T)
    init, trans, emit, ll = e[:8], e[8:72].reshape(8, 8), e[72:104].reshape(8, 4), e[104]
    assert abs(init.sum() - 1.0) < 1e-12
    assert abs(trans.sum() - (T - 1)) < 1e-9 * T           # sum_t sum xi = T-1
    assert abs(emit.sum() - T) < 1e-9 * T                  # sum_t sum gamma = T
    # emission column identity: emit[j] = init[j] + sum_i trans[i][j]
    col = init + trans.sum(axis=0)
    assert np.allclose(emit.sum(axis=1), col, rtol=1e-12, atol=1e-9)
    # deterministic emission preserved: only b[i][i%4] non-zero
    for i in range(8):
        for k in range(4):
            if k != i % 4:
                assert emit[i][k] == 0.0
    m1 = co.normalize(e)
    assert np.allclose(m1[8:72].reshape(8, 8).sum(axis=1), 1.0)
    assert np.array_equal(m1[72:].reshape(8, 4), np.array(pr.INITIAL_B))
    assert ll < 0


# ---------------------------------------------------------------- labelled counts
def test_counts_c_vs_numpy():
    rng = np.random.default_rng(5)
    n = 5 * 4096 + 77
    obs = rng.integers(0, 4, n).astype(np.uint8)
    sign = (rng.random(n) < 0.3).astype(np.uint8)
    c = co.count_labelled(obs, sign, 4096)
    init, trans, emit, dinuc, mono = pr.count_labelled(obs, sign, 4096)
    assert np.array_equal(c, np.concatenate([init, trans.ravel(), emit.ravel(), dinuc.ravel(),
                                             mono]))
    assert c[8:72].sum() == 5 * 4095 and c[120:].sum() == 5 * 4096


# ---------------------------------------------------------------- islands
def _random_states(rng, T):
    out = []
    while len(out) < T:
        plus = rng.random() < 0.5
        L = int(rng.integers(1, 40))
        b = rng.choice(4, L, p=[0.15, 0.35, 0.35, 0.15])
        out += [int(x) + (0 if plus else 4) for x in b]
    return np.array(out[:T], np.int32)


def test_islands_c_vs_python_random():
    rng = np.random.default_rng(9)
    for _ in range(300):
        T = int(rng.integers(1, 400))
        st = _random_states(rng, T)
        ch = int(rng.integers(0, 5000))
        a = co.islands(st, ch)
        b = pr.islands(st.tolist(), ch)
        assert [tuple(r)[:2] + (r["len"], r["cg"], r["oe"]) for r in a] == \
            [tuple(r) for r in b]


def test_islands_open_at_chunk_end_dropped():
    st = np.array([5, 1, 2, 1, 2, 1, 2], np.int32)     # island runs to the end: never closed
    assert len(co.islands(st, 0)) == 0
    st = np.array([5, 1, 2, 1, 2, 1, 2, 4], np.int32)
    r = co.islands(st, 0)
    assert len(r) == 1 and r[0]["beg1"] == 2 and r[0]["end1"] == 7 and r[0]["len"] == 6


def test_islands_stale_atC_quirk():
    # island 1 ends with C; island 2 starts with A then G: the stale atC (:325-331)
    # counts a CpG at island 2's first pair
    st = np.array([1, 2, 1, 4, 0, 2, 2, 1, 6], np.int32)
    recs = pr.islands(st.tolist(), 0)
    c_recs = co.islands(st, 0)
    assert len(recs) == len(c_recs) == 2
    # island 2: A G G C -> C=1 G=2; CpG: stale atC -> 1 (else 0); oe = 1*4/(1*2) = 2.0
    assert recs[1][4] == 2.0 and c_recs[1]["oe"] == 2.0


def test_islands_int32_overflow_of_cg_times_len():
    # cgCount*islandLen is Java int arithmetic (:283): a long (CG)^n island overflows and
    # its negative O/E ratio filters it out
    n = 70000
    st = np.array([1, 2] * (n // 2) + [4], np.int32)
    assert n // 2 * n > 2 ** 31
    assert len(co.islands(st, 0)) == 0
    st2 = np.array([1, 2] * 500 + [4], np.int32)
    assert len(co.islands(st2, 0)) == 1


def test_islands_coordinate_wrap_at_chunk_2048():
    st = np.array([4, 1, 2, 4] + [4] * 28, np.int32)
    r = co.islands(np.resize(st, 1 << 20), 2048)       # chunk*0x100000 = 2^31 wraps
    # island at index 1..2 of chunk 2048: beg + 2048*0x100000 + 1 wraps to -2^31 + 2
    assert len(r) > 0 and r[0]["beg1"] == -(2 ** 31) + 2 and r[0]["end1"] == -(2 ** 31) + 3


def test_java_percent_f_half_up():
    # Java %f rounds the shortest repr HALF_UP: 1/128 -> 0.007813 (C printf: 0.007812)
    assert pr.java_f6(0.0078125) == "0.007813"
    r = np.zeros(1, co.ISLAND_DTYPE)[0]
    r["beg1"], r["end1"], r["len"], r["cg"], r["oe"] = 1, 128, 128, 0.0078125, 1.0
    assert co.format_island(r) == "1 128 128 0.007813 1.000000\n"
    for x in (0.5, 0.6000005, 1.2345675, 0.999999501, 123.4567895, 2.0 / 3.0):
        r["cg"] = x
        assert co.format_island(r).split()[3] == pr.java_f6(x)


# ---------------------------------------------------------------- golden vectors
def test_golden_vectors_reproduce():
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden.npz"))
    N = 1 << 20
    obs = pr.unpack(g["synth_packed"], N)
    truth = pr.unpack_bits(g["synth_truth"], N)
    m = g["model_initial"]
    assert np.array_equal(m, co.initial_model())
    states, isl, score = co.decode_chunks(m, obs, N)
    assert np.array_equal(pr.pack_bits((states < 4).astype(np.uint8)), g["viterbi_sign"])
    assert np.array_equal(score, g["viterbi_score"])
    assert np.array_equal(isl, g["islands"])
    assert "".join(co.format_island(r) for r in isl) == str(g["islands_txt"])
    assert np.array_equal(co.count_labelled(obs, truth, 65536), g["counts_labelled"])
    est = co.estep(m, obs, 65536)
    assert np.array_equal(est, g["estep_counts"])
    assert np.array_equal(co.normalize(est), g["model_trained1"])
    for k in range(6):
        o = g[f"small{k}_obs"]
        st, _ = co.viterbi8(m, o)
        assert np.array_equal(st, g[f"small{k}_states"])
        assert np.array_equal(co.estep(m, o, len(o)), g[f"small{k}_estep"])


def test_dead_end_model_both_restatements():
    """Zero transitions C+/C- -> G+/G-: after a 'CG' every candidate is -inf, so (A.2) every
    later delta is -inf, every later backpointer 0 and the final state 0 — both restatements
    agree on states and score (the steps before the dead end keep their real argmax)."""
    pi, a, b = co.model_split(m0())
    a3 = a.copy()
    a3[np.ix_([1, 5], [2, 6])] = 0.0
    a3 /= a3.sum(1, keepdims=True)
    m3 = co.model_flat(pi, a3, b)
    obs = np.array([0, 3, 1, 2, 0, 1, 3], np.uint8)
    st, best = co.viterbi8(m3, obs)
    # from the dead end (t = 3) on the path is state 0; before it the real argmax
    assert best == -np.inf and list(st[3:]) == [0] * (len(obs) - 3) and st[2] == 1
    seq, mp = pr.viterbi8(m3[:8].tolist(), m3[8:72].reshape(8, 8).tolist(),
                          m3[72:].reshape(8, 4).tolist(), obs.tolist())
    assert seq == list(st) and mp == best


def test_non_deterministic_emissions_both_restatements():
    rng = np.random.default_rng(7)
    b = rng.random((8, 4))
    b /= b.sum(1, keepdims=True)
    pi, a, _ = co.model_split(m0())
    m = co.model_flat(pi, a, b)
    obs = rng.integers(0, 4, 300).astype(np.uint8)
    st, best = co.viterbi8(m, obs)
    seq, mp = pr.viterbi8(m[:8].tolist(), m[8:72].reshape(8, 8).tolist(),
                          m[72:].reshape(8, 4).tolist(), obs.tolist())
    assert seq == list(st) and mp == best
