"""Generate tests/golden/golden.npz — CPU-oracle vectors for the parity tests.

PARITY UNPINNED: the Java reference (plus unvendored Mahout / MAHOUT-627 /
Hadoop) cannot run in this container and ships no tests or fixtures.  These vectors come from
the C restatement (oracle/cpg_oracle.c); every vector is cross-checked here against the
independent Python restatement (oracle/pyref.py) on the sizes it can afford, and the script
refuses to write a fixture the two disagree on.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import coracle as co, pyref as pr  # noqa: E402
from cpgisland_amd import device as D  # noqa: E402  (host-only: cpg_synth)

SEED = 20251015
N = 1 << 20            # one decode chunk, 16 training chunks
TRAIN = 65536


def main():
    out = {}
    packed, sign = D.synth_host(SEED, 0, N)
    packed, sign = packed[: N // 16].copy(), sign[: N // 32].copy()
    obs = pr.unpack(packed, N)
    truth = pr.unpack_bits(sign, N)
    m0 = co.initial_model()
    # initial model agrees with the Python transcription of :155-173
    assert np.array_equal(m0, co.model_flat(pr.INITIAL_PI, pr.INITIAL_A, pr.INITIAL_B))
    out["synth_packed"], out["synth_truth"], out["model_initial"] = packed, sign, m0

    states, isl, score = co.decode_chunks(m0, obs, N)
    sg2, best2 = co.viterbi2(m0, obs)                 # independent 2-state restatement
    assert np.array_equal(sg2, (states < 4).astype(np.uint8)) and best2 == score[0]
    out["viterbi_sign"] = pr.pack_bits((states < 4).astype(np.uint8))
    out["viterbi_score"] = score
    out["islands"] = isl
    py_isl = pr.islands(states.tolist(), 0)
    assert [tuple(r) for r in py_isl] == [(r["beg1"], r["end1"], r["len"], r["cg"], r["oe"])
                                          for r in isl]
    out["islands_txt"] = np.array("".join(co.format_island(r) for r in isl))
    assert str(out["islands_txt"]) == "".join(pr.format_island(r) for r in py_isl)

    cnt = co.count_labelled(obs, truth, TRAIN)
    init, trans, emit, dinuc, mono = pr.count_labelled(obs, truth, TRAIN)
    assert np.array_equal(cnt, np.concatenate([init, trans.ravel(), emit.ravel(),
                                               dinuc.ravel(), mono]))
    out["counts_labelled"] = cnt

    est = co.estep(m0, obs, TRAIN)
    out["estep_counts"] = est
    m1 = co.normalize(est)
    out["model_trained1"] = m1
    st1, _, sc1 = co.decode_chunks(m1, obs, N)
    out["viterbi_sign_trained1"] = pr.pack_bits((st1 < 4).astype(np.uint8))
    out["viterbi_score_trained1"] = sc1

    # small cases: Python restatement == C oracle, bit for bit
    rng = np.random.default_rng(SEED)
    smalls = []
    for T in (1, 2, 3, 7, 64, 300):
        o = rng.integers(0, 4, T).astype(np.uint8)
        st, best = co.viterbi8(m0, o)
        seq, mp = pr.viterbi8(pr.INITIAL_PI, pr.INITIAL_A, pr.INITIAL_B, o.tolist())
        assert list(st) == seq and best == mp
        e = co.estep(m0, o, T)
        i, t, em, ll = pr.estep8(pr.INITIAL_PI, pr.INITIAL_A, pr.INITIAL_B, o.tolist())
        assert np.array_equal(e, np.concatenate([i, np.ravel(t), np.ravel(em), [ll]]))
        smalls.append((o, st, e))
    for k, (o, st, e) in enumerate(smalls):
        out[f"small{k}_obs"], out[f"small{k}_states"], out[f"small{k}_estep"] = o, st, e

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes;", len(isl), "islands")


if __name__ == "__main__":
    main()
