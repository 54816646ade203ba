"""Pin the library and both oracles to the reference's OWN bytes.

tests/golden/ref_constants.json is extracted from /root/reference/CpGIslandFinder.java by
tests/golden/make_ref_constants.py (the Java text parsed for its literals; nothing of the
reference runs).  Every constant the hot path uses is compared bitwise with it:
  * the initial model π / A / B (:155-173) — cpg_initial_model (libcpg.so, C-ABI), the C
    oracle and the Python oracle;
  * the chunk sizes 0x10000 / 0x100000 (:130-131, :230, :256-257) — cpg.h and the host module;
  * the island filter cg > 0.5, oe > 0.6 (:285) — the oracle's filter at the exact boundary
    values (the GPU island scan at the same boundaries: tests/test_gpu_parity.py);
  * the symbol map (:114-123) — cpg_ingest; the state order (:182-189) — HmmModel;
  * the island line format (:287) and the CLI argument order (:347-352) — the writers and
    cpgisland_amd.cli.
CPU only: no compute call touches a device.
"""
import json
import os
import re

import numpy as np
import pytest

from oracle import coracle as co
from oracle import pyref as pr

HERE = os.path.dirname(os.path.abspath(__file__))
REF = json.load(open(os.path.join(HERE, "golden", "ref_constants.json")))


def _hex(rows):
    return np.array([[float.fromhex(h) for h in r] for r in rows]) if isinstance(rows[0], list) \
        else np.array([float.fromhex(h) for h in rows])


def _bits_equal(a, b):
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    return a.shape == b.shape and np.array_equal(a.view(np.uint64), b.view(np.uint64))


PI = _hex(REF["initialP"]["hex"])
A = _hex(REF["transitionP"]["hex"])
B = _hex(REF["emissionP"]["hex"])


def test_fixture_literals_roundtrip():
    """The hex column is the correctly rounded binary64 of each literal (as javac rounds)."""
    for key in ("initialP", "transitionP", "emissionP"):
        lits = REF[key]["literals"]
        hexs = REF[key]["hex"]
        flat_l = sum(lits, []) if isinstance(lits[0], list) else lits
        flat_h = sum(hexs, []) if isinstance(hexs[0], list) else hexs
        assert [float(x).hex() for x in flat_l] == flat_h
    assert REF["initialP"]["lines"] == [155, 155]
    assert REF["transitionP"]["lines"] == [157, 164]
    assert REF["emissionP"]["lines"] == [166, 173]


def test_library_initial_model_bitwise():
    from cpgisland_amd import HmmModel
    m = HmmModel.initial()          # cpg_initial_model through the C-ABI (host function)
    assert _bits_equal(m.getInitialProbabilities(), PI)
    assert _bits_equal(m.getTransitionMatrix(), A)
    assert _bits_equal(m.getEmissionMatrix(), B)


def test_oracles_initial_model_bitwise():
    pi, a, b = co.model_split(co.initial_model())
    assert _bits_equal(pi, PI) and _bits_equal(a, A) and _bits_equal(b, B)
    assert _bits_equal(pr.INITIAL_PI, PI)
    assert _bits_equal(pr.INITIAL_A, A)
    assert _bits_equal(pr.INITIAL_B, B)


def test_chunk_constants():
    from cpgisland_amd import _lib
    ch = REF["chunks"]
    assert ch["train_chunk"]["line"] == 130 and ch["decode_chunk"]["line"] == 256
    assert _lib.TRAIN_CHUNK == ch["train_chunk"]["value"] == ch["train_vector_len"]["value"]
    assert _lib.DECODE_CHUNK == ch["decode_chunk"]["value"] == ch["decode_array_len"]["value"]
    hdr = open(os.path.join(HERE, "..", "include", "cpg.h")).read()
    assert int(re.search(r"#define CPG_TRAIN_CHUNK\s+(\d+)", hdr).group(1)) == 0x10000
    assert int(re.search(r"#define CPG_DECODE_CHUNK\s+(\d+)", hdr).group(1)) == 0x100000


def test_state_order_and_symbol_map():
    from cpgisland_amd import _lib
    hs = REF["hidden_states"]
    assert [k for k, _ in sorted(hs.items(), key=lambda kv: kv[1])] == \
        ["A+", "C+", "G+", "T+", "A-", "C-", "G-", "T-"]
    # symbols through the library's ingest: 'ACGTacgt' -> the reference's codes
    sym = REF["symbol_map"]
    txt = ("".join(sym.keys()) * 8192).encode()        # 65,536 bases: one training chunk
    packed = np.zeros(65536 // 16, np.uint32)
    nb = np.zeros(1, np.int64)
    _lib.check(_lib.lib.cpg_ingest(txt, len(txt), 0, 1, _lib.ptr(packed), 65536, _lib.ptr(nb)))
    assert nb[0] == 65536
    assert list(pr.unpack(packed, 8)) == [sym[c] for c in sym.keys()]


def _island_states(C, G, CG, L):
    """One island of length L with C C's, G G's and CG CpG steps, between '-' runs, in a
    1 Mi chunk of states (A- background)."""
    body = [1, 2] * CG + [1, 0] * (C - CG) + [2] * (G - CG)   # no other C->G step
    body += [0] * (L - len(body))
    assert len(body) == L and body.count(1) == C and body.count(2) == G
    st = np.full(1 << 20, 4, np.int32)
    st[1000:1000 + L] = body
    return st


@pytest.mark.parametrize("C,G,CG,L,keep", [
    (3, 2, 1, 10, False),       # cg = 0.5 exactly: not > 0.5
    (3, 3, 1, 11, True),        # cg = 6/11 > 0.5, oe = 11/9
    (5, 5, 1, 15, False),       # oe = 15/25 = 0.6 exactly: not > 0.6
    (5, 5, 1, 16, True),        # oe = 16/25 > 0.6, cg = 10/16
    (5, 5, 0, 15, False),       # oe = 0
])
def test_island_filter_thresholds(C, G, CG, L, keep):
    flt = REF["island_filter"]
    assert flt["line"] == 285 and flt["length_filter_commented_out"]
    cg_t, oe_t = float.fromhex(flt["cg_gt"]["hex"]), float.fromhex(flt["oe_gt"]["hex"])
    cg = (C + G) / L
    oe = (CG * L) / (C * G) if C and G else 0.0
    assert (cg > cg_t and oe > oe_t) == keep
    st = _island_states(C, G, CG, L)
    recs = co.islands(st, 0)
    assert len(recs) == (1 if keep else 0)
    assert len(pr.islands(st.tolist(), 0)) == len(recs)
    if keep:
        assert recs[0]["beg1"] == 1001 and recs[0]["end1"] == 1000 + L and recs[0]["len"] == L


def test_island_format_and_cli_args():
    assert REF["island_format"]["format"] == "%d %d %d %f %f\\n"
    assert [a for a, _ in REF["main_args"]] == ["trainingFile", "testFile", "stateSeqFile",
                                               "trainedHmmFile", "convergence", "numIter"]
    assert REF["bw_conf"]["SCALING_OPTION_KEY"] == "rescaling"
    assert REF["bw_conf"]["NUMBER_OF_HIDDEN_STATES_KEY"] == "8"
    assert REF["bw_conf"]["NUMBER_OF_EMITTED_STATES_KEY"] == "4"
