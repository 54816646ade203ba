"""C-ABI boundary (CPU only): libcpg.so loads, exports every symbol include/cpg.h declares,
and its host-side utilities (no device) agree with the oracle.  No compute calls."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from oracle import coracle as co
from oracle import pyref as pr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(ROOT, "include", "cpg.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(cpg_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from cpgisland_amd import _lib
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(_lib.lib, n), n
        assert n in _lib.SIGNATURES, f"{n} not bound in _lib.SIGNATURES"
    assert _lib.lib.cpg_abi_version() == 1


def test_struct_sizes_match_header():
    from cpgisland_amd import _lib
    assert _lib.ISLAND_DTYPE.itemsize == 32
    assert _lib.COUNTS_I64_N == 8 + 64 + 32 + 16 + 4
    assert _lib.COUNTS_F64_N == 8 + 64 + 32 + 1


def test_initial_model_matches_oracle():
    from cpgisland_amd import HmmModel
    assert np.array_equal(HmmModel.initial().to_struct(), co.initial_model())


def _ingest(txt, mode, quirks=1):
    from cpgisland_amd import _lib
    cap = len(txt) + (1 << 21)
    packed = np.zeros(cap // 16 + 8, np.uint32)
    nb = C.c_int64()
    rc = _lib.lib.cpg_ingest(txt, len(txt), mode, quirks, _lib.ptr(packed), cap, C.byref(nb))
    return rc, pr.unpack(packed, nb.value)


def test_ingest_train_matches_oracle():
    rng = np.random.default_rng(2)
    raw = rng.choice(list(b"ACGTacgtNn\n>"), 3 * 65536 + 999).astype(np.uint8).tobytes()
    rc, syms = _ingest(raw, 0)
    assert rc == 0
    assert np.array_equal(syms, co.ingest_train(raw))


def test_ingest_train_quirk_chunk():
    bases = (b"ACGT" * 16384)
    rc, syms = _ingest(bases + b"\n\n" + b"C" * 5, 0)
    assert rc == 0 and len(syms) == 3 * 65536 and not syms[65536:].any()
    rc, syms = _ingest(bases + b"\n\n", 0, quirks=0)
    assert rc == 0 and len(syms) == 65536


def test_ingest_decode_crash_code():
    from cpgisland_amd import _lib
    rc, syms = _ingest(b"G" * 0x100000 + b"\n", 1)
    assert rc == _lib.CPG_E_REF_CRASH and len(syms) == 0x100000
    rc, syms = _ingest(b"G" * 0x100000 + b"\n", 1, quirks=0)
    assert rc == 0 and len(syms) == 0x100000


def test_synth_is_counter_based_and_deterministic():
    from cpgisland_amd import device as D
    p1, s1 = D.synth_host(7, 0, 200000)
    p2, s2 = D.synth_host(7, 0, 200000, nthreads=1)
    assert np.array_equal(p1, p2) and np.array_equal(s1, s2)
    # a slice generated on its own equals the same bases of the whole
    p3, s3 = D.synth_host(7, 65536 + 32 * 5, 70000)
    whole = pr.unpack(p1, 200000)
    assert np.array_equal(pr.unpack(p3, 70000), whole[65536 + 160: 65536 + 160 + 70000])
    ws = pr.unpack_bits(s1, 200000)
    assert np.array_equal(pr.unpack_bits(s3, 70000), ws[65536 + 160: 65536 + 160 + 70000])
    # islands are planted: some '+' and mostly '-'
    assert 0.001 < ws.mean() < 0.1


def test_bw_normalize_bitwise_vs_oracle():
    from cpgisland_amd import _lib
    rng = np.random.default_rng(1)
    counts = rng.random(105) * 1000
    m = np.zeros(104)
    assert _lib.lib.cpg_bw_normalize(_lib.ptr(counts), _lib.ptr(m)) == 0
    assert np.array_equal(m, co.normalize(counts))


def test_counts_normalize():
    from cpgisland_amd import _lib
    rng = np.random.default_rng(1)
    c = rng.integers(1, 10 ** 9, 124).astype(np.int64)
    m = np.zeros(104)
    assert _lib.lib.cpg_counts_normalize(_lib.ptr(c), _lib.ptr(m)) == 0
    f = np.zeros(105)
    f[:104] = c[:104].astype(np.float64)
    assert np.array_equal(m, co.normalize(f))


def test_errors_are_codes_not_crashes():
    from cpgisland_amd import _lib
    assert _lib.lib.cpg_initial_model(None) == _lib.CPG_E_INVALID
    assert b"null" in _lib.lib.cpg_last_error()
    nb = C.c_int64()
    assert _lib.lib.cpg_ingest(None, 0, 0, 0, None, 0, C.byref(nb)) == _lib.CPG_E_INVALID
    assert _lib.lib.cpg_count_labelled_d(None, None, None, 0, 65536, None, None) == \
        _lib.CPG_E_INVALID


def test_open_without_gpu_reports_device_error():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from cpgisland_amd import _lib, Context
    with pytest.raises(_lib.CpgError) as e:
        Context(0)
    assert e.value.code == _lib.CPG_E_DEVICE
