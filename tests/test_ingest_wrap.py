"""The readers' Java `int count` wrap at 2^32 bases (CpGIslandFinder.java:107/:127 training,
:236/:253 decode), reached through the test hooks that start `count` just below 2^32 with an
empty list (cpgx_ingest_at in libcpg.so — host code, no GPU; oracle orc_ingest_*_at; pyref
ingest(count0=...)).  All three against a hand-derived expectation:

* decode reader (:256-259): at count 2^32 the test is skipped (count == 0), the list keeps
  its 2^20 bases and grows; at the next multiple get(0 .. 2^20-1) copies the HELD chunk and
  clear() drops the 2^20 bases read after the wrap — no exception; a non-ACGT byte read while
  count == 0 fires nothing;
* training reader (:130-141): the same skipped test leaves 65,536 bases in the list; at the
  next multiple the 131,072-base list overflows DenseVector(0x10000).set (:133-134) — the run
  dies at the valid byte that brings count to 2^32 + 65,536.

PARITY UNPINNED (no JVM here): the expectation is derived from the Java text."""
import ctypes as C

import numpy as np
import pytest

from oracle import coracle as co
from oracle import pyref as pr

TRAIN = 65536
DECODE = 1 << 20
WRAP = 1 << 32


def _host_at(txt, mode, count0, cap, quirks=1):
    from cpgisland_amd import _lib
    packed = np.zeros(cap // 16 + 8, np.uint32)
    nb = C.c_int64()
    rc = _lib.lib.cpgx_ingest_at(txt, len(txt), mode, quirks, _lib.ptr(packed), cap,
                                 C.byref(nb), C.c_uint32(count0))
    return rc, nb.value, pr.unpack(packed, nb.value)


def _text(syms, inserts):
    """ACGT text of `syms` with bytes inserted after the given base indices."""
    seq = np.frombuffer(b"ACGT", np.uint8)[syms]
    parts, prev = [], 0
    for j, b in sorted(inserts.items()):
        parts += [seq[prev:j + 1].tobytes(), b]
        prev = j + 1
    parts.append(seq[prev:].tobytes())
    return b"".join(parts)


def _byte_of_base(txt, j):
    valid = np.isin(np.frombuffer(txt, np.uint8), np.frombuffer(b"ACGTacgt", np.uint8))
    return int(np.flatnonzero(valid)[j])


@pytest.fixture(scope="module")
def syms():
    return np.random.default_rng(77).integers(0, 4, 5 * DECODE + 123).astype(np.uint8)


def test_decode_reader_keeps_held_chunk_and_drops_the_next(syms):
    from cpgisland_amd import _lib
    c0 = WRAP - 2 * DECODE
    # a newline right after the base that wraps count to 0: fires nothing (count == 0)
    txt = _text(syms, {2 * DECODE - 1: b"\n", 100: b">x\n"})
    want = np.concatenate([syms[:2 * DECODE], syms[3 * DECODE:5 * DECODE]])
    got, cb = co.ingest_at(txt, 1, c0)
    assert cb == -1 and np.array_equal(got, want)
    rc, nb, hp = _host_at(txt, 1, c0, 8 * DECODE)
    assert rc == 0 and nb == 4 * DECODE and np.array_equal(hp, want)
    chunks, crash = pr.ingest(txt, DECODE, count0=c0)
    assert not crash and np.array_equal(np.concatenate(chunks), want)
    # without the wrap (count0 = 0) the same newline sits on count 2^21 with an empty list
    rc, nb, hp = _host_at(txt, 1, 0, 8 * DECODE)
    assert rc == _lib.CPG_E_REF_CRASH and np.array_equal(hp, syms[:2 * DECODE])


def test_decode_reader_crash_after_the_held_chunk(syms):
    from cpgisland_amd import _lib
    c0 = WRAP - 2 * DECODE
    # the newline after the base that brings count to 2^32 + 2^20 (the held chunk's commit)
    # finds the list empty: get(0) throws
    txt = _text(syms, {3 * DECODE - 1: b"\n"})
    kb = _byte_of_base(txt, 3 * DECODE - 1) + 1
    got, cb = co.ingest_at(txt, 1, c0)
    assert cb == kb and np.array_equal(got, syms[:2 * DECODE])
    rc, nb, hp = _host_at(txt, 1, c0, 8 * DECODE)
    assert rc == _lib.CPG_E_REF_CRASH and nb == 2 * DECODE
    assert np.array_equal(hp, syms[:2 * DECODE])
    assert f"byte {kb} " in _lib.lib.cpg_last_error().decode()
    chunks, crash = pr.ingest(txt, DECODE, count0=c0)
    assert crash and np.array_equal(np.concatenate(chunks), syms[:2 * DECODE])


def test_training_reader_throws_at_count_wrap_plus_chunk(syms):
    from cpgisland_amd import _lib
    c0 = WRAP - 2 * TRAIN
    s = syms[:4 * TRAIN]
    # a newline at count == 0 (after the wrap) emits no all-A chunk
    txt = _text(s, {2 * TRAIN - 1: b"\n"})
    kb = _byte_of_base(txt, 3 * TRAIN - 1)     # count -> 2^32 + 65,536: set(65536) throws
    got, cb = co.ingest_at(txt, 0, c0)
    assert cb == kb and np.array_equal(got, s[:TRAIN])
    rc, nb, hp = _host_at(txt, 0, c0, 16 * TRAIN)
    assert rc == _lib.CPG_E_REF_CRASH and nb == TRAIN and np.array_equal(hp, s[:TRAIN])
    assert f"byte {kb} " in _lib.lib.cpg_last_error().decode()
    chunks, crash = pr.ingest(txt, TRAIN, count0=c0)
    assert crash and np.array_equal(np.concatenate(chunks), s[:TRAIN])
    # ending before count 2^32 + 65,536: no crash, the held chunk is an unprocessed tail
    short = _text(s[:3 * TRAIN - 1], {2 * TRAIN - 1: b"\n"})
    got, cb = co.ingest_at(short, 0, c0)
    assert cb == -1 and np.array_equal(got, s[:TRAIN])
    rc, nb, hp = _host_at(short, 0, c0, 16 * TRAIN)
    assert rc == 0 and nb == TRAIN and np.array_equal(hp, s[:TRAIN])


def test_training_quirk_chunks_around_the_wrap(syms):
    """Newlines at count 2^32 - 65,536 (a multiple: one all-A chunk each) still count; the
    crash's committed-chunk count includes them."""
    from cpgisland_amd import _lib
    c0 = WRAP - 2 * TRAIN
    s = syms[:4 * TRAIN]
    txt = _text(s, {TRAIN - 1: b"\n\n"})
    want = np.concatenate([s[:TRAIN], np.zeros(2 * TRAIN, np.uint8)])
    got, cb = co.ingest_at(txt, 0, c0)
    assert cb == _byte_of_base(txt, 3 * TRAIN - 1) and np.array_equal(got, want)
    rc, nb, hp = _host_at(txt, 0, c0, 16 * TRAIN)
    assert rc == _lib.CPG_E_REF_CRASH and nb == 3 * TRAIN and np.array_equal(hp, want)
    chunks, crash = pr.ingest(txt, TRAIN, count0=c0)
    assert crash and np.array_equal(np.concatenate(chunks), want)


def test_count0_must_be_a_chunk_multiple():
    from cpgisland_amd import _lib
    rc, _, _ = _host_at(b"ACGT", 1, 12345, DECODE)
    assert rc == _lib.CPG_E_INVALID
