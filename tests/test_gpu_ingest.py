"""GPU parity of the device-side reader (cpg_ingest_d / cpg_ingest_gpu)
against the oracle's restatement of CpGIslandFinder.java:112-145 / :238-259 (Appendix A.1)
and the host cpg_ingest: committed chunks, the training reader's extra all-A chunks, the
decode reader's crash byte, capacity errors.  Bit-exact.  PARITY UNPINNED (no reference
fixtures exist; the restatement is cross-checked in tests/test_oracle.py)."""
import ctypes as C

import numpy as np
import pytest

from oracle import coracle as co
from oracle import pyref as pr

pytestmark = pytest.mark.gpu

TRAIN = 65536
DECODE = 1 << 20


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def fasta(rng, nbases, width, alphabet=b"ACGT", header=b">chr21 synthetic CGTA\n",
          nruns=()):
    seq = bytearray(rng.choice(list(alphabet), nbases).astype(np.uint8).tobytes())
    for pos, ln in nruns:          # N runs replacing bases
        seq[pos:pos + ln] = b"N" * ln
    lines = [bytes(seq[i:i + width]) for i in range(0, len(seq), width)]
    return header + b"\n".join(lines) + b"\n"


def _host(txt, mode, quirks, cap):
    from cpgisland_amd import _lib
    packed = np.zeros(cap // 16 + 8, np.uint32)
    nb = C.c_int64()
    rc = _lib.lib.cpg_ingest(txt, len(txt), mode, quirks, _lib.ptr(packed), cap, C.byref(nb))
    return rc, nb.value, packed


def _gpu(ctx, dev, txt, mode, quirks, cap):
    import torch
    from cpgisland_amd import device as D
    dt = D.text_to_device(txt, dev)
    out, res = D.ingest(ctx, dt, len(txt), mode, quirks, cap_bases=cap)
    torch.cuda.synchronize()
    return res.cpu().numpy(), out.cpu().numpy().view(np.uint32)


def _check(ctx, dev, txt, mode, quirks=1, cap=None):
    from cpgisland_amd import _lib
    chunk = TRAIN if mode == 0 else DECODE
    if cap is None:
        cap = (len(txt) // chunk + 8) * chunk
    rc, nb, hp = _host(txt, mode, quirks, cap)
    res, gp = _gpu(ctx, dev, txt, mode, quirks, cap)
    status = int(res[1])
    assert status == rc, (status, rc)
    assert int(res[0]) == nb
    assert np.array_equal(pr.unpack(gp, nb), pr.unpack(hp, nb))
    if rc == 0 and quirks:      # the oracle's reader (test restatement of A.1)
        if mode == 0:
            ref = co.ingest_train(txt)
        else:
            ref, crash = co.ingest_decode(txt)
            assert not crash
        assert np.array_equal(pr.unpack(gp, nb), ref)
    if rc == _lib.CPG_E_REF_CRASH:
        assert int(res[2]) >= 0
    return res, gp


@pytest.mark.parametrize("width", [60, 61, 64, 80, 128])
def test_fasta_train_all_line_widths(gpu_ctx, torch_dev, width):
    """Widths 64/128 put a newline on EVERY chunk boundary: one extra all-A chunk each."""
    rng = np.random.default_rng(width)
    txt = fasta(rng, 5 * TRAIN + 12345, width, alphabet=b"ACGTacgt", header=b">hmm\n")
    res, _ = _check(gpu_ctx, torch_dev, txt, 0)
    _check(gpu_ctx, torch_dev, fasta(rng, 5 * TRAIN + 12345, width), 0)   # header has ACGT
    if width in (64, 128):
        assert int(res[4]) == 5       # extra chunks
        assert int(res[0]) == 10 * TRAIN


def test_train_n_runs_across_boundaries_and_tiles(gpu_ctx, torch_dev):
    rng = np.random.default_rng(5)
    nb = 9 * TRAIN + 77
    runs = [(TRAIN - 3, 50000), (3 * TRAIN, 40000), (5 * TRAIN - 1, 70000), (8 * TRAIN, 3)]
    txt = fasta(rng, nb, 70, nruns=runs)
    _check(gpu_ctx, torch_dev, txt, 0)
    _check(gpu_ctx, torch_dev, txt, 0, quirks=0)


def test_train_random_bytes(gpu_ctx, torch_dev):
    rng = np.random.default_rng(2)
    raw = rng.choice(list(b"ACGTacgtNn\n>"), 3 * TRAIN + 999).astype(np.uint8).tobytes()
    _check(gpu_ctx, torch_dev, raw, 0)
    # every byte value, including 0x00 and high bytes, is skipped unless ACGT/acgt
    raw = rng.integers(0, 256, 2 * TRAIN * 3).astype(np.uint8).tobytes()
    _check(gpu_ctx, torch_dev, raw, 0)


EDGE = [b"", b"\n", b"NNNN", b"ACGT", b"A" * TRAIN, b"A" * TRAIN + b"\n",
        b"\n" * 40000 + b"C" * TRAIN + b"\n\n"]


@pytest.mark.parametrize("txt", EDGE, ids=[f"edge{i}" for i in range(len(EDGE))])
def test_small_and_edge_inputs(gpu_ctx, torch_dev, txt):
    _check(gpu_ctx, torch_dev, txt, 0)
    _check(gpu_ctx, torch_dev, txt, 1)


def test_decode_reader(gpu_ctx, torch_dev):
    from cpgisland_amd import _lib
    rng = np.random.default_rng(9)
    # width 60: no newline lands on a 2^20 multiple within 3 chunks -> no crash
    txt = fasta(rng, 3 * DECODE + 5000, 60)
    res, _ = _check(gpu_ctx, torch_dev, txt, 1)
    assert int(res[1]) == 0 and int(res[0]) == 3 * DECODE
    # width 64: the newline after base 2^20 is read on an empty list -> crash, 1 chunk kept
    txt = fasta(rng, 2 * DECODE + 5000, 64, header=b"")
    res, _ = _check(gpu_ctx, torch_dev, txt, 1)
    assert int(res[1]) == _lib.CPG_E_REF_CRASH and int(res[0]) == DECODE
    assert int(res[2]) == DECODE + DECODE // 64 - 1   # the newline ending line 16384
    _check(gpu_ctx, torch_dev, txt, 1, quirks=0)


def test_capacity(gpu_ctx, torch_dev):
    rng = np.random.default_rng(3)
    txt = fasta(rng, 6 * TRAIN + 5, 64)
    res, _ = _check(gpu_ctx, torch_dev, txt, 0, cap=5 * TRAIN + 100)
    assert int(res[1]) == -4 and int(res[0]) == 5 * TRAIN


def test_ingest_gpu_host_entry_matches_cpu_reader(gpu_ctx):
    from cpgisland_amd import _lib
    rng = np.random.default_rng(4)
    txt = fasta(rng, 4 * TRAIN + 1, 64, alphabet=b"ACGTNacgtn")
    cap = 16 * TRAIN
    for mode in (0, 1):
        rc, nb, hp = _host(txt, mode, 1, cap)
        gp = np.zeros(cap // 16 + 8, np.uint32)
        nb2 = C.c_int64()
        rc2 = _lib.lib.cpg_ingest_gpu(gpu_ctx.handle, txt, len(txt), mode, 1, _lib.ptr(gp), cap,
                                      C.byref(nb2))
        assert rc2 == rc and nb2.value == nb
        assert np.array_equal(pr.unpack(gp, nb), pr.unpack(hp, nb))


def test_large_synthetic_text_roundtrip(gpu_ctx, torch_dev):
    """46 Mbp-scale text (FASTA width 60): every committed base equals the packed genome."""
    import torch
    from cpgisland_amd import device as D
    n = 44 * DECODE
    packed, _ = D.synth_host(77, 0, n)
    syms = pr.unpack(packed, n)
    seq = np.frombuffer(b"ACGT", np.uint8)[syms]
    w = 60
    body = seq[: n // w * w].reshape(-1, w)
    txt = b">chr\n" + b"\n".join(bytes(r) for r in body) + b"\n" + bytes(seq[n // w * w:])
    dt = D.text_to_device(txt, torch_dev)
    for mode, chunk in ((0, TRAIN), (1, DECODE)):
        out, res = D.ingest(gpu_ctx, dt, len(txt), mode, True)
        torch.cuda.synchronize()
        r = res.cpu().numpy()
        # header ">chr" contributes C: 1 base before the sequence
        assert r[1] == 0 and r[3] == n + 1
        nb = int(r[0])
        got = pr.unpack(out.cpu().numpy().view(np.uint32), nb)
        ref = np.concatenate([[1], syms])[:nb]
        assert nb == (n + 1) // chunk * chunk + int(r[4]) * chunk
        if r[4] == 0:
            assert np.array_equal(got, ref)


def _gpu_at(ctx, txt, mode, count0, cap):
    from cpgisland_amd import _lib
    gp = np.zeros(cap // 16 + 8, np.uint32)
    nb = C.c_int64()
    rc = _lib.lib.cpgx_ingest_gpu_at(ctx.handle, txt, len(txt), mode, 1, _lib.ptr(gp), cap,
                                     C.byref(nb), C.c_uint32(count0))
    msg = _lib.lib.cpg_last_error().decode() if rc else ""
    return rc, nb.value, pr.unpack(gp, nb.value), msg


def _crash_byte(msg):
    import re
    m = re.search(r"byte (\d+) ", msg)
    return int(m.group(1)) if m else -1


WRAP_CASES = [   # (mode, count0, bases, FASTA width): the Java int count wraps inside the text
    (1, (1 << 32) - 2 * DECODE, 6 * DECODE + 77, 60),    # held chunk decoded, next dropped
    (1, (1 << 32) - 3 * DECODE, 7 * DECODE + 5, 61),
    (1, (1 << 32) - 2 * DECODE, 2 * DECODE + 5000, 60),  # ends inside the dropped window
    (0, (1 << 32) - 2 * TRAIN, 4 * TRAIN + 9, 64),       # all-A chunk, then the crash
    (0, (1 << 32) - 2 * TRAIN, 3 * TRAIN - 1, 60),       # ends before the crash
    (0, (1 << 32) - 5 * TRAIN, 9 * TRAIN, 70),
]


@pytest.mark.parametrize("case", WRAP_CASES, ids=[f"wrap{i}" for i in range(len(WRAP_CASES))])
def test_count_wrap_device_matches_host_and_oracle(gpu_ctx, case):
    """The device reader at the Java int count's 2^32 wrap (test hook cpgx_ingest_gpu_at:
    count starts at count0) against the host reader, the C oracle and the pure-Python one:
    committed bases, status, crash byte (tests/test_ingest_wrap.py derives the rules)."""
    from cpgisland_amd import _lib
    mode, c0, nbases, width = case
    rng = np.random.default_rng(nbases)
    txt = fasta(rng, nbases, width, header=b"")   # count0 sits on a multiple
    chunk = TRAIN if mode == 0 else DECODE
    cap = (nbases // chunk + 8) * chunk + len(txt) // width * chunk * (mode == 0)
    rc, nb, gp, msg = _gpu_at(gpu_ctx, txt, mode, c0, cap)
    hp_packed = np.zeros(cap // 16 + 8, np.uint32)
    hnb = C.c_int64()
    hrc = _lib.lib.cpgx_ingest_at(txt, len(txt), mode, 1, _lib.ptr(hp_packed), cap,
                                  C.byref(hnb), C.c_uint32(c0))
    hmsg = _lib.lib.cpg_last_error().decode() if hrc else ""
    assert (rc, nb) == (hrc, hnb.value)
    assert np.array_equal(gp, pr.unpack(hp_packed, nb))
    ref, cb = co.ingest_at(txt, mode, c0)
    assert np.array_equal(gp, ref)
    assert _crash_byte(msg) == _crash_byte(hmsg) == cb
    assert (rc == _lib.CPG_E_REF_CRASH) == (cb >= 0)
