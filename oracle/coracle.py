"""ctypes loader for the C oracle (oracle/cpg_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker / the timed CPU baseline.  Never by the product.
PARITY UNPINNED (see cpg_oracle.h).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libcpg_oracle.so")
_lib = None

ISLAND_DTYPE = np.dtype([("beg1", "<i4"), ("end1", "<i4"), ("len", "<i4"),
                         ("chunk", "<i4"), ("cg", "<f8"), ("oe", "<f8")])
MODEL_N = 104
COUNTS_F64_N = 105
COUNTS_I64_N = 124

_P = C.c_void_p
_I64 = C.c_int64


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        L.orc_initial_model.argtypes = [_P]
        L.orc_ingest_train.argtypes = [_P, _I64, _P, _I64]
        L.orc_ingest_train.restype = _I64
        L.orc_ingest_decode.argtypes = [_P, _I64, _P, _I64, _P]
        L.orc_ingest_decode.restype = _I64
        L.orc_ingest_train_at.argtypes = [_P, _I64, _P, _I64, C.c_uint32, _P]
        L.orc_ingest_train_at.restype = _I64
        L.orc_ingest_decode_at.argtypes = [_P, _I64, _P, _I64, C.c_uint32, _P, _P]
        L.orc_ingest_decode_at.restype = _I64
        L.orc_viterbi8.argtypes = [_P, _P, _I64, _P]
        L.orc_viterbi8.restype = C.c_double
        L.orc_viterbi2.argtypes = [_P, _P, _I64, _P]
        L.orc_viterbi2.restype = C.c_double
        L.orc_estep8.argtypes = [_P, _P, _I64, _P]
        L.orc_normalize.argtypes = [_P, _P]
        L.orc_count_labelled.argtypes = [_P, _P, _I64, _I64, _P]
        L.orc_islands.argtypes = [_P, _I64, C.c_int32, _P, _I64]
        L.orc_islands.restype = _I64
        L.orc_format_island.argtypes = [_P, C.c_char_p, C.c_int]
        L.orc_format_island.restype = C.c_int
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.c_void_p)


# -- model helpers: a model is a flat float64[104] = pi[8] | a[8][8] | b[8][4] ---------
def model_flat(pi, a, b) -> np.ndarray:
    return np.concatenate([np.asarray(pi, np.float64).ravel(),
                           np.asarray(a, np.float64).ravel(),
                           np.asarray(b, np.float64).ravel()]).copy()


def model_split(m: np.ndarray):
    return m[:8].copy(), m[8:72].reshape(8, 8).copy(), m[72:104].reshape(8, 4).copy()


def initial_model() -> np.ndarray:
    m = np.zeros(MODEL_N, np.float64)
    lib().orc_initial_model(_ptr(m))
    return m


def ingest_train(txt: bytes) -> np.ndarray:
    buf = np.frombuffer(txt, np.uint8).copy()
    cap = (len(buf) // 0x10000 + len(buf) + 1) * 0x10000 if len(buf) < 1 << 20 else \
        (len(buf) // 0x10000 + 64) * 0x10000 * 2
    out = np.zeros(cap, np.uint8)
    n = lib().orc_ingest_train(_ptr(buf), len(buf), _ptr(out), cap)
    assert n >= 0
    return out[:n]


def ingest_decode(txt: bytes):
    buf = np.frombuffer(txt, np.uint8).copy()
    cap = (len(buf) // 0x100000 + 1) * 0x100000
    out = np.zeros(cap, np.uint8)
    crash = C.c_int(0)
    n = lib().orc_ingest_decode(_ptr(buf), len(buf), _ptr(out), cap, C.byref(crash))
    assert n >= 0
    return out[:n], bool(crash.value)


def ingest_at(txt: bytes, mode: int, count0: int):
    """The reader of `mode` (0 training, 1 decode) starting from Java count = count0 with an
    empty list (the 2^32-wrap test hook).  Returns (symbols, crash_byte or -1)."""
    buf = np.frombuffer(txt, np.uint8).copy()
    chunk = 0x10000 if mode == 0 else 0x100000
    extra = 0 if mode else int(np.count_nonzero(~np.isin(buf, np.frombuffer(b"ACGTacgt", np.uint8))))
    cap = (len(buf) // chunk + 2 + extra) * chunk
    out = np.zeros(cap, np.uint8)
    cb = C.c_int64(-1)
    if mode == 0:
        n = lib().orc_ingest_train_at(_ptr(buf), len(buf), _ptr(out), cap, count0, C.byref(cb))
    else:
        crash = C.c_int(0)
        n = lib().orc_ingest_decode_at(_ptr(buf), len(buf), _ptr(out), cap, count0,
                                       C.byref(crash), C.byref(cb))
    assert n >= 0
    return out[:n], int(cb.value)


def viterbi8(model: np.ndarray, obs: np.ndarray):
    obs = np.ascontiguousarray(obs, np.uint8)
    st = np.zeros(len(obs), np.int32)
    best = lib().orc_viterbi8(_ptr(model), _ptr(obs), len(obs), _ptr(st))
    return st, best


def viterbi2(model: np.ndarray, obs: np.ndarray):
    obs = np.ascontiguousarray(obs, np.uint8)
    sg = np.zeros(len(obs), np.uint8)
    best = lib().orc_viterbi2(_ptr(model), _ptr(obs), len(obs), _ptr(sg))
    return sg, best


def estep(model: np.ndarray, obs: np.ndarray, chunk_len: int) -> np.ndarray:
    """Sum of per-chunk E-step counts over whole chunks (chunk order)."""
    obs = np.ascontiguousarray(obs, np.uint8)
    acc = np.zeros(COUNTS_F64_N, np.float64)
    for c in range(len(obs) // chunk_len):
        lib().orc_estep8(_ptr(model), _ptr(obs[c * chunk_len:]), chunk_len, _ptr(acc))
    return acc


def normalize(counts: np.ndarray) -> np.ndarray:
    m = np.zeros(MODEL_N, np.float64)
    lib().orc_normalize(_ptr(np.ascontiguousarray(counts, np.float64)), _ptr(m))
    return m


def count_labelled(obs: np.ndarray, sign: np.ndarray, chunk_len: int) -> np.ndarray:
    acc = np.zeros(COUNTS_I64_N, np.int64)
    lib().orc_count_labelled(_ptr(np.ascontiguousarray(obs, np.uint8)),
                             _ptr(np.ascontiguousarray(sign, np.uint8)),
                             len(obs), chunk_len, _ptr(acc))
    return acc


def islands(states: np.ndarray, chunk: int) -> np.ndarray:
    states = np.ascontiguousarray(states, np.int32)
    n = lib().orc_islands(_ptr(states), len(states), chunk, None, 0)
    out = np.zeros(max(n, 1), ISLAND_DTYPE)
    lib().orc_islands(_ptr(states), len(states), chunk, _ptr(out), n)
    return out[:n]


def format_island(rec) -> str:
    r = np.zeros(1, ISLAND_DTYPE)
    r[0] = rec
    buf = C.create_string_buffer(256)
    n = lib().orc_format_island(_ptr(r), buf, 256)
    return buf.raw[:n].decode()


def decode_chunks(model: np.ndarray, obs: np.ndarray, chunk_len: int):
    """testModel (:256-340): Viterbi per whole chunk + island scan.  Returns
    (states int32[nchunks*chunk_len], islands records, best score per chunk)."""
    nch = len(obs) // chunk_len
    states = np.zeros(nch * chunk_len, np.int32)
    scores = np.zeros(nch, np.float64)
    recs = []
    for c in range(nch):
        st, best = viterbi8(model, obs[c * chunk_len:(c + 1) * chunk_len])
        states[c * chunk_len:(c + 1) * chunk_len] = st
        scores[c] = best
        recs.append(islands(st, c))
    isl = np.concatenate(recs) if recs else np.zeros(0, ISLAND_DTYPE)
    return states, isl, scores
