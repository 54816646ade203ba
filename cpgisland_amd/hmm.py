"""Host-side mirror of the reference's HMM types and decode entry point.

Mirrors the Mahout classes CpGIslandFinder uses (HmmModel, HmmEvaluator — imported at
/root/reference/CpGIslandFinder.java:9-10) with the same names, argument meaning and error
behaviour, over libcpg.so.  The compute is on the GPU (cpg_decode_states); this module
only validates and marshals.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import CpgInvalid, check, lib, ptr

# state order A+ C+ G+ T+ A- C- G- T- (:182-189); emitted symbols a c g t (:191-194)
HIDDEN_STATE_NAMES = ("A+", "C+", "G+", "T+", "A-", "C-", "G-", "T-")
EMITTED_STATE_NAMES = ("a", "c", "g", "t")


class HmmModel:
    """Mahout HmmModel(transitionMatrix, emissionMatrix, initialProbabilities)."""

    def __init__(self, transition, emission, initial):
        self.a = np.ascontiguousarray(transition, dtype=np.float64).reshape(8, 8).copy()
        self.b = np.ascontiguousarray(emission, dtype=np.float64).reshape(8, 4).copy()
        self.pi = np.ascontiguousarray(initial, dtype=np.float64).reshape(8).copy()

    # Mahout getters used at :204-222
    def getInitialProbabilities(self):
        return self.pi

    def getTransitionMatrix(self):
        return self.a

    def getEmissionMatrix(self):
        return self.b

    def getNrOfHiddenStates(self):
        return 8

    def getNrOfOutputStates(self):
        return 4

    def to_struct(self) -> np.ndarray:
        """cpg_model layout: pi[8] | a[8][8] | b[8][4]."""
        return np.concatenate([self.pi, self.a.ravel(), self.b.ravel()]).astype(np.float64)

    @classmethod
    def from_struct(cls, m: np.ndarray) -> "HmmModel":
        m = np.asarray(m, np.float64)
        return cls(m[8:72].reshape(8, 8), m[72:104].reshape(8, 4), m[:8])

    @classmethod
    def initial(cls) -> "HmmModel":
        """The model CpGIslandFinder.trainModel starts Baum-Welch from (:155-173)."""
        m = np.zeros(_lib.MODEL_N, np.float64)
        check(lib.cpg_initial_model(ptr(m)))
        return cls.from_struct(m)

    def __eq__(self, other):
        return isinstance(other, HmmModel) and np.array_equal(self.to_struct(), other.to_struct())

    def __repr__(self):
        return f"HmmModel(pi={self.pi.tolist()})"


class Context:
    """One libcpg context = one device (one process per GPU)."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        check(lib.cpg_open(device, C.byref(h)))
        self.handle = h
        self.device = device

    def close(self):
        if self.handle:
            lib.cpg_close(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self, stream=None):
        check(lib.cpg_sync(self.handle, stream))

    def reserve(self, nbases: int, general: bool = False, chunk_len: int | None = None):
        """cpg_reserve_ex: size the workspace for inputs of up to nbases bases at every decode
        chunk length that is a multiple of 256 (general=True: also the general-model
        Viterbi's, ~26 B per base); with chunk_len, cpg_reserve_chunk: for that one decode
        chunk length only."""
        if chunk_len is None:
            check(lib.cpg_reserve_ex(self.handle, int(nbases), 1 if general else 0))
        else:
            check(lib.cpg_reserve_chunk(self.handle, int(nbases), int(chunk_len),
                                        1 if general else 0))

    def workspace_bytes(self) -> int:
        """cpg_workspace_bytes: device workspace held by the context."""
        v = C.c_int64()
        check(lib.cpg_workspace_bytes(self.handle, C.byref(v)))
        return v.value


_default_ctx: Context | None = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


class HmmEvaluator:
    """Mahout HmmEvaluator — decode() is the entry point CpGIslandFinder calls (:260)."""

    @staticmethod
    def decode(model: HmmModel, observations, scaled: bool = True, ctx: Context | None = None):
        """Most likely hidden state sequence (int32 states 0..7), bit-identical to
        Mahout's sequential fp64 Viterbi (scaled=True).  Raises CpgInvalid (the
        reference's ArrayIndexOutOfBounds / NegativeArraySize) on symbols outside 0..3
        or an empty array."""
        if not scaled:
            raise ValueError("only scaled=True decoding is on the hot path "
                             "(CpGIslandFinder.java:260)")
        obs = np.ascontiguousarray(observations, dtype=np.int32)
        if obs.ndim != 1:
            raise CpgInvalid(_lib.CPG_E_INVALID, "observations must be 1-D")
        ctx = ctx or default_context()
        out = np.zeros(max(len(obs), 1), np.int32)
        m = model.to_struct()
        check(lib.cpg_decode_states(ctx.handle, ptr(m), ptr(obs) if len(obs) else None,
                                    len(obs), ptr(out)))
        return out[: len(obs)]


def format_islands(records) -> bytes:
    """The island file lines of CpGIslandFinder.java:287-288, byte-exact (cpg_format_islands)."""
    import ctypes as C

    from ._lib import ISLAND_DTYPE, check, lib, ptr
    recs = np.ascontiguousarray(records, dtype=ISLAND_DTYPE)
    need = C.c_int64(0)
    cap = max(64, len(recs) * 64)
    buf = C.create_string_buffer(cap)
    check(lib.cpg_format_islands(ptr(recs) if len(recs) else None, len(recs), buf, cap,
                                 C.byref(need)))
    return buf.raw[:need.value]


def format_model(model: "HmmModel") -> bytes:
    """The trained-model file of CpGIslandFinder.java:207-224, byte-exact (cpg_format_model)."""
    import ctypes as C

    from ._lib import check, lib, ptr
    need = C.c_int64(0)
    buf = C.create_string_buffer(8192)
    check(lib.cpg_format_model(ptr(model.to_struct()), buf, 8192, C.byref(need)))
    return buf.raw[:need.value]
