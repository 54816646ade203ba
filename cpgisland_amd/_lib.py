"""ctypes binding of libcpg.so (include/cpg.h) — the only way into the hot path.

There is deliberately no fallback: if the in-tree native library is missing, importing
this module raises.  Build it with `python -c "import __graft_entry__ as g; g.build()"`
or `make -C cpgisland_amd/csrc`.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libcpg.so")   # the in-tree build, nothing else

CPG_OK = 0
CPG_E_INVALID = -1
CPG_E_DEVICE = -2
CPG_E_UNSUPPORTED = -3
CPG_E_CAPACITY = -4
CPG_E_REF_CRASH = -5
CPG_E_VERIFY = -6
TRAIN_CHUNK = 65536
DECODE_CHUNK = 1048576
COUNTS_I64_N = 124
COUNTS_F64_N = 105
MODEL_N = 104

ISLAND_DTYPE = np.dtype([("beg1", "<i4"), ("end1", "<i4"), ("len", "<i4"),
                         ("chunk", "<i4"), ("cg", "<f8"), ("oe", "<f8")])

_NAMES = {CPG_E_INVALID: "CPG_E_INVALID", CPG_E_DEVICE: "CPG_E_DEVICE",
          CPG_E_UNSUPPORTED: "CPG_E_UNSUPPORTED", CPG_E_CAPACITY: "CPG_E_CAPACITY",
          CPG_E_REF_CRASH: "CPG_E_REF_CRASH", CPG_E_VERIFY: "CPG_E_VERIFY"}


class CpgError(RuntimeError):
    """A negative status from libcpg (code + cpg_last_error message)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"{_NAMES.get(code, code)}: {msg}")
        self.code = code


class CpgInvalid(CpgError, ValueError):
    """CPG_E_INVALID — the reference's IllegalArgument / IndexOutOfBounds family."""


_P = C.c_void_p
_I64 = C.c_int64
_INT = C.c_int

# (name, argtypes) for every symbol include/cpg.h declares
SIGNATURES = {
    "cpg_open": [_INT, _P],
    "cpg_close": [_P],
    "cpg_last_error": [],
    "cpg_abi_version": [],
    "cpg_reserve": [_P, _I64],
    "cpg_reserve_ex": [_P, _I64, _INT],
    "cpg_reserve_chunk": [_P, _I64, _I64, _INT],
    "cpg_workspace_bytes": [_P, _P],
    "cpg_sync": [_P, _P],
    "cpg_stream_create_cu": [_INT, _P, _INT, _P],
    "cpg_stream_destroy": [_P],
    "cpg_initial_model": [_P],
    "cpg_ingest": [C.c_char_p, C.c_size_t, _INT, _INT, _P, _I64, _P],
    "cpg_synth": [C.c_uint64, _I64, _I64, _P, _P, _INT],
    "cpg_bw_normalize": [_P, _P],
    "cpg_counts_normalize": [_P, _P],
    "cpg_count_labelled_d": [_P, _P, _P, _I64, _I64, _P, _P],
    "cpg_bw_estep_d": [_P, _P, _P, _I64, _I64, _P, _P],
    "cpg_train_pass_d": [_P, _P, _P, _P, _I64, _I64, _P, _P, _P],
    "cpg_merge_train_d": [_P, _P, _INT, _P, _P, _P],
    "cpg_viterbi_d": [_P, _P, _P, _I64, _I64, _P, _P, _P],
    "cpg_viterbi_states_d": [_P, _P, _P, _I64, _I64, _P, _P, _P],
    "cpg_islands_d": [_P, _P, _P, _I64, _I64, _P, _I64, _P, _P],
    "cpg_islands_at_d": [_P, _P, _P, _I64, _I64, _I64, _P, _I64, _P, _P],
    "cpg_decode_d": [_P, _P, _P, _I64, _I64, _I64, _P, _P, _P, _I64, _P, _P],
    "cpg_count_labelled": [_P, _P, _P, _I64, _I64, _P],
    "cpg_bw_estep": [_P, _P, _P, _I64, _I64, _P],
    "cpg_viterbi": [_P, _P, _P, _I64, _I64, _P, _P],
    "cpg_decode_states": [_P, _P, _P, _I64, _P],
    "cpg_islands": [_P, _P, _P, _I64, _I64, _P, _I64, _P],
    "cpg_ingest_d": [_P, _P, _I64, _INT, _INT, _P, _I64, _P, _P],
    "cpg_ingest_gpu": [_P, C.c_char_p, C.c_size_t, _INT, _INT, _P, _I64, _P],
    "cpg_genome_run": [_P, _P, _P, _P, _P, _I64, _P, _P, _P, _P, _P, _P, _I64, _P],
    "cpg_contigs_order_d": [_P, _P, _I64, _P, _P],
    "cpg_format_islands": [_P, _I64, _P, _I64, _P],
    "cpg_format_model": [_P, _P, _I64, _P],
    "cpg_contigs_count_labelled_d": [_P, _P, _P, _I64, _P, _P, _P, _I64, _P, _P],
    "cpg_contigs_estep_d": [_P, _P, _P, _I64, _P, _P, _P, _I64, _P, _P],
    "cpg_contigs_viterbi_d": [_P, _P, _P, _I64, _P, _P, _P, _I64, _P, _P, _P],
    "cpg_contigs_islands_d": [_P, _P, _P, _I64, _P, _P, _P, _I64, _P, _I64, _P, _P],
}

# test hooks exported by libcpg.so outside the C-ABI (cpg_internal.h): the readers started
# from a given Java `count` (the 2^32 wrap with a few MB of text; tests only)
TEST_HOOKS = {
    "cpgx_ingest_at": [C.c_char_p, C.c_size_t, _INT, _INT, _P, _I64, _P, C.c_uint32],
    "cpgx_ingest_gpu_at": [_P, C.c_char_p, C.c_size_t, _INT, _INT, _P, _I64, _P, C.c_uint32],
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libcpg.so not built at {LIB_PATH}: run `make -C cpgisland_amd/csrc` "
            "(there is no CPU fallback for the hot path)")
    # ONE HIP runtime per process: torch bundles its own libamdhip64 (soname libamdhip64.so.7,
    # the same as /opt/rocm's, which libcpg.so needs), but torch's libraries ask for it as
    # "libamdhip64.so".  Loaded after libcpg.so, torch therefore maps a second runtime beside
    # the first, and whichever initialises second finds no device (seen on the GPU box when
    # this package was imported before torch).  Loaded first, torch's runtime is the one
    # libcpg.so's dependency resolves to.  (A host without torch — the Java FFM binding — uses
    # /opt/rocm's runtime alone.)
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(LIB_PATH)
    for name, args in {**SIGNATURES, **TEST_HOOKS}.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = _INT
    lib.cpg_last_error.restype = C.c_char_p
    lib.cpg_close.restype = None
    return lib


lib = _load()


def check(rc: int) -> int:
    if rc < 0:
        msg = lib.cpg_last_error().decode(errors="replace")
        if rc == CPG_E_INVALID:
            raise CpgInvalid(rc, msg)
        raise CpgError(rc, msg)
    return rc


def ptr(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return C.c_void_p(a.ctypes.data)
