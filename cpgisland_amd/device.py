"""HBM-resident hot path: torch tensors as device buffers, libcpg "_d" entry points.

PyTorch is plumbing here (device memory, streams, torch.distributed); every byte of the
hot path is computed by libcpg's HIP kernels.  Buffers are int32 tensors holding the raw
uint32 words of the packed / sign-bit layouts (include/cpg.h).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from ._lib import check, lib, ptr
from .hmm import Context, HmmModel


def _dp(t: torch.Tensor):
    assert t.is_cuda and t.is_contiguous()
    return C.c_void_p(t.data_ptr())


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def cu_stream(device_index: int, cus) -> "torch.cuda.ExternalStream":
    """A stream whose kernels run only on the compute units `cus` (cpg_stream_create_cu),
    wrapped for torch (events, `torch.cuda.stream(...)`).  Release it with
    cu_stream_destroy(stream) after its work has completed."""
    ncu = torch.cuda.get_device_properties(device_index).multi_processor_count
    words = np.zeros((ncu + 31) // 32, np.uint32)
    for cu in cus:
        words[cu // 32] |= np.uint32(1 << (cu % 32))
    h = C.c_void_p()
    check(lib.cpg_stream_create_cu(device_index, ptr(words), len(words), C.byref(h)))
    return torch.cuda.ExternalStream(h.value, device=torch.device("cuda", device_index))


def cu_stream_destroy(stream: "torch.cuda.ExternalStream") -> None:
    stream.synchronize()
    check(lib.cpg_stream_destroy(C.c_void_p(stream.cuda_stream)))


def words16(nbases: int) -> int:
    return (nbases + 15) // 16


def words32(nbases: int) -> int:
    return (nbases + 31) // 32


def synth_host(seed: int, start: int, n: int, nthreads: int = 0):
    """Synthetic genome slice (cpg_synth): (packed uint32[], sign uint32[])."""
    packed = np.zeros(words16(n) + 4, np.uint32)
    sign = np.zeros(words32(n) + 4, np.uint32)
    check(lib.cpg_synth(C.c_uint64(seed), start, n, ptr(packed), ptr(sign), nthreads))
    return packed, sign


def to_device(a: np.ndarray, device) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(device)


def count_labelled(ctx: Context, packed: torch.Tensor, sign: torch.Tensor, nbases: int,
                   chunk_len: int = _lib.TRAIN_CHUNK, out: torch.Tensor | None = None):
    if out is None:
        out = torch.empty(_lib.COUNTS_I64_N, dtype=torch.int64, device=packed.device)
    check(lib.cpg_count_labelled_d(ctx.handle, _dp(packed), _dp(sign), nbases, chunk_len,
                                   _dp(out), _stream()))
    return out


def bw_estep(ctx: Context, model: HmmModel, packed: torch.Tensor, nbases: int,
             chunk_len: int = _lib.TRAIN_CHUNK, out: torch.Tensor | None = None):
    if out is None:
        out = torch.empty(_lib.COUNTS_F64_N, dtype=torch.float64, device=packed.device)
    m = model.to_struct()
    check(lib.cpg_bw_estep_d(ctx.handle, ptr(m), _dp(packed), nbases, chunk_len, _dp(out),
                             _stream()))
    return out


def train_pass(ctx: Context, model: HmmModel, packed: torch.Tensor, sign: torch.Tensor,
               nbases: int, chunk_len: int = _lib.TRAIN_CHUNK,
               estep_out: torch.Tensor | None = None, counts_out: torch.Tensor | None = None):
    """bw_estep + count_labelled over the same chunks in one call (cpg_train_pass_d: one
    launch for chunk_len >= 16384).  Returns (E-step counts f64, labelled counts i64)."""
    if estep_out is None:
        estep_out = torch.empty(_lib.COUNTS_F64_N, dtype=torch.float64, device=packed.device)
    if counts_out is None:
        counts_out = torch.empty(_lib.COUNTS_I64_N, dtype=torch.int64, device=packed.device)
    m = model.to_struct()
    check(lib.cpg_train_pass_d(ctx.handle, ptr(m), _dp(packed), _dp(sign), nbases, chunk_len,
                               _dp(estep_out), _dp(counts_out), _stream()))
    return estep_out, counts_out


def merge_train(ctx: Context, gathered: torch.Tensor, world: int, estep_out: torch.Tensor,
                counts_out: torch.Tensor):
    """cpg_merge_train_d: `world` gathered rank records (TRAIN_RECORD words each: the E-step
    doubles, then the labelled-count int64) -> the fp64 sums in rank order + the int64 sums."""
    check(lib.cpg_merge_train_d(ctx.handle, _dp(gathered), world, _dp(estep_out),
                                _dp(counts_out), _stream()))
    return estep_out, counts_out


def viterbi(ctx: Context, model: HmmModel, packed: torch.Tensor, nbases: int,
            chunk_len: int = _lib.DECODE_CHUNK, sign_out: torch.Tensor | None = None,
            score: torch.Tensor | None = None):
    nch = nbases // chunk_len
    if sign_out is None:
        sign_out = torch.empty(words32(nbases) + 4, dtype=torch.int32, device=packed.device)
    if score is None:
        score = torch.empty(max(nch, 1), dtype=torch.float64, device=packed.device)
    m = model.to_struct()
    check(lib.cpg_viterbi_d(ctx.handle, ptr(m), _dp(packed), nbases, chunk_len, _dp(sign_out),
                            _dp(score), _stream()))
    return sign_out, score


def viterbi_states(ctx: Context, model: HmmModel, packed: torch.Tensor, nbases: int,
                   chunk_len: int = _lib.DECODE_CHUNK, states_out: torch.Tensor | None = None,
                   score: torch.Tensor | None = None):
    """HmmEvaluator.decode for ANY model (cpg_viterbi_states_d): one uint8 state per position
    of the whole chunks, and the best log-probability per chunk.  Returns (states, score)."""
    nch = nbases // chunk_len
    if states_out is None:
        states_out = torch.empty(max(nch * chunk_len, 1), dtype=torch.uint8, device=packed.device)
    if score is None:
        score = torch.empty(max(nch, 1), dtype=torch.float64, device=packed.device)
    m = model.to_struct()
    check(lib.cpg_viterbi_states_d(ctx.handle, ptr(m), _dp(packed), nbases, chunk_len,
                                   _dp(states_out), _dp(score), _stream()))
    return states_out, score


def islands(ctx: Context, packed: torch.Tensor, sign: torch.Tensor, nbases: int,
            chunk_len: int = _lib.DECODE_CHUNK, cap: int = 1 << 20, first_chunk: int = 0,
            out: torch.Tensor | None = None, count: torch.Tensor | None = None):
    """Island records (cpg_island, 32 B each) as a uint8 tensor [cap, 32] + int64 count."""
    if out is None:
        out = torch.empty((max(cap, 1), _lib.ISLAND_DTYPE.itemsize), dtype=torch.uint8,
                          device=packed.device)
    if count is None:
        count = torch.zeros(1, dtype=torch.int64, device=packed.device)
    check(lib.cpg_islands_at_d(ctx.handle, _dp(packed), _dp(sign), nbases, chunk_len,
                               first_chunk, _dp(out), cap, _dp(count), _stream()))
    return out, count


def decode(ctx: Context, model: HmmModel, packed: torch.Tensor, nbases: int,
           chunk_len: int = _lib.DECODE_CHUNK, cap: int = 1 << 20, first_chunk: int = 0,
           sign_out: torch.Tensor | None = None, score: torch.Tensor | None = None,
           out: torch.Tensor | None = None, count: torch.Tensor | None = None):
    """viterbi() then islands() in one call (cpg_decode_d): the reference's decode loop body
    (CpGIslandFinder.java:260 then :262-339).  Returns (sign_out, score, out, count)."""
    nch = nbases // chunk_len
    dev = packed.device
    if sign_out is None:
        sign_out = torch.empty(words32(nbases) + 4, dtype=torch.int32, device=dev)
    if score is None:
        score = torch.empty(max(nch, 1), dtype=torch.float64, device=dev)
    if out is None:
        out = torch.empty((max(cap, 1), _lib.ISLAND_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    if count is None:
        count = torch.zeros(1, dtype=torch.int64, device=dev)
    m = model.to_struct()
    check(lib.cpg_decode_d(ctx.handle, ptr(m), _dp(packed), nbases, chunk_len, first_chunk,
                           _dp(sign_out), _dp(score), _dp(out), cap, _dp(count), _stream()))
    return sign_out, score, out, count


def islands_to_numpy(out: torch.Tensor, count: torch.Tensor) -> np.ndarray:
    n = int(count.item())
    n = min(n, out.shape[0])
    return out[:n].cpu().numpy().reshape(-1).view(_lib.ISLAND_DTYPE)


def sign_to_numpy(sign: torch.Tensor, nbases: int) -> np.ndarray:
    w = sign.cpu().numpy().view(np.uint32)
    bits = ((w[:, None] >> np.arange(32, dtype=np.uint32)[None, :]) & 1).astype(np.uint8)
    return bits.ravel()[:nbases]


INGEST_RESULT_N = 8   # int64 fields of cpg_ingest_result


def text_to_device(txt: bytes, device) -> torch.Tensor:
    """Raw text bytes as a uint8 device tensor (16-byte aligned by the allocator)."""
    return torch.frombuffer(bytearray(txt) or bytearray(1), dtype=torch.uint8).to(device)


def ingest(ctx: Context, d_txt: torch.Tensor, n: int, mode: int, compat_quirks: bool = True,
           cap_bases: int | None = None, out: torch.Tensor | None = None,
           result: torch.Tensor | None = None):
    """Device-side reader (cpg_ingest_d): raw text in HBM -> packed committed chunks.

    Returns (packed int32 tensor, result int64[8] tensor = cpg_ingest_result), asynchronous
    on the current stream.  cap_bases defaults to n plus 1/8 slack for the training
    reader's extra all-A chunks (a FASTA file whose line cadence meets the chunk cadence gets
    one every few chunks), rounded to whole chunks; result[1] reports CPG_E_CAPACITY."""
    chunk = _lib.TRAIN_CHUNK if mode == 0 else _lib.DECODE_CHUNK
    if cap_bases is None:
        cap_bases = ((n + n // 8) // chunk + 8) * chunk
    if out is None:
        out = torch.empty(words16(cap_bases) + 4, dtype=torch.int32, device=d_txt.device)
    if result is None:
        result = torch.empty(INGEST_RESULT_N, dtype=torch.int64, device=d_txt.device)
    check(lib.cpg_ingest_d(ctx.handle, _dp(d_txt), n, mode, int(bool(compat_quirks)), _dp(out),
                           cap_bases, _dp(result), _stream()))
    return out, result


def genome_run(ctx: Context, train_model: HmmModel | None, decode_model: HmmModel | None,
               packed: np.ndarray, sign: np.ndarray | None, nbases: int,
               window_bases: int = 0, nbuf: int = 0, want_sign_out: bool = True,
               island_cap: int = 1 << 20, first_chunk: int = 0):
    """Streamed whole-genome pass from HOST memory (cpg_genome_run, BASELINE config C5).

    Returns a dict: estep (105 doubles) | counts (124 int64) | sign_out (uint32 words) |
    scores (per decode chunk) | islands (records)."""
    assert packed.dtype == np.uint32 and packed.flags["C_CONTIGUOUS"]
    opts = np.zeros(3, np.int64)
    opts[0] = window_bases
    opts[1] = nbuf            # nbuf (int32) + reserved (int32), little endian
    opts[2] = first_chunk
    est = np.zeros(_lib.COUNTS_F64_N, np.float64) if train_model is not None else None
    cnt = np.zeros(_lib.COUNTS_I64_N, np.int64) if sign is not None else None
    ndec = nbases // _lib.DECODE_CHUNK
    sg = np.zeros(words32(nbases) + 1, np.uint32) if (decode_model is not None and
                                                       want_sign_out) else None
    sc = np.zeros(max(ndec, 1), np.float64) if decode_model is not None else None
    isl = np.zeros(max(island_cap, 1), _lib.ISLAND_DTYPE) if decode_model is not None else None
    icount = C.c_int64(0)
    tm = train_model.to_struct() if train_model is not None else None
    dm = decode_model.to_struct() if decode_model is not None else None

    def p(a):
        return ptr(a) if a is not None else None

    check(lib.cpg_genome_run(ctx.handle, p(tm), p(dm), ptr(packed),
                             p(sign) if sign is not None else None, nbases, ptr(opts),
                             p(est), p(cnt), p(sg), p(sc), p(isl), island_cap if isl is not None
                             else 0, C.byref(icount) if dm is not None else None))
    return {"estep": est, "counts": cnt, "sign_out": sg, "scores": sc[:ndec] if sc is not None
            else None, "islands": isl[:icount.value] if isl is not None else None,
            "island_count": icount.value}


# ---- ragged contig batches (BASELINE config C4) ------------------------------------------
def contig_layout(lens: np.ndarray, gap: int = 0):
    """64-aligned offsets for contigs of the given lengths packed back to back (plus `gap`
    bases between them): (offs int64[n], nbases span)."""
    lens = np.asarray(lens, np.int64)
    step = (lens + gap + 63) // 64 * 64
    offs = np.zeros(len(lens), np.int64)
    if len(lens) > 1:
        offs[1:] = np.cumsum(step)[:-1]
    span = int(offs[-1] + lens[-1]) if len(lens) else 0
    return offs, span


def contigs_order(ctx: Context, lens: torch.Tensor, n: int, out: torch.Tensor | None = None):
    if out is None:
        out = torch.empty(max(n, 1), dtype=torch.int32, device=lens.device)
    check(lib.cpg_contigs_order_d(ctx.handle, _dp(lens), n, _dp(out), _stream()))
    return out


def _opt(t):
    return _dp(t) if t is not None else None


def contigs_count_labelled(ctx, packed, sign, nbases, offs, lens, order, n, out=None):
    if out is None:
        out = torch.empty(_lib.COUNTS_I64_N, dtype=torch.int64, device=packed.device)
    check(lib.cpg_contigs_count_labelled_d(ctx.handle, _dp(packed), _dp(sign), nbases, _dp(offs),
                                           _dp(lens), _opt(order), n, _dp(out), _stream()))
    return out


def contigs_estep(ctx, model: HmmModel, packed, nbases, offs, lens, order, n, out=None):
    if out is None:
        out = torch.empty(_lib.COUNTS_F64_N, dtype=torch.float64, device=packed.device)
    m = model.to_struct()
    check(lib.cpg_contigs_estep_d(ctx.handle, ptr(m), _dp(packed), nbases, _dp(offs), _dp(lens),
                                  _opt(order), n, _dp(out), _stream()))
    return out


def contigs_viterbi(ctx, model: HmmModel, packed, nbases, offs, lens, order, n,
                    sign_out=None, score=None):
    if sign_out is None:
        sign_out = torch.zeros(words32(nbases) + 4, dtype=torch.int32, device=packed.device)
    if score is None:
        score = torch.empty(max(n, 1), dtype=torch.float64, device=packed.device)
    m = model.to_struct()
    check(lib.cpg_contigs_viterbi_d(ctx.handle, ptr(m), _dp(packed), nbases, _dp(offs), _dp(lens),
                                    _opt(order), n, _dp(sign_out), _dp(score), _stream()))
    return sign_out, score


def contigs_islands(ctx, packed, sign, nbases, offs, lens, order, n, cap=1 << 20, out=None,
                    count=None):
    if out is None:
        out = torch.empty((max(cap, 1), _lib.ISLAND_DTYPE.itemsize), dtype=torch.uint8,
                          device=packed.device)
    if count is None:
        count = torch.zeros(1, dtype=torch.int64, device=packed.device)
    check(lib.cpg_contigs_islands_d(ctx.handle, _dp(packed), _dp(sign), nbases, _dp(offs),
                                    _dp(lens), _opt(order), n, _dp(out), cap, _dp(count),
                                    _stream()))
    return out, count
