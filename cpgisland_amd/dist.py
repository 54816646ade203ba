"""Multi-GPU layer: one process per GPU, contiguous genome shards, RCCL for the reducer only.

The reference's two stages are chunk-independent (training chunks of 65,536 bases,
CpGIslandFinder.java:130-141; decode chunks of 1,048,576 bases, :256-260), so a shard made of
whole decode chunks needs no data-path exchange at all:

  * shard_bounds()       rank r owns a contiguous run of whole 1 Mi chunks; the last rank also
                         owns the tail, which both stages drop exactly as the unsharded run does
  * merge_counts_i64()   labelled int64 counts: all-reduce sum (exact in any order)
  * merge_counts_f64()   E-step fp64 counts (the MapReduce reducer's sum): all-gather + sum in
                         rank order, so every rank gets the same bits on every run
  * gather_islands()     island records of every rank in rank (= chunk) order; coordinates are
                         global because each shard decodes with its first chunk index
                         (cpg_islands_at_d)
  * ShardRunner          the per-rank training pass + decode on that rank's device

Backend "nccl" is RCCL over xGMI on the GPU box; "gloo" runs the same code on CPU tensors
(tests/test_dist.py).  All messages are < 1 KiB except the island gather.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from . import _lib


def shard_bounds(nbases: int, world: int, rank: int,
                 align: int = _lib.DECODE_CHUNK) -> tuple[int, int]:
    """(start, length) of rank's contiguous shard: whole `align` chunks, balanced, the
    remainder (tail) on the last rank.  Shards of whole decode chunks are whole training
    chunks too (2^20 is a multiple of 2^16)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    nch = nbases // align
    per, extra = divmod(nch, world)
    c0 = rank * per + min(rank, extra)
    c1 = c0 + per + (1 if rank < extra else 0)
    start = c0 * align
    end = nbases if rank == world - 1 else c1 * align
    return start, end - start


def _group_size(group) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def merge_counts_i64(counts: torch.Tensor, group=None) -> torch.Tensor:
    """Labelled counts (cpg_counts_i64 layout): integer sums are exact in any order."""
    if _group_size(group) > 1:
        dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=group)
    return counts


def merge_counts_f64(counts: torch.Tensor, group=None) -> torch.Tensor:
    """E-step counts (cpg_counts_f64 layout): gathered, then summed in rank order on every
    rank — bitwise identical everywhere, independent of the collective's algorithm."""
    ws = _group_size(group)
    if ws == 1:
        return counts
    parts = [torch.empty_like(counts) for _ in range(ws)]
    dist.all_gather(parts, counts, group=group)
    acc = parts[0].clone()
    for p in parts[1:]:
        acc += p
    counts.copy_(acc)
    return counts


def gather_islands(records: np.ndarray, device, group=None) -> np.ndarray:
    """Concatenate every rank's island records (ISLAND_DTYPE) in rank order, on all ranks."""
    ws = _group_size(group)
    if ws == 1:
        return records
    raw = np.ascontiguousarray(records).view(np.uint8).reshape(-1)
    n = torch.tensor([raw.size], dtype=torch.int64, device=device)
    sizes = [torch.empty_like(n) for _ in range(ws)]
    dist.all_gather(sizes, n, group=group)
    mx = max(int(s.item()) for s in sizes)
    buf = torch.zeros(max(mx, 1), dtype=torch.uint8, device=device)
    buf[: raw.size] = torch.from_numpy(raw).to(device)
    bufs = [torch.empty_like(buf) for _ in range(ws)]
    dist.all_gather(bufs, buf, group=group)
    out = [b[: int(s.item())].cpu().numpy() for b, s in zip(bufs, sizes)]
    return np.concatenate(out).view(_lib.ISLAND_DTYPE)


class ShardRunner:
    """One rank's part of the training pass and the decode, on its own device.

    packed / sign: this rank's shard (device tensors, words of include/cpg.h layouts),
    start: the shard's first base in genome coordinates (a multiple of 2^20)."""

    def __init__(self, ctx, packed: torch.Tensor, nbases: int, start: int,
                 sign: torch.Tensor | None = None, group=None):
        if start % _lib.DECODE_CHUNK:
            raise ValueError("shard start must be 1 Mi-aligned (decode chunk boundary)")
        self.ctx, self.packed, self.sign, self.n, self.start = ctx, packed, sign, nbases, start
        self.group = group

    def labelled_counts(self) -> torch.Tensor:
        from . import device as D
        return merge_counts_i64(D.count_labelled(self.ctx, self.packed, self.sign, self.n),
                                self.group)

    def estep(self, model) -> np.ndarray:
        from . import device as D
        return merge_counts_f64(D.bw_estep(self.ctx, model, self.packed, self.n),
                                self.group).cpu().numpy()

    def decode(self, model, cap: int = 1 << 20):
        """Exact Viterbi of the shard's whole chunks + island scan with global chunk
        numbering; returns (sign tensor, scores, all ranks' islands in genome order)."""
        from . import device as D
        sign, score = D.viterbi(self.ctx, model, self.packed, self.n)
        out, cnt = D.islands(self.ctx, self.packed, sign, self.n, cap=cap,
                             first_chunk=self.start // _lib.DECODE_CHUNK)
        isl = D.islands_to_numpy(out, cnt)
        return sign, score, gather_islands(isl, self.packed.device, self.group)
