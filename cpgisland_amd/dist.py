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

Shards need not be chunk-aligned: with boundaries at any multiple of 64 bases (an even split
of a genome, shard_bounds(..., align=64)), every chunk is processed by the rank that holds its
first base, and a chunk that runs past the end of that rank's shard is completed with the
next rank's first bases — one all-gather of every rank's first 2^20 bases (packed + sign words,
384 KB per rank), the halo:

  * shard_plan()         the chunks a rank owns and the base range its local buffer covers
  * halo_exchange()      the all-gather; returns the next rank's head
  * local_buffers()      the rank's own words from its first owned chunk + the halo
  * HaloShardRunner      ShardRunner over such a shard

Every chunk is then computed whole, on one device, by the same kernels as the unsharded run:
counts, island records and decoded paths are bit-identical to it for any shard boundaries.

Backend "nccl" is RCCL over xGMI on the GPU box; "gloo" runs the same code on CPU tensors
(tests/test_dist.py).  All messages are < 1 KiB except the island gather.
"""
from __future__ import annotations

from dataclasses import dataclass

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


TRAIN_RECORD = 105 + 124   # words: cpg_counts_f64 doubles, then cpg_counts_i64 int64


def train_record(device):
    """One rank's training-pass record (CPG_TRAIN_RECORD_BYTES): a float64 tensor whose first
    105 words are the E-step counts and whose last 124 are the labelled counts (int64 view)
    — pass the two views to device.train_pass as its outputs."""
    rec = torch.empty(TRAIN_RECORD, dtype=torch.float64, device=device)
    return rec, rec[:105], rec[105:].view(torch.int64)


def merge_train_records(ctx, rec: torch.Tensor, estep_out: torch.Tensor, counts_out: torch.Tensor,
                        group=None, gathered: torch.Tensor | None = None):
    """The reducer over ranks in one collective: all-gather of every rank's record, then every
    rank sums the records itself (cpg_merge_train_d on the GPU: doubles in rank order —
    bitwise identical on every rank — and exact integers; numpy on CPU tensors)."""
    ws = _group_size(group)
    if gathered is None:
        gathered = torch.empty(ws * TRAIN_RECORD, dtype=torch.float64, device=rec.device)
    if ws > 1:
        if dist.get_backend(group) == "nccl":
            dist.all_gather_into_tensor(gathered, rec, group=group)
        else:
            dist.all_gather(list(gathered.view(ws, TRAIN_RECORD)), rec, group=group)
    else:
        gathered.copy_(rec)
    if rec.is_cuda:
        from . import device as D
        D.merge_train(ctx, gathered, ws, estep_out, counts_out)
    else:
        g = gathered.view(ws, TRAIN_RECORD)
        e = g[0, :105].clone()
        for r in range(1, ws):
            e += g[r, :105]
        estep_out.copy_(e)
        counts_out.copy_(g[:, 105:].contiguous().view(torch.int64).sum(dim=0))
    return estep_out, counts_out


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


# ---------------------------------------------------------------- unaligned shards (halo)
HALO_ALIGN = 64   # shard boundaries: whole sign words (32 bases) and count blocks (64 bases)


def chunk_span(start: int, n: int, nbases: int, chunk: int) -> tuple[int, int]:
    """Indices [c0, c1) of the whole `chunk`-base chunks of a genome of `nbases` bases (the
    reference drops the tail) whose first base lies in [start, start + n)."""
    last = nbases // chunk
    c0 = min(-(-start // chunk), last)
    c1 = min(-(-(start + n) // chunk), last)
    return c0, max(c0, c1)


@dataclass(frozen=True)
class ShardPlan:
    start: int      # the shard: bases [start, start + n) of the genome
    n: int
    t0: int         # owned training chunks [t0, t1) and decode chunks [d0, d1)
    t1: int
    d0: int
    d1: int
    base: int       # the local buffer: bases [base, end)
    end: int
    train: int
    decode: int

    @property
    def halo(self) -> int:
        """Bases past the shard's end that its last chunk needs (from the next rank)."""
        return max(0, self.end - (self.start + self.n))


def shard_plan(start: int, n: int, nbases: int, train: int = _lib.TRAIN_CHUNK,
               decode: int = _lib.DECODE_CHUNK) -> ShardPlan:
    if start % HALO_ALIGN or (start + n < nbases and n % HALO_ALIGN) or decode % train:
        raise ValueError("shard boundaries must be multiples of 64 bases; decode chunk a "
                         "multiple of the training chunk")
    t0, t1 = chunk_span(start, n, nbases, train)
    d0, d1 = chunk_span(start, n, nbases, decode)
    firsts = ([t0 * train] if t1 > t0 else []) + ([d0 * decode] if d1 > d0 else [])
    ends = ([t1 * train] if t1 > t0 else []) + ([d1 * decode] if d1 > d0 else [])
    base = min(firsts) if firsts else start
    end = max(ends) if ends else base
    return ShardPlan(start, n, t0, t1, d0, d1, base, end, train, decode)


def halo_exchange(packed: torch.Tensor, sign: torch.Tensor, n: int, group=None,
                  width: int = _lib.DECODE_CHUNK):
    """All-gather of every rank's first `width` bases (packed and sign words, zero-padded)
    and of every rank's shard length; returns the next rank's (packed head, sign head, shard
    length), or (None, None, 0) on the last rank.  The length lets local_buffers refuse a
    halo that would run past the next rank's shard into its zero padding."""
    ws = _group_size(group)
    if ws == 1:
        return None, None, 0
    rank = dist.get_rank(group)
    w16, w32 = width // 16, width // 32
    hp = torch.zeros(w16, dtype=packed.dtype, device=packed.device)
    hs = torch.zeros(w32, dtype=sign.dtype, device=sign.device)
    k16, k32 = min(w16, (n + 15) // 16), min(w32, (n + 31) // 32)
    hp[:k16] = packed[:k16]
    hs[:k32] = sign[:k32]
    gp = [torch.empty_like(hp) for _ in range(ws)]
    gs = [torch.empty_like(hs) for _ in range(ws)]
    nt = torch.tensor([n], dtype=torch.int64, device=packed.device)
    gn = [torch.empty_like(nt) for _ in range(ws)]
    dist.all_gather(gp, hp, group=group)
    dist.all_gather(gs, hs, group=group)
    dist.all_gather(gn, nt, group=group)
    if rank == ws - 1:
        return None, None, 0
    return gp[rank + 1], gs[rank + 1], int(gn[rank + 1].item())


def local_buffers(packed: torch.Tensor, sign: torch.Tensor, plan: ShardPlan,
                  head_p: torch.Tensor | None, head_s: torch.Tensor | None,
                  head_n: int | None = None):
    """The rank's packed / sign words of bases [plan.base, plan.end): its own words from
    plan.base, then the halo from the next rank's head (padded by 4 words, as the kernels'
    buffers are).  head_n: the next rank's shard length (halo_exchange returns it); a halo
    longer than it would take zero padding for bases, so it is refused."""
    if plan.halo and (head_p is None or plan.halo > head_p.numel() * 16):
        raise ValueError("the halo reaches past the next rank's head: shards must hold at "
                         "least one decode chunk")
    if plan.halo and head_n is not None and plan.halo > head_n:
        raise ValueError(f"the halo ({plan.halo} bases) runs past the next rank's shard "
                         f"({head_n} bases): every shard but the last must hold at least "
                         f"one decode chunk")
    off = plan.base - plan.start
    own = min(plan.start + plan.n, plan.end) - plan.base
    if own < 0 or off < 0:
        raise ValueError("bad shard plan")
    p = [packed[off // 16: off // 16 + (own + 15) // 16]]
    s = [sign[off // 32: off // 32 + (own + 31) // 32]]
    if plan.halo:
        p.append(head_p[: (plan.halo + 15) // 16])
        s.append(head_s[: (plan.halo + 31) // 32])
    pad_p = torch.zeros(4, dtype=packed.dtype, device=packed.device)
    pad_s = torch.zeros(4, dtype=sign.dtype, device=sign.device)
    return torch.cat(p + [pad_p]), torch.cat(s + [pad_s])


class HaloShardRunner:
    """ShardRunner over a shard with boundaries at any multiple of 64 bases: the chunks whose
    first base the shard holds, each computed whole (with the halo from the next rank)."""

    def __init__(self, ctx, packed: torch.Tensor, sign: torch.Tensor, start: int, n: int,
                 nbases: int, group=None, heads=None):
        """heads: (packed head, sign head, next shard length) as halo_exchange returns them
        (None: run the exchange here)."""
        self.ctx, self.group = ctx, group
        self.plan = shard_plan(start, n, nbases)
        hd = heads if heads is not None else halo_exchange(packed, sign, n, group)
        hp, hs = hd[0], hd[1]
        hn = hd[2] if len(hd) > 2 else None
        self.packed, self.sign = local_buffers(packed, sign, self.plan, hp, hs, hn)

    def _train_view(self):
        pl = self.plan
        o = pl.t0 * pl.train - pl.base
        return (self.packed[o // 16:], self.sign[o // 32:], (pl.t1 - pl.t0) * pl.train)

    def labelled_counts(self) -> torch.Tensor:
        from . import device as D
        p, s, n = self._train_view()
        return merge_counts_i64(D.count_labelled(self.ctx, p, s, n), self.group)

    def estep(self, model) -> np.ndarray:
        from . import device as D
        p, _, n = self._train_view()
        return merge_counts_f64(D.bw_estep(self.ctx, model, p, n), self.group).cpu().numpy()

    def decode(self, model, cap: int = 1 << 20):
        """Exact Viterbi of the owned decode chunks + island scan with global chunk numbers;
        returns (sign tensor of the owned chunks, scores, all ranks' islands in genome
        order)."""
        from . import device as D
        pl = self.plan
        o = pl.d0 * pl.decode - pl.base
        p = self.packed[o // 16:]
        n = (pl.d1 - pl.d0) * pl.decode
        sign, score = D.viterbi(self.ctx, model, p, n)
        out, cnt = D.islands(self.ctx, p, sign, n, cap=cap, first_chunk=pl.d0)
        isl = D.islands_to_numpy(out, cnt)
        return sign, score, gather_islands(isl, self.packed.device, self.group)
