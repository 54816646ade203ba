"""Multi-process (world size 2 and 3, gloo on CPU) tests of the multi-GPU host layer
(cpgisland_amd/dist.py, baumwelch.run(distributed=True)).

The per-shard compute is the oracle here (test infrastructure, CPU), standing in for the
per-rank GPU kernels, so that the sharding, the reducer merges and the island gather — the
code that runs unchanged over RCCL on the GPU box — are checked against the unsharded run.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cpgisland_amd import HmmModel
from cpgisland_amd import dist as cd
from cpgisland_amd import _lib
from oracle import coracle as co
from oracle import pyref as pr

TRAIN = 4096          # small chunks keep the oracle fast; the logic is size-independent
DECODE = 65536
N = 5 * DECODE + 1234  # 5 whole decode chunks + a tail both stages drop


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _genome():
    from cpgisland_amd import device as D
    packed, sign = D.synth_host(4242, 0, N)
    return pr.unpack(packed, N), pr.unpack_bits(sign, N)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        obs, truth = _genome()
        start, n = cd.shard_bounds(N, world, rank, align=DECODE)
        o, tr = obs[start:start + n], truth[start:start + n]
        m = co.initial_model()
        # labelled counts: int64 all-reduce
        li = cd.merge_counts_i64(torch.from_numpy(co.count_labelled(o, tr, TRAIN)))
        # E-step counts: all-gather + rank-order sum (identical bits on every rank)
        part = co.estep(m, o, TRAIN)
        fe = cd.merge_counts_f64(torch.from_numpy(part.copy()))
        # the same reduction as one all-gather of each rank's training record (bench.py's
        # reducer): identical bits
        rec, re, rc = cd.train_record("cpu")
        re.copy_(torch.from_numpy(part))
        rc.copy_(torch.from_numpy(co.count_labelled(o, tr, TRAIN)))
        me, mc = torch.empty(105, dtype=torch.float64), torch.empty(124, dtype=torch.int64)
        cd.merge_train_records(None, rec, me, mc)
        assert torch.equal(me, fe) and torch.equal(mc, li)
        # decode: per shard, global chunk numbering, gathered in genome order
        recs = [co.islands(co.viterbi8(m, o[c * DECODE:(c + 1) * DECODE])[0],
                           start // DECODE + c) for c in range(n // DECODE)]
        isl = np.concatenate(recs) if recs else np.zeros(0, co.ISLAND_DTYPE)
        gi = cd.gather_islands(isl.view(_lib.ISLAND_DTYPE), torch.device("cpu"))
        # Baum-Welch driver over the shards (oracle mapper), 3 iterations
        bw, it, ll = __import__("cpgisland_amd.baumwelch", fromlist=["run"]).run(
            None, None, n, max_iter=3, convergence=0.0, distributed=True,
            mapper=lambda mm: torch.from_numpy(co.estep(mm.to_struct(), o, TRAIN)))
        q.put((rank, start, n, li.numpy(), fe.numpy(), part, gi.view(np.uint8).copy(),
               bw.to_struct(), it, ll))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_pass_equals_unsharded(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_worker, args=(world, _free_port(), q), nprocs=world, join=True,
                       start_method="spawn")
    res = sorted([q.get() for _ in range(world)], key=lambda r: r[0])
    obs, truth = _genome()
    m = co.initial_model()
    # shards tile the genome, whole decode chunks each, the tail on the last rank
    assert res[0][1] == 0 and sum(r[2] for r in res) == N
    assert all(r[1] % DECODE == 0 for r in res)
    # labelled counts: bit-exact vs the unsharded run, on every rank
    full_i = co.count_labelled(obs, truth, TRAIN)
    for r in res:
        assert np.array_equal(r[3], full_i)
    # E-step: every rank has the same bits = rank-order sum of the parts; ~ unsharded
    ref_sum = res[0][5].copy()
    for r in res[1:]:
        ref_sum += r[5]
    for r in res:
        assert np.array_equal(r[4], ref_sum)
    full_e = co.estep(m, obs, TRAIN)
    nz = full_e != 0
    assert np.max(np.abs(ref_sum[nz] - full_e[nz]) / np.abs(full_e[nz])) < 1e-12
    # islands: the gathered records equal the unsharded decode's, in genome order
    _, isl, _ = co.decode_chunks(m, obs, DECODE)
    assert len(isl) > 0
    for r in res:
        assert np.array_equal(r[6].view(co.ISLAND_DTYPE), isl)
    # Baum-Welch over shards: identical models on every rank, ~ the unsharded driver
    for r in res:
        assert np.array_equal(r[7], res[0][7]) and r[8] == 3
    mo = m
    for _ in range(3):
        mo = co.normalize(co.estep(mo, obs, TRAIN))
    assert np.allclose(res[0][7], mo, rtol=1e-11, atol=0)


@pytest.mark.parametrize("n,world", [(0, 1), (DECODE - 1, 2), (3 * DECODE, 2),
                                     (7 * DECODE + 5, 4), (2 * DECODE, 8)])
def test_shard_bounds_tile(n, world):
    spans = [cd.shard_bounds(n, world, r, align=DECODE) for r in range(world)]
    pos = 0
    for s, ln in spans:
        assert s == pos and s % DECODE == 0 and ln >= 0
        pos += ln
    assert pos == n
    # whole chunks are balanced within one chunk
    whole = [ln // DECODE for _, ln in spans]
    assert max(whole) - min(whole) <= 1 and sum(whole) == n // DECODE


def test_single_process_merges_are_identity():
    t = torch.arange(5, dtype=torch.float64)
    assert cd.merge_counts_f64(t.clone()).equal(t)
    assert cd.merge_counts_i64(t.long()).equal(t.long())
    with pytest.raises(ValueError):
        cd.shard_bounds(10, 2, 2)


# ---------------------------------------------------------------- unaligned shards (halo)
def _halo_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        obs, truth = _genome()
        start, n = cd.shard_bounds(N, world, rank, align=cd.HALO_ALIGN)
        # this rank's own words only (its first base at bit 0), as a loader would produce them
        pk = torch.from_numpy(pr.pack(obs[start:start + n]).view(np.int32).copy())
        sg = torch.from_numpy(pr.pack_bits(truth[start:start + n]).view(np.int32).copy())
        plan = cd.shard_plan(start, n, N, train=TRAIN, decode=DECODE)
        hp, hs, hn = cd.halo_exchange(pk, sg, n, width=DECODE)
        lp, ls = cd.local_buffers(pk, sg, plan, hp, hs, hn)
        span = plan.end - plan.base
        lo = pr.unpack(lp.numpy().view(np.uint32), span)
        lt = pr.unpack_bits(ls.numpy().view(np.uint32), span)
        # the local buffer IS the genome's bases [base, end): halo included
        assert np.array_equal(lo, obs[plan.base:plan.end])
        assert np.array_equal(lt, truth[plan.base:plan.end])
        m = co.initial_model()
        to, tn = plan.t0 * TRAIN - plan.base, (plan.t1 - plan.t0) * TRAIN
        li = cd.merge_counts_i64(torch.from_numpy(
            co.count_labelled(lo[to:to + tn], lt[to:to + tn], TRAIN)))
        fe = cd.merge_counts_f64(torch.from_numpy(co.estep(m, lo[to:to + tn], TRAIN)))
        do = plan.d0 * DECODE - plan.base
        recs = [co.islands(co.viterbi8(m, lo[do + c * DECODE:do + (c + 1) * DECODE])[0],
                           plan.d0 + c) for c in range(plan.d1 - plan.d0)]
        isl = np.concatenate(recs) if recs else np.zeros(0, co.ISLAND_DTYPE)
        gi = cd.gather_islands(isl.view(_lib.ISLAND_DTYPE), torch.device("cpu"))
        q.put((rank, start, n, plan.halo, li.numpy(), fe.numpy(), gi.view(np.uint8).copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_unaligned_shards_with_halo_equal_unsharded(world):
    """Shards split at multiples of 64 bases (not at chunk boundaries): every chunk is run by
    the rank holding its first base, completed by the halo all-gather — counts and island
    records equal the unsharded run's."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_halo_worker, args=(world, _free_port(), q), nprocs=world, join=True,
                       start_method="spawn")
    res = sorted([q.get() for _ in range(world)], key=lambda r: r[0])
    obs, truth = _genome()
    assert sum(r[2] for r in res) == N
    assert any(r[1] % DECODE for r in res)       # really unaligned
    assert any(r[3] > 0 for r in res)            # some chunk needed the halo
    full_i = co.count_labelled(obs, truth, TRAIN)
    m = co.initial_model()
    full_e = co.estep(m, obs, TRAIN)
    _, isl, _ = co.decode_chunks(m, obs, DECODE)
    nz = full_e != 0
    for r in res:
        assert np.array_equal(r[4], full_i)
        assert np.array_equal(r[5], res[0][5])
        assert np.max(np.abs(r[5][nz] - full_e[nz]) / np.abs(full_e[nz])) < 1e-12
        assert np.array_equal(r[6].view(co.ISLAND_DTYPE), isl)


def test_halo_longer_than_next_shard_is_refused():
    """a short middle shard cannot supply the previous rank's halo; the halo would
    be read from the zero padding of its head (as base 'A'), so local_buffers raises."""
    n_genome = 4 * DECODE
    # rank 0: [0, DECODE + 64) owns decode chunk 0 and chunk 1 (first base DECODE) -> halo
    plan = cd.shard_plan(0, DECODE + 64, n_genome, train=TRAIN, decode=DECODE)
    assert plan.halo == DECODE - 64
    pk = torch.zeros((DECODE + 64) // 16, dtype=torch.int32)
    sg = torch.zeros((DECODE + 64) // 32, dtype=torch.int32)
    hp = torch.zeros(DECODE // 16, dtype=torch.int32)
    hs = torch.zeros(DECODE // 32, dtype=torch.int32)
    with pytest.raises(ValueError, match="next rank's shard"):
        cd.local_buffers(pk, sg, plan, hp, hs, 4096)          # next shard: 4096 bases only
    lp, ls = cd.local_buffers(pk, sg, plan, hp, hs, DECODE)   # long enough: accepted
    assert lp.numel() == (plan.end - plan.base) // 16 + 4


@pytest.mark.parametrize("n,world", [(5 * DECODE + 1234, 2), (5 * DECODE + 1234, 4),
                                     (3_100_000_000, 8)])
def test_shard_plans_cover_every_chunk_once(n, world):
    plans = [cd.shard_plan(*cd.shard_bounds(n, world, r, align=cd.HALO_ALIGN), n)
             for r in range(world)]
    for a, b in zip(plans, plans[1:]):
        assert a.t1 == b.t0 and a.d1 == b.d0       # chunk ranges tile
        assert a.halo <= b.n                        # the halo is inside the next shard
    assert plans[0].t0 == 0 and plans[-1].t1 == n // _lib.TRAIN_CHUNK
    assert plans[0].d0 == 0 and plans[-1].d1 == n // _lib.DECODE_CHUNK
    for p in plans:
        assert p.halo < _lib.DECODE_CHUNK
    with pytest.raises(ValueError):
        cd.shard_plan(100, 64, n)                   # not a multiple of 64


# ---------------------------------------------------------------- bench.py's C3 step transfers
def _c3_comm_worker(rank, world, port, q):
    """bench.py's C3 halo (point to point: rank r sends its first plans[r-1].halo bases to
    r-1, received into the tail of r-1's local buffer) and island gather to rank 0, with the
    gloo staging of the rehearsal path, on CPU tensors."""
    import importlib.util
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        spec = importlib.util.spec_from_file_location(
            "bench", os.path.join(os.path.dirname(os.path.dirname(__file__)), "bench.py"))
        bench = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(bench)
        obs, truth = _genome()
        spans = [cd.shard_bounds(N, world, r, align=cd.HALO_ALIGN) for r in range(world)]
        plans = [cd.shard_plan(s, n, N, train=TRAIN, decode=DECODE) for s, n in spans]
        start, n = spans[rank]
        pl = plans[rank]
        own = pr.pack(obs[start:start + n]).view(np.int32)
        span = pl.end - pl.base
        buf = torch.zeros((span + 15) // 16 + 4, dtype=torch.int32)
        ow = min(start + n, pl.end) - pl.base
        o16 = (pl.base - start) // 16
        buf[:(ow + 15) // 16] = torch.from_numpy(own[o16:o16 + (ow + 15) // 16].copy())
        ops = []
        ph = plans[rank - 1].halo if rank > 0 else 0
        if ph:
            ops.append(("send", torch.from_numpy(own[:(ph + 15) // 16].copy()), rank - 1))
        if pl.halo:
            t16 = (start + n - pl.base) // 16
            ops.append(("recv", buf[t16:t16 + (pl.halo + 15) // 16], rank + 1))
        if ops:
            bench._p2p(ops, "gloo")
        got = pr.unpack(buf.numpy().view(np.uint32), span)
        ok_halo = bool(np.array_equal(got, obs[pl.base:pl.end]))
        recs = torch.full((3, 4), rank, dtype=torch.int64)
        outs = [torch.empty(3, 4, dtype=torch.int64) for _ in range(world)] if rank == 0 else None
        bench._gather0(recs, world, rank, "gloo", outs)
        ok_gather = rank != 0 or all(bool((o == r).all()) for r, o in enumerate(outs))
        q.put((rank, pl.halo, ok_halo, ok_gather))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bench_c3_halo_p2p_and_island_gather(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_c3_comm_worker, args=(world, _free_port(), q), nprocs=world, join=True,
                       start_method="spawn")
    res = sorted([q.get() for _ in range(world)])
    assert any(r[1] > 0 for r in res)             # some rank's last chunk needed the halo
    assert all(r[2] for r in res) and all(r[3] for r in res)


_RANK_WORKER = r'''
import os, sys, torch, torch.distributed as dist
dist.init_process_group("gloo")
r, w = dist.get_rank(), dist.get_world_size()
assert int(os.environ["LOCAL_RANK"]) == r and os.environ["MASTER_ADDR"] == "127.0.0.1"
t = torch.tensor([r + 1], dtype=torch.int64)
dist.all_reduce(t)
if r == 0:
    print("SUM", int(t.item()), w, flush=True)
dist.destroy_process_group()
sys.exit(int(os.environ.get("FAIL_RANK", "-1")) == r)
'''


def test_bench_launcher_starts_n_ranks(tmp_path, capfd):
    """bench.py --gpus N without WORLD_SIZE starts N rank processes itself (the launcher the
    driver's `python bench.py --gpus N` relies on): RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*
    set, one collective over gloo, rank 0's line on stdout; a failing rank fails the launch."""
    import bench
    w = tmp_path / "worker.py"
    w.write_text(_RANK_WORKER)
    env_keep = {k: os.environ.pop(k) for k in ("RANK", "WORLD_SIZE", "FAIL_RANK") if k in os.environ}
    try:
        assert bench.launch_ranks(3, [sys.executable, str(w)]) == 0
        out = capfd.readouterr().out.splitlines()    # (gloo itself prints connection lines)
        assert [x for x in out if x.startswith("SUM")] == ["SUM 6 3"]
        os.environ["FAIL_RANK"] = "1"
        assert bench.launch_ranks(2, [sys.executable, str(w)]) != 0
    finally:
        os.environ.pop("FAIL_RANK", None)
        os.environ.update(env_keep)


def test_bench_rejects_world_size_mismatch():
    """Launched with WORLD_SIZE != --gpus, bench.py exits non-zero before touching a GPU."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0 and "WORLD_SIZE=2 but --gpus 4" in p.stderr
