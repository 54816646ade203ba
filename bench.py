#!/usr/bin/env python3
"""bench.py — CpG-island HMM hot path on MI355X: train + Viterbi bases/s.

Metric (BASELINE.json): bases/sec train+Viterbi at 1/2/4/8 MI355X; % HBM peak; CPU ref bases/s.
Workload (configs[1]): 46 Mbp chr21-sized synthetic sequence per GPU.  One step =
  train  : Baum-Welch E-step (expected counts, 65,536-base chunks, :130-141/:200)
           + labelled int64 counts (truth labels) + the reducer's cross-GPU merge
           (int64 all-reduce, fp64 all-gather + fixed-order sum over RCCL)
  decode : exact Viterbi of every whole 1,048,576-base chunk (:256-260)
           + island scan/filter (:262-339)
over bases already resident in HBM.  Weak scaling: rank r owns its own contiguous,
1 Mi-aligned 46 Mbp shard of the genome; value = bases of all ranks / step time (max over
ranks).  Launched as `python bench.py` (N=1) or via torch.distributed.run for N>1.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

# kernel arguments in device memory (must precede HIP initialisation)
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "bases/sec train+Viterbi at 1/2/4/8 MI355X; % HBM peak; CPU ref bases/s"
SEED = 20251015 + 1            # seed + config index
N_PER_GPU = 46_000_000         # configs[1]: 46 Mbp chr21-sized
SHARD_STRIDE = 44 << 20        # 1 Mi-aligned shard starts (44 decode chunks >= 46e6 bases)
TRAIN = 65536
DECODE = 1 << 20
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
# fp64 vector peak of the MI355X (AMD's published 78.6 TFLOP/s: 256 CUs x 2.4 GHz x 128 fp64
# flops per clock; the guides give no fp64 figure) and the E-step's ALGORITHMIC fp64 flops
# per base (FMA = 2): forward alpha 2 mul + 2 fma = 6, backward 4 mul + 4 fma + 2 add = 14,
# lane products 4 two-by-two products per 16 positions = 3 — implementation recomputation
# (the second forward pass over half of each mini-block) not counted
FP64_PEAK_TFLOPS = 78.6
# the training pass's kernel (the E-step chunk kernel; its kCnt instantiation in the fused pass);
# launches of >= 2,048 chunks run its lane-private-rows form (k_estep.hip, k_estep_chunk_rep)
ESTEP_KERNEL = "k_estep_chunk"
ESTEP_KERNEL_REP = "k_estep_chunk_rep"
EST_REP_MIN_CHUNKS = 2048


def estep_kernel(nbases):
    return ESTEP_KERNEL_REP if nbases // TRAIN >= EST_REP_MIN_CHUNKS else ESTEP_KERNEL
ESTEP_FLOPS_PER_BASE = 23
# algorithmic bytes per base of each phase: the fused
# decode (cpg_decode_d) reads the packed bases once and writes the 1-bit path (0.375); the
# separate island call re-reads bases + path (another 0.375)
BYTES_PER_BASE = {"estep": 0.25, "counts": 0.375, "viterbi": 0.375, "islands": 0.375,
                  "decode_fused": 0.375}
# VALU issue roof: one wave64 instruction per 2 cycles per SIMD (SIMD-32, MI355X_MICROARCH.md
# "Wave scheduling"), 1,024 SIMDs at 2.4 GHz; fp64 instructions occupy the SIMD twice as long,
# so for an fp64-heavy mix the true roof is lower — the fraction is an upper bound on issue use
VALU_PEAK_WINST = 1024 * 2.4e9 / 2
DECODE_KERNELS = ("k_vit_approx", "k_vit_scan", "k_vit_exact", "k_vit_chain", "k_vit_chain_seg",
                  "k_vit_forward", "k_vit_tscan", "k_vit_trace", "k_isl_tile", "k_isl_resolve")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _pmc(name):
    try:
        with open(os.path.join(ROOT, "profiles", name)) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def _pmc_traffic(kernel, nbases, name="pmc_latest.json", scale=False):
    """HBM bytes per launch of `kernel` from a committed PMC summary of this bench
    (tools/pmc.sh + tools/pmc_summary.py: FETCH_SIZE x2 + WRITE_SIZE, gfx950 correction of
    MI355X_MICROARCH.md): as collected when it was collected on the same workload size, or
    (scale=True: the N>1 shards) scaled linearly from the bytes per base of that profile."""
    d = _pmc(name)
    try:
        k = d["kernels"][kernel]
        b = d.get("bases")
        if b != nbases and not (scale and b):
            return None
        t = k["traffic_bytes"] if b == nbases else k["traffic_bytes"] / b * nbases
        return {"traffic_bytes": int(t),
                "source": f"profiles/{name} ({d.get('collected', '?')})" +
                          ("" if b == nbases else f", scaled from {b} bases")}
    except (TypeError, KeyError, ValueError):
        return None


def _decode_valu(nbases, phase_ms, name="pmc_latest.json"):
    """VALU issue roofline of the decode phase: wave-level VALU instructions per call of its
    kernels (PMC SQ_INSTS_VALU, committed profile of the same size) / the phase time, against
    VALU_PEAK_WINST."""
    d = _pmc(name)
    if not d or d.get("bases") != nbases or phase_ms <= 0:
        return None
    ks = {k: v for k, v in d["kernels"].items() if k in DECODE_KERNELS and "SQ_INSTS_VALU" in v}
    if not ks:
        return None
    winst = sum(v["SQ_INSTS_VALU"] for v in ks.values())
    ach = winst / (phase_ms / 1e3)
    return {"bound": "valu-issue", "phase": "decode", "kernels": sorted(ks),
            "valu_wave_instructions": int(winst), "achieved": round(ach / 1e9, 2),
            "peak": round(VALU_PEAK_WINST / 1e9, 1), "unit": "G wave-instructions/s",
            "frac": round(ach / VALU_PEAK_WINST, 4),
            "source": f"profiles/{name} ({d.get('collected', '?')})"}


def cpu_baseline(seed, sample_bases, threads):
    """The oracle (C restatement of the reference: Mahout-order 8-state Viterbi with
    Math.log in the inner loop, textbook E-step, labelled counts, island scan) on the GPU
    box's host cores over a bounded sample of the same workload: every decode chunk and every
    training chunk is an independent job (as the reference's per-chunk Viterbi calls and
    mapper tasks are), run by `threads` workers (ctypes releases the GIL).  The 1-thread
    time of the same sample is reported next to it."""
    from concurrent.futures import ThreadPoolExecutor

    from cpgisland_amd import device as D
    from oracle import coracle as co
    from oracle import pyref as pr
    packed, sign = D.synth_host(seed, 0, sample_bases)
    obs = pr.unpack(packed, sample_bases)
    truth = pr.unpack_bits(sign, sample_bases)
    m = co.initial_model()
    ndec = sample_bases // DECODE
    jobs = [("decode", c) for c in range(ndec)] + \
           [("train", c) for c in range(0, sample_bases // TRAIN, DECODE // TRAIN)]

    def run(job):
        kind, c = job
        if kind == "decode":
            co.decode_chunks(m, obs[c * DECODE:(c + 1) * DECODE], DECODE)
        else:   # 16 training chunks per job
            sl = slice(c * TRAIN, (c + DECODE // TRAIN) * TRAIN)
            co.estep(m, obs[sl], TRAIN)
            co.count_labelled(obs[sl], truth[sl], TRAIN)

    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(run, jobs))
    dt = time.perf_counter() - t0
    # the 1-thread rate on a quarter of the sample (bounded run time)
    q = jobs[: max(1, ndec // 4)] + [j for j in jobs if j[0] == "train"][: max(1, ndec // 4)]
    t1 = time.perf_counter()
    for j in q:
        run(j)
    dt1 = time.perf_counter() - t1
    return {"value": sample_bases / dt, "unit": "bases/s", "cores": threads, "kind": "port",
            "sample": f"{sample_bases} bases ({ndec} decode chunks, {sample_bases // TRAIN} "
                      f"train chunks) of the same synthetic genome; oracle/cpg_oracle.c, one "
                      f"job per decode chunk / 16 train chunks on {threads} threads, "
                      f"{dt:.1f} s",
            "seconds": dt, "value_1thread": len(q) / 2 * DECODE / dt1,
            "cpu": _cpu_model()}


def train_step(ctx, model0, dp, ds, N, ecnt, lcnt, fused):
    """The training pass: E-step (model0) + labelled counts of the same chunks — one launch
    (cpg_train_pass_d) or the two single calls (--separate-train)."""
    from cpgisland_amd import device as D
    if fused:
        D.train_pass(ctx, model0, dp, ds, N, TRAIN, estep_out=ecnt, counts_out=lcnt)
    else:
        D.bw_estep(ctx, model0, dp, N, TRAIN, out=ecnt)
        D.count_labelled(ctx, dp, ds, N, TRAIN, out=lcnt)


def decode_step(ctx, model1, dp, N, so, score, iout, icnt, fused, first_chunk=0):
    """The decode: Viterbi + island scan of the same chunks — one call (cpg_decode_d: the
    traceback writes the island scan's run records) or the two single calls
    (--separate-decode)."""
    from cpgisland_amd import device as D
    if fused:
        D.decode(ctx, model1, dp, N, DECODE, cap=iout.shape[0], first_chunk=first_chunk,
                 sign_out=so, score=score, out=iout, count=icnt)
    else:
        D.viterbi(ctx, model1, dp, N, DECODE, sign_out=so, score=score)
        D.islands(ctx, dp, so, N, DECODE, cap=iout.shape[0], first_chunk=first_chunk, out=iout,
                  count=icnt)


def cold_cache_steps(ln, dp, ds, N, model0, model1, nsteps, main_s, dev, first_chunk, flush_mb=1024,
                     fused=True, fused_decode=True):
    """The headline step's two streams (training pass on the lane's training stream, decode on
    its high-priority decode stream, concurrently), each step behind a `flush_mb` scratch write
    that evicts the shard from the 256 MB Infinity Cache (SURVEY 8(d)'s protocol).  Events: one
    on the main stream after the flush (both streams wait on it), one at the end of each
    stream's work; a step's time = the later end - that start, so the flush is excluded.  The
    same joined steps without the flush are timed beside it (`warm_joined_ms`): the cold/warm
    ratio is the Infinity Cache's share at equal step structure (the headline itself also
    overlaps consecutive steps, which a flush between steps rules out)."""
    buf = torch.empty(flush_mb << 18, dtype=torch.float32, device=dev)
    s_tr, s_dec = ln["s_tr"], ln["s_dec"]
    ctx = ln["ctx"]

    def joined(flush):
        marks = []
        for _ in range(nsteps):
            with torch.cuda.stream(main_s):
                if flush:
                    buf.fill_(1.0)
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record(main_s)
            s_dec.wait_event(e0)
            s_tr.wait_event(e0)
            with torch.cuda.stream(s_dec):
                decode_step(ctx, model1, dp, N, ln["so"], ln["score"], ln["iout"], ln["icnt"],
                            fused_decode, first_chunk)
                ed = torch.cuda.Event(enable_timing=True)
                ed.record(s_dec)
            with torch.cuda.stream(s_tr):
                train_step(ctx, model0, dp, ds, N, ln["ecnt"], ln["lcnt"], fused)
                et = torch.cuda.Event(enable_timing=True)
                et.record(s_tr)
            main_s.wait_event(ed)
            main_s.wait_event(et)
            marks.append((e0, ed, et))
        torch.cuda.synchronize()
        ctx.sync(None)
        return sum(max(a.elapsed_time(b), a.elapsed_time(c)) for a, b, c in marks) / len(marks)
    joined(False)   # (first use of this step shape: untimed)
    warm = joined(False)
    cold = joined(True)
    del buf
    return {"value": N / (cold / 1e3), "unit": "bases/s", "ms_per_step": round(cold, 4),
            "warm_joined_ms": round(warm, 4), "cold_over_warm": round(cold / warm, 4),
            "steps": nsteps, "flush_mb": flush_mb, "streams": 2, "step_overlap": False,
            "note": ("the headline's two concurrent streams per step, each step behind a 1 GiB "
                     "scratch write (excluded by events); warm_joined_ms: the same joined steps "
                     "without the flush")}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def warm_up(step_fn, args, dist, dev):
    """The untimed warm-up: args.warmup steps, then — until args.settle_ms of wall time have
    passed since the warm-up began — more untimed steps, in batches of 10.  A GPU that has been
    idle runs its first ~150 steps of sustained load at lower clocks: at the driver's
    `--warmup 5` the timed steps read 0.18 ms against 0.156 ms over 400 steps (DESIGN.md 5,
    profiles/r03_settle).  Every rank runs the same number of steps (the steps hold
    collectives): rank 0's clock decides, per batch.  step_fn(i) runs warm-up step i; returns
    the count run."""
    t0 = time.perf_counter()
    for w in range(args.warmup):
        step_fn(w)
    torch.cuda.synchronize()
    done = args.warmup
    while args.settle_ms > 0 and done < args.warmup + 10000:
        more = (time.perf_counter() - t0) * 1e3 < args.settle_ms
        if dist:
            t = torch.tensor([1 if more else 0], dtype=torch.int64, device=dev)
            torch.distributed.broadcast(t, 0)
            more = bool(t.item())
        if not more:
            break
        for w in range(done, done + 10):
            step_fn(w)
        done += 10
        torch.cuda.synchronize()
    return done


def launch_ranks(n, cmd=None):
    """`bench.py --gpus N` (N > 1) started without a launcher: start N rank processes of this
    same command line (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, one GPU each), before
    this process has touched the GPU, and return the worst exit status.  Rank 0's JSON line
    is the only stdout line (the children inherit stdout).  `cmd`: another command per rank
    (tests/test_dist.py)."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so_:
        so_.bind(("127.0.0.1", 0))
        port = so_.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen(cmd or ([sys.executable, os.path.abspath(__file__)] +
                                              sys.argv[1:]), env=env))
    rc = 0
    try:
        for p in procs:
            c = p.wait()
            rc = rc or c
            if c:   # one rank failed: the others would wait in a collective forever
                for q in procs:
                    if q.poll() is None:
                        q.kill()
    finally:
        for q in procs:
            if q.poll() is None:
                q.kill()
    return rc


def sha256_hex(*arrays):
    import hashlib
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).view(np.uint8).tobytes())
    return h.hexdigest()


def oracle_fixture(name, seed, start, nbases):
    """The oracle's whole-genome results for this workload (tests/golden/fingerprints.json,
    cpgisland_amd/fingerprint.py), or None when the workload is not the digested one."""
    from cpgisland_amd import fingerprint as F
    try:
        fx = F.load().get(name)
    except (OSError, ValueError):
        return None
    if not fx or (fx["seed"], fx["start"], fx["nbases"]) != (seed, start, nbases):
        return None
    return fx


def decode_model(fx, fallback):
    """The decode model: the fixture's committed one-iteration model (bit patterns: the GPU
    and the oracle decode with identical constants), else fallback() (a GPU E-step + the
    reducer, for workloads the fixture does not cover)."""
    from cpgisland_amd import HmmModel
    from cpgisland_amd import fingerprint as F
    if fx is not None:
        return HmmModel.from_struct(F.hex_to_f64(fx["decode"]["model_hex"]))
    return fallback()


def c2_fingerprint(fx, so, score, iout, icnt, ecnt, lcnt, ndec, nsplit):
    """Digest of one C2 step's results and, for the digested genome, the comparison with the
    oracle's results over every chunk (cpgisland_amd/fingerprint.py)."""
    from cpgisland_amd import device as D
    from cpgisland_amd import fingerprint as F
    if nsplit != 1:
        return {"oracle_match": None, "note": "--decode-split: records spread over parts"}
    dd = F.decode_digest(so.cpu().numpy(), score.cpu().numpy(), D.islands_to_numpy(iout, icnt),
                         ndec, DECODE, per_chunk=fx is not None)
    est, cnt = ecnt.cpu().numpy()[:105], lcnt.cpu().numpy()
    fp = {"path_sha256": dd["path_sha256"], "records_sha256": dd["records_sha256"],
          "counts_sha256": sha256_hex(cnt), "islands": dd["islands"], "oracle_match": None}
    if fx is not None:
        r = F.compare(fx, estep=est, counts=cnt, decode=dd)
        fp.update({k: r[k] for k in ("counts", "estep", "estep_max_rel_err", "path", "scores",
                                     "records", "oracle_match")})
        fp["oracle"] = ("tests/golden/fingerprints.json C2: oracle/cpg_oracle.c over all "
                        f"{fx['train']['chunks']} training and {fx['decode']['chunks']} decode "
                        "chunks; the decode model is its committed one-iteration model")
    return fp


def chunks_match(fx, sign_words, scores, c0, c1):
    """This rank's decode chunks [c0, c1) against the fixture's per-chunk path digests and
    scores: (path_ok, scores_ok)."""
    from cpgisland_amd import fingerprint as F
    fd = fx["decode"]
    dig = F.chunk_digests(sign_words, c1 - c0, DECODE)
    sc = F.f64_to_hex(np.asarray(scores, np.float64)[: c1 - c0])
    return dig == fd["chunk_path_digests"][c0:c1], sc == fd["scores_hex"][c0:c1]


def bw_iteration_leg(ctx, estep_fn, decode_fn, nbases, iters, dist, dev, backend="nccl"):
    """Real Baum-Welch iterations back to back (BaumWelchDriver.runBaumWelchMR's loop,
    :200-203): E-step on the current model (the mapper; its per-model tables built when the
    model is new) -> the reducer over ranks -> row normalisation on the host -> the next
    E-step, `iters` times from the reference's initial model, then one decode (Viterbi +
    islands) with the trained model (its per-model tables built there).  Wall time, priced
    with every per-model cost the fixed-model headline builds before its timed region."""
    from cpgisland_amd import HmmModel, baumwelch
    from cpgisland_amd import dist as cdist
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    m = HmmModel.initial()
    per, lls = [], []
    t0 = time.perf_counter()
    for _ in range(iters):
        ta = time.perf_counter()
        e = estep_fn(m)
        if dist and backend == "nccl":
            cdist.merge_counts_f64(e)
            c = e.cpu().numpy()
        elif dist:
            c = cdist.merge_counts_f64(e.cpu()).numpy()
        else:
            c = e.cpu().numpy()
        lls.append(float(c[-1]))
        m = baumwelch.normalize(c)
        per.append((time.perf_counter() - ta) * 1e3)
    tb = time.perf_counter()
    decode_fn(m)
    torch.cuda.synchronize()
    ctx.sync(None)
    t1 = time.perf_counter()
    dec_ms = (t1 - tb) * 1e3
    return {"iterations": iters, "ms_per_iteration": round(sum(per) / iters, 4),
            "iteration_ms": [round(x, 4) for x in per], "decode_ms": round(dec_ms, 4),
            "total_ms": round((t1 - t0) * 1e3, 4),
            "bases_per_s": nbases * (iters + 1) / (t1 - t0),
            "loglik": lls,
            "note": ("E-step -> merge -> host normalize -> next E-step (per-model tables built "
                     "for every new model), then one decode with the trained model; bases_per_s "
                     "counts each iteration and the decode as one pass over the bases")}


C3_BASES = 3_100_000_000       # configs[2]: 3.1 Gbp hg38-sized genome over the node's GPUs
C3_SEED = 20251015 + 2         # seed + config index


def _p2p(ops_spec, backend):
    """Point-to-point transfers [(kind, tensor, peer)] on the current stream (RCCL over xGMI),
    or staged through host memory for the gloo rehearsal."""
    D_ = torch.distributed
    if backend == "nccl":
        ops = [D_.P2POp(D_.isend if k == "send" else D_.irecv, t, peer) for k, t, peer in ops_spec]
        for w in D_.batch_isend_irecv(ops):
            w.wait()
        return
    host = []
    for k, t, peer in ops_spec:
        h = t.cpu() if k == "send" else torch.empty(t.shape, dtype=t.dtype)
        host.append((k, t, h, peer))
    ops = [D_.P2POp(D_.isend if k == "send" else D_.irecv, h, peer) for k, _, h, peer in host]
    for w in D_.batch_isend_irecv(ops):
        w.wait()
    for k, t, h, _ in host:
        if k == "recv":
            t.copy_(h)


def _gather0(t, world, rank, backend, out_list):
    """t from every rank to rank 0 (out_list on rank 0), on the current stream."""
    D_ = torch.distributed
    if backend == "nccl":
        D_.gather(t, out_list if rank == 0 else None, dst=0)
        return
    h = t.cpu()
    hl = [torch.empty_like(h) for _ in range(world)] if rank == 0 else None
    D_.gather(h, hl, dst=0)
    if rank == 0:
        for o, x in zip(out_list, hl):
            o.copy_(x)


def count_leg(ctx, dp, ds, n, reps=20):
    """The labelled-count kernel (cpg_count_labelled_d) alone over an
    HBM-resident genome (the C3 genome: 1.16 GB of packed bases + label bits, far past the
    256 MB Infinity Cache): HIP events around each call on the stream it runs on; the
    north_star's count-kernel roofline."""
    from cpgisland_amd import device as D
    out = torch.empty(124, dtype=torch.int64, device=dp.device)
    for _ in range(3):
        D.count_labelled(ctx, dp, ds, n, TRAIN, out=out)
    ev = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        D.count_labelled(ctx, dp, ds, n, TRAIN, out=out)
        b.record()
        ev.append((a, b))
    torch.cuda.synchronize()
    ctx.sync(None)
    ms = sorted(a.elapsed_time(b) for a, b in ev)[reps // 2]
    c = out.cpu().numpy()
    nch = n // TRAIN
    ok = bool(c[:8].sum() == nch and c[8:72].sum() == nch * (TRAIN - 1) and c[120:].sum() == n)
    bpb = BYTES_PER_BASE["counts"]
    ach = bpb * n / (ms / 1e3) / 1e9
    r = {"bound": "hbm", "kernel": "k_count_main", "bases": n, "achieved": round(ach, 1),
         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
         "traffic": None, "algorithmic_bytes": bpb * n, "bytes_per_base": bpb,
         "ms_median": round(ms, 4), "reps": reps, "identities_ok": ok,
         "note": "median of event-timed calls over the HBM-resident C3 genome"}
    pmc = _pmc_traffic("k_count_main", n, name="pmc_count.json")
    if pmc:
        r["traffic"] = pmc["traffic_bytes"]
        r["traffic_source"] = "stored PMC profile, not this run: " + pmc["source"]
    return r


def run_c3(args, world, rank, local, dist, backend, dev, emit=True):
    """configs[2] — the north_star workload: ONE 3.1 Gbp genome split evenly over the world's
    ranks at multiples of 64 bases (cpgisland_amd/dist.py shard_bounds(align=64), not at chunk
    boundaries).  A chunk belongs to the rank holding its first base; a rank's last chunk is
    completed by the halo — the next rank's first bases, received point to point over xGMI
    (rank r sends its head to r-1) — so every chunk runs whole, through the same kernels as
    the unsharded run (bit-identical counts, paths and islands: tests/test_dist.py,
    tests/test_gpu_halo.py).  One step = halo exchange + training pass (E-step + labelled
    counts) of the rank's training chunks + the reducer (all-gather of the rank records +
    rank-order merge) + exact Viterbi + islands of its decode chunks + the island records
    gathered to rank 0.  Strong scaling: value = genome bases per step / step time (max over
    ranks)."""
    from cpgisland_amd import Context, HmmModel, baumwelch
    from cpgisland_amd import device as D
    from cpgisland_amd import dist as cdist
    G = args.bases if args.bases != N_PER_GPU else C3_BASES
    spans = [cdist.shard_bounds(G, world, r, align=cdist.HALO_ALIGN) for r in range(world)]
    plans = [cdist.shard_plan(s, n, G) for s, n in spans]
    start, n = spans[rank]
    pl = plans[rank]
    for r in range(world - 1):   #  every halo comes from the next shard alone
        if plans[r].halo > spans[r + 1][1]:
            raise ValueError(f"rank {r}'s halo ({plans[r].halo}) exceeds rank {r + 1}'s shard")
    log(f"[rank {rank}] C3: genome {G} bases, shard [{start}, {start + n}), local "
        f"[{pl.base}, {pl.end}) halo {pl.halo}")
    packed, sign = D.synth_host(C3_SEED, start, n)
    span = pl.end - pl.base
    own = min(start + n, pl.end) - pl.base
    o16, o32 = (pl.base - start) // 16, (pl.base - start) // 32
    w16, w32 = D.words16(span) + 4, D.words32(span) + 4
    # the local genome twice (step k uses copy k & 1): the halo of step k+2 is received into
    # a copy that step k's kernels no longer read
    bufs = []
    for _ in range(2):
        bp = torch.zeros(w16, dtype=torch.int32, device=dev)
        bs = torch.zeros(w32, dtype=torch.int32, device=dev)
        if own > 0:
            bp[:D.words16(own)] = torch.from_numpy(packed[o16:o16 + D.words16(own)].view(np.int32)).to(dev)
            bs[:D.words32(own)] = torch.from_numpy(sign[o32:o32 + D.words32(own)].view(np.int32)).to(dev)
        bufs.append((bp, bs))
    # what this rank sends: its first plans[rank-1].halo bases (static data)
    ph = plans[rank - 1].halo if rank > 0 else 0
    head = (torch.from_numpy(packed[:D.words16(ph)].view(np.int32).copy()).to(dev),
            torch.from_numpy(sign[:D.words32(ph)].view(np.int32).copy()).to(dev)) if ph else None
    t16, t32 = (start + n - pl.base) // 16, (start + n - pl.base) // 32
    h16, h32 = D.words16(pl.halo), D.words32(pl.halo)
    del packed, sign
    tr_o, tr_n = pl.t0 * TRAIN - pl.base, (pl.t1 - pl.t0) * TRAIN
    de_o, de_n = pl.d0 * DECODE - pl.base, (pl.d1 - pl.d0) * DECODE
    ctx = Context(local)
    ctx.reserve(max(span, 1), chunk_len=DECODE)
    model0 = HmmModel.initial()
    icap = de_n // 32768 + 2048   # island records per rank per step (~3x the ~1 per 100 kbp)
    nd_total = G // DECODE
    rec = [cdist.train_record(dev) for _ in range(2)]
    gath = [torch.empty(world * cdist.TRAIN_RECORD, dtype=torch.float64, device=dev) for _ in range(2)]
    emerged = torch.empty(105, dtype=torch.float64, device=dev)
    lmerged = torch.empty(124, dtype=torch.int64, device=dev)
    so = torch.empty(D.words32(max(de_n, 1)) + 4, dtype=torch.int32, device=dev)
    score = torch.empty(max(pl.d1 - pl.d0, 1), dtype=torch.float64, device=dev)
    iout = [torch.empty((icap, 32), dtype=torch.uint8, device=dev) for _ in range(2)]
    icnt = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(2)]
    gat_i = [[torch.empty((icap, 32), dtype=torch.uint8, device=dev) for _ in range(world)]
             if rank == 0 else None for _ in range(2)]
    gat_c = [[torch.empty(1, dtype=torch.int64, device=dev) for _ in range(world)]
             if rank == 0 else None for _ in range(2)]
    main_s = torch.cuda.current_stream()
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    ntc = args.c3_train_cus if 0 < args.c3_train_cus < ncu else 0
    # the training pass on a CU-masked stream of ntc compute units (0: every CU), the decode
    # at high priority on all of them
    s_tr = D.cu_stream(local, list(range(ntc))) if ntc else torch.cuda.Stream()
    s_dec = torch.cuda.Stream(priority=-1 if args.prio else 0)
    # N = 1: no halo, no collective, no gather — the training stream runs the merge itself and no
    # other stream is made.  Streams beyond the hardware queues (GPU_MAX_HW_QUEUES, 4) share
    # queues, and a cross-stream wait queued behind one stream's kernels then holds the other's:
    # with five streams the C3 steps had joined at every step boundary (profiles/r05_c3q/)
    s_halo, s_red, s_isl = ((torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream())
                            if world > 1 else (None, s_tr, None))
    ev = {k: [torch.cuda.Event() for _ in range(2)] for k in
          ("halo", "tr_done", "dec_done", "rec", "red", "isl")}
    # several ranks on ONE GPU (the CPG_BENCH_BACKEND=gloo rehearsal on a one-GPU box): their
    # decodes run concurrently — the island records of a shard this size are placed by the
    # two-pass resolve (k_islands.hip: no workgroup waits for another)
    shared = bool(dist) and torch.cuda.device_count() < world
    ntr = []   # (start, end) timing events of the training pass, every 4th timed step

    def halo_into(b):
        if world == 1:
            return
        ops = []
        if head is not None:
            ops += [("send", head[0], rank - 1), ("send", head[1], rank - 1)]
        if pl.halo:
            ops += [("recv", bufs[b][0][t16:t16 + h16], rank + 1),
                    ("recv", bufs[b][1][t32:t32 + h32], rank + 1)]
        if ops:
            _p2p(ops, backend)
    if dist:
        torch.distributed.barrier()   # (a full collective first: not every rank has a P2P op)
    for b in range(2):
        halo_into(b)
    torch.cuda.synchronize()
    # the decode model: one Baum-Welch iteration over the whole genome from the reference's
    # model — the oracle's, committed with its whole-genome results (every rank the same);
    # for other genome sizes the GPU E-step of every rank merged in rank order, before timing
    fx = oracle_fixture("C3", C3_SEED, 0, G)

    def gpu_model1():
        e0 = D.bw_estep(ctx, model0, bufs[0][0][tr_o // 16:], tr_n, TRAIN)
        if dist and backend == "nccl":
            cdist.merge_counts_f64(e0)
        elif dist:
            e0.copy_(cdist.merge_counts_f64(e0.cpu()).to(dev))
        return baumwelch.normalize(e0.cpu().numpy())
    model1 = decode_model(fx, gpu_model1)

    def step1(k, timed):   # N = 1: two streams, no cross-stream event
        b = k & 1
        bp, bs = bufs[b]
        with torch.cuda.stream(s_dec):
            D.decode(ctx, model1, bp[de_o // 16:], de_n, DECODE, cap=icap, first_chunk=pl.d0,
                     sign_out=so, score=score, out=iout[b], count=icnt[b])
        with torch.cuda.stream(s_tr):
            mark = timed and k % 4 == 0
            if mark:
                ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ea.record(s_tr)
            D.train_pass(ctx, model0, bp[tr_o // 16:], bs[tr_o // 32:], tr_n, TRAIN,
                         estep_out=rec[b][1], counts_out=rec[b][2])
            if mark:
                eb.record(s_tr)
                ntr.append((ea, eb))
            cdist.merge_train_records(ctx, rec[b][0], emerged, lmerged, gathered=gath[b])

    def step(k, timed):
        if world == 1:
            return step1(k, timed)
        b = k & 1
        bp, bs = bufs[b]
        with torch.cuda.stream(s_halo):
            if k >= 2:   # step k-2's kernels have finished reading this copy
                s_halo.wait_event(ev["tr_done"][b])
                s_halo.wait_event(ev["dec_done"][b])
            halo_into(b)
            ev["halo"][b].record(s_halo)
        with torch.cuda.stream(s_dec):
            s_dec.wait_event(ev["halo"][b])
            if k >= 2:
                s_dec.wait_event(ev["isl"][b])   # step k-2's island gather has read the records
            D.decode(ctx, model1, bp[de_o // 16:], de_n, DECODE, cap=icap, first_chunk=pl.d0,
                     sign_out=so, score=score, out=iout[b], count=icnt[b])
            ev["dec_done"][b].record(s_dec)
        with torch.cuda.stream(s_tr):
            s_tr.wait_event(ev["halo"][b])
            if k >= 2:
                s_tr.wait_event(ev["red"][b])    # step k-2's all-gather has read the record
            mark = timed and k % 4 == 0
            if mark:
                ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ea.record(s_tr)
            D.train_pass(ctx, model0, bp[tr_o // 16:], bs[tr_o // 32:], tr_n, TRAIN,
                         estep_out=rec[b][1], counts_out=rec[b][2])
            if mark:
                eb.record(s_tr)
                ntr.append((ea, eb))
            ev["tr_done"][b].record(s_tr)
        with torch.cuda.stream(s_red):
            s_red.wait_event(ev["tr_done"][b])
            cdist.merge_train_records(ctx, rec[b][0], emerged, lmerged, gathered=gath[b])
            ev["red"][b].record(s_red)
        with torch.cuda.stream(s_isl):
            s_isl.wait_event(ev["dec_done"][b])
            if world > 1:
                _gather0(icnt[b], world, rank, backend, gat_c[b])
                _gather0(iout[b], world, rank, backend, gat_i[b])
            ev["isl"][b].record(s_isl)

    nwarm = warm_up(lambda w: step(w, False), args, dist, dev)
    ctx.sync(None)
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for it in range(args.steps):
        step(nwarm + it, True)
    issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ctx.sync(None)      # raises if a kernel self-check (exactness) or look-back failed
    tr_ms = sum(a.elapsed_time(b) for a, b in ntr) / max(1, len(ntr))
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    last = (nwarm + args.steps - 1) & 1
    counts = [int(c.item()) for c in gat_c[last]] if (rank == 0 and world > 1) else \
        [int(icnt[last].item())]
    if max(counts) > icap:
        raise RuntimeError(f"island records per rank {max(counts)} exceed the gather capacity {icap}")
    # fingerprints of the last step's results, comparable across N (bit-exact by
    # construction): the island records gathered on rank 0 in chunk order (rank order = chunk
    # order, each rank's in chunk order) and the merged labelled int64 counts
    fp = None
    # against the oracle (every chunk: tests/golden/fingerprints.json): each rank checks its own
    # decode chunks' paths and scores, one MIN all-reduce; rank 0 the gathered records and the
    # merged counts / E-step
    chk = None
    if fx is not None:
        pth, scs = chunks_match(fx, so.cpu().numpy().view(np.uint32), score.cpu().numpy(),
                                pl.d0, pl.d1)
        chk = torch.tensor([int(pth), int(scs)], dtype=torch.int64, device=dev)
        if dist:
            if backend == "nccl":
                torch.distributed.all_reduce(chk, op=torch.distributed.ReduceOp.MIN)
            else:
                h = chk.cpu()
                torch.distributed.all_reduce(h, op=torch.distributed.ReduceOp.MIN)
                chk = h
        chk = [bool(x) for x in chk.tolist()]
    if rank == 0:
        if world > 1:
            recs = np.concatenate([gat_i[last][r][:counts[r]].cpu().numpy().reshape(-1)
                                   for r in range(world)])
        else:
            recs = iout[last][:counts[0]].cpu().numpy().reshape(-1)
        lm = lmerged.cpu().numpy()
        fp = {"records_sha256": sha256_hex(recs), "counts_sha256": sha256_hex(lm),
              "islands": int(sum(counts)), "oracle_match": None}
        if fx is not None:
            from cpgisland_amd import fingerprint as F
            ok, rel = F.estep_close(emerged.cpu().numpy()[:105], fx["train"]["estep_hex"],
                                    fx["train"]["estep_bound_hex"])
            parts = {"counts": bool(np.array_equal(lm, np.asarray(fx["train"]["counts"], np.int64))),
                     "estep": ok,
                     "path": chk[0], "scores": chk[1],
                     "records": (sha256_hex(recs) == fx["decode"]["records_sha256"] and
                                 int(sum(counts)) == fx["decode"]["islands"])}
            fp.update(parts)
            fp["estep_max_rel_err"] = rel
            fp["oracle_match"] = all(parts.values())
            fp["oracle"] = ("tests/golden/fingerprints.json C3: oracle/cpg_oracle.c over all "
                            f"{fx['train']['chunks']} training and {fx['decode']['chunks']} "
                            "decode chunks; the decode model is its committed one-iteration "
                            "model")
    bw = None
    if args.bw_iters > 0:
        def dec_fn(m):
            D.decode(ctx, m, bufs[0][0][de_o // 16:], de_n, DECODE, cap=icap, first_chunk=pl.d0,
                     sign_out=so, score=score, out=iout[0], count=icnt[0])
        bw = bw_iteration_leg(ctx, lambda m: D.bw_estep(ctx, m, bufs[0][0][tr_o // 16:], tr_n, TRAIN),
                              dec_fn, G, args.bw_iters, dist, dev, backend)
    if rank == 0:
        ms = elapsed * 1e3 / args.steps
        value = G * args.steps / elapsed
        bpb = BYTES_PER_BASE["estep"] + 0.125
        ach = bpb * tr_n / (tr_ms / 1e3) / 1e9 if tr_ms > 0 else 0.0
        out = {"metric": METRIC, "value": value, "unit": "bases/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "warmup_steps_run": nwarm,
               "settle_ms": args.settle_ms, "ms_per_step": ms,
               "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
               "dtype": "f64", "data": f"synthetic (counter-based planted-island genome, seed {C3_SEED})",
               "config": {"workload": f"C3: {G / 1e9:.1f} Gbp hg38-sized genome split over "
                                      f"{world} GPU(s) at 64-base boundaries; halo P2P + BW "
                                      "E-step + labelled counts + RCCL reduce + exact Viterbi + "
                                      "islands + island gather to rank 0",
                          "genome_bases": G, "bases_per_gpu": n, "parallelism": f"dp{world}",
                          "train_chunk": TRAIN, "decode_chunk": DECODE,
                          "decode_chunks": nd_total, "island_capacity_per_rank": icap,
                          "collectives": (("rccl" if backend == "nccl" else backend)
                                          if dist else None),
                          "train_cus": ntc or ncu,
                          "decode_priority": "high" if args.prio else "normal",
                          "ranks_share_gpu": shared,
                          "islands_found": sum(counts)},
               "phases_ms": {"train_pass": round(tr_ms, 4)},
               "host_issue_ms_per_step": round(issue * 1e3 / args.steps, 4),
               "roofline": {"bound": "hbm", "kernel": estep_kernel(tr_n), "phase": "train_pass",
                            "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                            "algorithmic_bytes": bpb * tr_n, "bytes_per_base": bpb},
               "cpu_baseline": None,
               "cpu_baseline_note": ("the CPU baseline is measured on rank 0 at N = 1 only (the "
                                     "bench contract): the n_gpus = 1 line's cpu_baseline, the "
                                     "oracle on a bounded sample of the same synthetic genome"),
               "fingerprint": fp, "bw_iteration": bw}
        # HBM traffic of the training pass at this rank's size: the PMC profile of the C3
        # workload on one GPU (tools/pmc.sh c3), scaled to the shard's bases
        pmc = _pmc_traffic(estep_kernel(tr_n), tr_n, name="pmc_c3.json", scale=True)
        if pmc:
            out["roofline"]["traffic"] = pmc["traffic_bytes"]
            out["roofline"]["traffic_source"] = "stored PMC profile, not this run: " + pmc["source"]
        if world == 1:   # the count kernel alone over the same HBM-resident genome
            out["roofline_count"] = count_leg(ctx, bufs[0][0][tr_o // 16:], bufs[0][1][tr_o // 32:],
                                              tr_n)
        if emit:
            print(json.dumps(out), flush=True)
    else:
        out = None
    if ntc:
        D.cu_stream_destroy(s_tr)
    ctx.close()
    if dist:
        torch.distributed.destroy_process_group()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--settle-ms", type=float, default=100.0,
                    help="untimed warm-up lasts at least this long: after the --warmup steps, "
                         "more untimed steps until about this much wall time has passed (an "
                         "idle GPU's clocks rise over its first ~25 ms of load; the count run is "
                         "reported as warmup_steps_run; 0 = exactly --warmup steps)")
    ap.add_argument("--bases", type=int, default=N_PER_GPU,
                    help="bases per GPU (C2), or the whole genome with --workload c3 "
                         "(default there: 3.1e9)")
    ap.add_argument("--workload", choices=("auto", "c2", "c3"), default="auto",
                    help="c2: 46 Mbp per GPU (configs[1], weak scaling); c3: one 3.1 Gbp genome "
                         "split over the GPUs (configs[2], the north_star workload, strong "
                         "scaling); auto: c2 on one GPU, c3 on several")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--c3-train-cus", type=int, default=0,
                    help="C3 workload: the training pass on a CU-masked stream of this many compute "
                         "units (0 = all; the decode stream runs on all of them at high priority)")
    ap.add_argument("--c3-steps", type=int, default=20,
                    help="N=1: timed steps of the C3 leg (the 3.1 Gbp strong-scaling workload of "
                         "the N>1 lines on this one GPU, reported as c3_single_gpu, with the "
                         "count kernel's HBM roofline over its genome); 0 = skip")
    ap.add_argument("--probe-sleep", type=str, default="",
                    help="measurement probe: STREAM:CYCLES adds a one-thread spin kernel "
                         "(torch.cuda._sleep) per step on the decode ('dec') or training ('tr') "
                         "stream, to price a stream's latency")
    ap.add_argument("--separate-decode", action="store_true",
                    help="Viterbi and island scan as two calls instead of the fused decode "
                         "(cpg_decode_d)")
    ap.add_argument("--separate-train", action="store_true",
                    help="E-step and labelled counts as two launches instead of the fused "
                         "training pass (cpg_train_pass_d)")
    ap.add_argument("--bw-iters", type=int, default=5,
                    help="after the timed steps: this many real Baum-Welch iterations back to back "
                         "(new model every iteration) + one decode, reported as bw_iteration (0 = "
                         "skip)")
    ap.add_argument("--cpu-sample", type=int, default=192 * DECODE)
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="host threads for the CPU baseline (the GPU box's CPU share is 16)")
    ap.add_argument("--prio", type=int, default=1,
                    help="1: decode stream at high priority (two-stream mode)")
    ap.add_argument("--serial", action="store_true",
                    help="train and decode phases on one stream (isolated phase timing)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="join both streams after every step (by default step k+1's training "
                         "pass may start while step k's decode still runs: the steps are "
                         "independent batches, pipelined for throughput)")
    ap.add_argument("--lanes", type=int, default=2,
                    help="pipeline lanes: step k runs on lane k %% lanes, each lane with its own "
                         "context (workspace), stream pair and outputs, so consecutive steps' "
                         "kernels of the same kind may run concurrently (default 2: since the "
                         "decode has no cross-workgroup waits, two steps' decodes and training "
                         "passes overlap; 1, 3, 4 measured slower, DESIGN.md 5)")
    ap.add_argument("--decode-lanes", type=int, default=1,
                    help="decodes of consecutive steps alternate over this many contexts, "
                         "streams and output buffers, so that two steps' per-chunk kernels may "
                         "run concurrently")
    ap.add_argument("--train-lanes", type=int, default=1,
                    help="training passes of consecutive steps alternate over this many "
                         "contexts (workspaces) and CU-masked streams, so that step k+1's pass "
                         "may start on the CUs step k's last round of workgroups leaves idle")
    ap.add_argument("--train-cus", type=int, default=-1,
                    help="run the training pass on this many compute units only (a CU-masked "
                         "stream, the first bits of the mask), leaving the rest to the decode; "
                         "0 = all, -1 = 14/16 of them (default; round 6, two pipeline lanes, "
                         "200 steps: 160: 366, 192: 397-401, 208: 402-404, 216: 413, "
                         "224: 419-427, 232: 422-423, 240: 418-419, 248: 415-416, all 256: "
                         "393-395 Gbase/s; one lane (rounds 3-5) peaked at 192 = 12/16)")
    ap.add_argument("--decode-cus-from", type=int, default=0,
                    help="> 0: the decode stream CU-masked to compute units [this, all) (a masked "
                         "stream has no priority: the decode then runs at normal priority)")
    ap.add_argument("--train-cu-stride", type=int, default=0,
                    help="with --train-cus: leave out every k-th CU instead of the last ones")
    ap.add_argument("--phase-events", action="store_true",
                    help="record HIP events around every phase (default: E-step and decode)")
    ap.add_argument("--decode-event-every", type=int, default=16,
                    help="record the decode phase's events on every k-th timed step")
    ap.add_argument("--estep-event-every", type=int, default=16,
                    help="record the E-step phase's events on every k-th timed step (an event "
                         "record is a release at its point in the stream: every 4th step cost "
                         "1.5 %% of the rate against none, every 16th 0.9 %%; 25 samples per "
                         "400 steps)")
    ap.add_argument("--no-phase-events", action="store_true",
                    help="(diagnostic) record no per-phase HIP events inside the timed steps")
    ap.add_argument("--decode-split", type=int, default=1,
                    help="decode each step's chunks as this many independent parts, each on "
                         "its own context and stream (the per-chunk kernels of the parts "
                         "overlap)")
    ap.add_argument("--flush-mb", type=int, default=0,
                    help="write this many MiB of scratch between steps (cold Infinity Cache)")
    ap.add_argument("--cold-steps", type=int, default=10,
                    help="N=1: after the timed region, this many extra two-stream steps each "
                         "behind a 1 GiB scratch write (cold Infinity Cache), reported as "
                         "cold_cache beside the headline with the same joined steps warm "
                         "(0 = skip)")
    args = ap.parse_args()
    if args.flush_mb:
        args.serial = True   # the flushed step time is the sum of isolated phase times
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))     # one process per GPU, started here
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={os.environ.get('WORLD_SIZE')} but --gpus {args.gpus}")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    # CPG_BENCH_BACKEND=gloo rehearses the N-rank path on fewer GPUs (ranks share devices,
    # the reducer's collectives staged through host memory); the measured runs use RCCL
    backend = os.environ.get("CPG_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    if dist:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.distributed.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    workload = args.workload if args.workload != "auto" else ("c3" if dist else "c2")
    if workload == "c3":
        return run_c3(args, world, rank, local, dist, backend, dev)

    from cpgisland_amd import Context, HmmModel
    from cpgisland_amd import device as D
    from cpgisland_amd import dist as cdist

    N = args.bases
    start = rank * SHARD_STRIDE if N <= SHARD_STRIDE else rank * ((N + DECODE - 1) // DECODE * DECODE)
    log(f"[rank {rank}] synthesising {N} bases at offset {start}")
    packed, sign = D.synth_host(SEED, start, N)
    dp = D.to_device(packed, dev)
    ds = D.to_device(sign, dev)
    ctx = Context(local)
    ctx.reserve(N, chunk_len=DECODE)
    model0 = HmmModel.initial()
    ndec = N // DECODE
    first_chunk = start // DECODE
    flush = torch.empty(args.flush_mb << 18, dtype=torch.float32, device=dev) if args.flush_mb else None
    nlanes = 1 if (args.serial or args.no_overlap) else max(1, args.lanes)
    icap = 1 << 20

    ntl = 1 if (args.serial or args.no_overlap) else max(1, args.train_lanes)
    nrec = ntl if ntl >= 2 else 2

    def make_lane(cx):
        # the training pass writes one rank record per step (E-step doubles | labelled-count
        # int64: cpgisland_amd/dist.py train_record), one per training lane and at least two,
        # so that step k+1's training pass does not wait for step k's all-gather and two
        # training streams never write the same record
        recs = [cdist.train_record(dev) for _ in range(nrec)]
        return {"ctx": cx, "recs": recs,
                "gath": [torch.empty(world * cdist.TRAIN_RECORD, dtype=torch.float64, device=dev)
                         for _ in range(nrec)],
                "ev_tr": [torch.cuda.Event() for _ in range(nrec)],
                "ev_red": [torch.cuda.Event() for _ in range(nrec)],
                "emerged": torch.empty(105, dtype=torch.float64, device=dev),
                "lmerged": torch.empty(124, dtype=torch.int64, device=dev),
                "so": torch.empty(D.words32(N) + 4, dtype=torch.int32, device=dev),
                "score": torch.empty(max(ndec, 1), dtype=torch.float64, device=dev),
                "ecnt": torch.empty(105, dtype=torch.float64, device=dev),
                "lcnt": torch.empty(124, dtype=torch.int64, device=dev),
                "iout": torch.empty((icap, 32), dtype=torch.uint8, device=dev),
                "icnt": torch.zeros(1, dtype=torch.int64, device=dev)}
    lanes = [make_lane(ctx)]
    for _ in range(1, nlanes):
        cx = Context(local)
        cx.reserve(N)
        lanes.append(make_lane(cx))

    # the decode model: one Baum-Welch iteration from the reference's model — the oracle's,
    # committed with its whole-genome results (tests/golden/fingerprints.json C2), for every
    # rank; for other workload sizes a GPU E-step over the shard + the reducer
    fx = oracle_fixture("C2", SEED, start, N)

    def gpu_model1():
        from cpgisland_amd import baumwelch
        ecnt = lanes[0]["ecnt"]
        D.bw_estep(ctx, model0, dp, N, TRAIN, out=ecnt)
        if dist:
            cdist.merge_counts_f64(ecnt)
        return baumwelch.normalize(ecnt.cpu().numpy())
    model1 = decode_model(oracle_fixture("C2", SEED, 0, N), gpu_model1)

    # HIP events inside the timed steps: the E-step phase (the roofline's dominant kernel) and
    # the decode phase (on every --decode-event-every-th step) by default; every phase with
    # --phase-events or --serial.  An event record is not free (a release at the stream's
    # point of record): 10 per step cost ~9 % of the overlapped throughput, 4 per step ~3 %,
    # both phases' on every 4th step 1.5 %, on every 16th 0.9 % (the default: 25 samples of
    # each phase per 400 steps; profiles/r02_v10/ab_phase_events.log).
    full_ev = args.phase_events or args.serial
    probe = None
    if args.probe_sleep:
        ps_, pc_ = args.probe_sleep.split(":")
        probe = (ps_, int(pc_))
    fused = not args.separate_train
    fused_decode = not args.separate_decode
    names = (("estep", "counts", "reduce") +
             (("decode",) if fused_decode else ("viterbi", "islands"))) if full_ev \
        else ("estep", "decode")
    # one pair of HIP events per phase per timed step, read after the final synchronize (no
    # host round trip between steps)
    evs = [{k: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            for k in names} for _ in range(args.steps)]
    acc = {k: 0.0 for k in names}
    recorded = set()

    # The training pass and the decode are independent within a step: by default they run
    # concurrently on two streams (the decode kernels are latency-bound and leave SIMDs idle
    # that the E-step fills), and consecutive steps (independent batches) are pipelined: no
    # join between steps (--no-overlap adds one).  --serial runs everything on one stream
    # (isolated phase times).
    main_s = torch.cuda.current_stream()
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    if args.train_cus < 0:
        args.train_cus = ncu * 14 // 16
    if args.train_cus and args.train_cus < ncu and not args.serial:
        if args.train_cu_stride:
            tr_cus = [i for i in range(ncu) if i % args.train_cu_stride != 0][:args.train_cus]
        else:
            tr_cus = list(range(args.train_cus))
    else:
        tr_cus = None
    nsplit = 1 if (args.serial or ndec < 2) else max(1, min(args.decode_split, ndec))
    bounds = [ndec * i // nsplit for i in range(nsplit + 1)]   # decode-chunk ranges
    for ln in lanes:
        ln["parts"] = []
        for pi in range(1, nsplit):
            cx2 = Context(local)
            cx2.reserve(N)
            ln["parts"].append({"ctx": cx2, "s": torch.cuda.Stream(priority=-1 if args.prio else 0),
                                "iout": torch.empty((icap, 32), dtype=torch.uint8, device=dev),
                                "icnt": torch.zeros(1, dtype=torch.int64, device=dev)})
    ndl = 1 if (args.serial or args.no_overlap) else max(1, args.decode_lanes)

    def train_stream():
        return (main_s if args.serial else
                D.cu_stream(local, tr_cus) if tr_cus else torch.cuda.Stream())
    for ln in lanes:
        ln["s_tr"] = train_stream()
        ln["tr"] = [(ln["ctx"], ln["s_tr"])]
        for _ in range(1, ntl):
            cx3 = Context(local)
            cx3.reserve(N)
            ln["tr"].append((cx3, train_stream()))
        # the decode stream at high priority: its latency-bound kernels get CUs first as the
        # E-step's workgroups retire, the E-step fills the rest
        ln["s_dec"] = (main_s if args.serial else
                       D.cu_stream(local, list(range(args.decode_cus_from, ncu)))
                       if args.decode_cus_from > 0 else
                       torch.cuda.Stream(priority=-1 if args.prio else 0))
        ln["dec"] = [(ln["ctx"], ln["s_dec"], ln["so"], ln["score"], ln["iout"], ln["icnt"])]
        for _ in range(1, ndl):
            cx4 = Context(local)
            cx4.reserve(N)
            ln["dec"].append((cx4, torch.cuda.Stream(priority=-1 if args.prio else 0),
                              torch.empty_like(ln["so"]), torch.empty_like(ln["score"]),
                              torch.empty_like(ln["iout"]), torch.zeros_like(ln["icnt"])))
        # the reducer's collective on a stream of its own: the next step's training pass does
        # not wait for it
        # (N = 1: no reducer, no stream: a HIP stream's hardware queue is created on its first
        # use, and that took ~5 ms of host time plus a disturbance of the running queues when
        # the first use was the final join of the timed region — profiles/r03_v1)
        ln["s_red"] = main_s if (args.serial or not dist) else torch.cuda.Stream()

    def step(it, k):
        ln = lanes[k % nlanes]
        cx, s_tr = ln["ctx"], ln["s_tr"]
        dcx, s_dec, d_so, d_score, d_iout, d_icnt = ln["dec"][k % ndl]

        def mark(name, i):
            if it is None or args.no_phase_events:
                return
            if full_ev:
                key = name
            elif name == "estep":
                if it % args.estep_event_every:
                    return
                key = name
            elif (name, i) in (("viterbi", 0), ("islands", 1)) and it % args.decode_event_every == 0:
                key, i = "decode", (0 if name == "viterbi" else 1)
            elif name == "decode" and it % args.decode_event_every == 0:
                key = "decode"
            else:
                return
            evs[it][key][i].record()
            if i == 1:
                recorded.add((it, key))
        if args.no_overlap or args.serial:
            s_tr.wait_stream(main_s)
            s_dec.wait_stream(main_s)
        # part 0 on the lane's decode stream (chunks [0, bounds[1]); with --decode-split the
        # other parts on their own streams: independent chunks, so independent calls
        for pi in range(nsplit - 1, -1, -1):
            c0, c1 = bounds[pi], bounds[pi + 1]
            nb = (c1 - c0) * DECODE if pi < nsplit - 1 else N - c0 * DECODE
            part = ln["parts"][pi - 1] if pi > 0 else None
            with torch.cuda.stream(part["s"] if part else s_dec):
                px = part["ctx"] if part else dcx
                pp, sg = dp[c0 * DECODE // 16:], d_so[c0 * DECODE // 32:]
                io = part["iout"] if part else d_iout
                ic = part["icnt"] if part else d_icnt
                if fused_decode:
                    if pi == 0:
                        mark("decode", 0)
                    D.decode(px, model1, pp, nb, DECODE, cap=icap, first_chunk=first_chunk + c0,
                             sign_out=sg, score=d_score[c0:], out=io, count=ic)
                    if pi == 0:
                        mark("decode", 1)
                else:
                    if pi == 0:
                        mark("viterbi", 0)
                    D.viterbi(px, model1, pp, nb, DECODE, sign_out=sg, score=d_score[c0:])
                    if pi == 0:
                        mark("viterbi", 1)
                        mark("islands", 0)
                    D.islands(px, pp, sg, nb, DECODE, cap=icap, first_chunk=first_chunk + c0,
                              out=io, count=ic)
                    if pi == 0:
                        mark("islands", 1)
                    if probe and probe[0] == "dec":
                        torch.cuda._sleep(probe[1])
        par = k % nrec   # (training lane k % ntl writes record k % nrec: ntl divides nrec)
        rec, ecnt, lcnt = ln["recs"][par]
        cx, s_tr = ln["tr"][k % ntl]   # (the decode above ran on the lane's own context)
        with torch.cuda.stream(s_tr):
            if dist and k >= nrec:   # this record's previous all-gather has read it
                s_tr.wait_event(ln["ev_red"][par])
            if fused:   # "estep" = the whole training pass (E-step + labelled counts)
                mark("estep", 0)
                D.train_pass(cx, model0, dp, ds, N, TRAIN, estep_out=ecnt, counts_out=lcnt)
                mark("estep", 1)
            else:
                mark("estep", 0)
                D.bw_estep(cx, model0, dp, N, TRAIN, out=ecnt)
                mark("estep", 1)
                mark("counts", 0)
                D.count_labelled(cx, dp, ds, N, TRAIN, out=lcnt)
                mark("counts", 1)
            if probe and probe[0] == "tr":
                torch.cuda._sleep(probe[1])
            if dist:
                ln["ev_tr"][par].record(s_tr)
        if dist:   # the reducer over ranks: one all-gather of the records + one merge launch
            with torch.cuda.stream(ln["s_red"]):
                ln["s_red"].wait_event(ln["ev_tr"][par])
                mark("reduce", 0)
                cdist.merge_train_records(cx, rec, ln["emerged"], ln["lmerged"],
                                          gathered=ln["gath"][par])
                mark("reduce", 1)
                ln["ev_red"][par].record(ln["s_red"])
        if args.no_overlap or args.serial:
            main_s.wait_stream(s_tr)
            main_s.wait_stream(s_dec)
            main_s.wait_stream(ln["s_red"])

    def warm_step(w):
        step(None, w)
        if flush is not None:
            flush.fill_(1.0)
    nwarm = warm_up(warm_step, args, dist, dev)
    for ln in lanes:
        ln["ctx"].sync(None)
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    # CPG_BENCH_TIMELINE=1: host timeline of the timed region's end and the GPU span of the
    # timed steps (events on the training and decode streams before step 0 / after the last)
    gpu_span = ([], []) if os.environ.get("CPG_BENCH_TIMELINE") else None
    t0 = time.perf_counter()
    if gpu_span is not None:
        for ln in lanes:
            for _, st in ln["tr"] + [(None, ln["s_dec"])]:
                gpu_span[0].append(torch.cuda.Event(enable_timing=True))
                gpu_span[0][-1].record(st)
    for it in range(args.steps):
        if flush is not None:
            flush.fill_(1.0)
        step(it, nwarm + it)
    issue = time.perf_counter() - t0   # host time to enqueue every step (launch-bound check)
    tl = [("issued", issue)]
    # the end of the timed region: one device-wide synchronize waits for every stream of
    # every lane (no per-stream joins: a join records an event on each stream, and a stream
    # never used before — the N = 1 reducer stream — created its hardware queue right there)
    if gpu_span is not None:
        for ln in lanes:
            for _, st in ln["tr"]:
                gpu_span[1].append(torch.cuda.Event(enable_timing=True))
                gpu_span[1][-1].record(st)
            gpu_span[1].append(torch.cuda.Event(enable_timing=True))
            gpu_span[1][-1].record(ln["s_dec"])
    tl.append(("joined", time.perf_counter() - t0))
    torch.cuda.synchronize()
    tl.append(("sync1", time.perf_counter() - t0))
    nrec = {k: 0 for k in names}
    for it, ev in enumerate(evs):
        for k, (a, b) in ev.items():
            if (it, k) in recorded:
                acc[k] += a.elapsed_time(b)
                nrec[k] += 1
    tl.append(("events", time.perf_counter() - t0))
    if dist:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    tl.append(("sync2", elapsed))
    if gpu_span is not None:
        a0 = gpu_span[0][0]
        span = max(a0.elapsed_time(e) for e in gpu_span[1]) - \
            min(a0.elapsed_time(e) for e in gpu_span[0])
        log("timeline ms: " + " ".join(f"{k}={v * 1e3:.3f}" for k, v in tl) +
            f" gpu_span={span:.3f}")
        for k in names:   # per-step phase durations in order (the warm-up of the clocks)
            ser = [round(ev[k][0].elapsed_time(ev[k][1]), 4) for it, ev in enumerate(evs)
                   if (it, k) in recorded]
            log(f"phase {k}: {ser}")
    for ln in lanes:
        ln["ctx"].sync(None)     # raises if any kernel self-check (exactness) failed
        for cx3, _ in ln["tr"][1:]:
            cx3.sync(None)
        for dl in ln["dec"][1:]:
            dl[0].sync(None)
    # the last timed step's results (its lane's buffers) against the oracle's over the whole
    # shard (rank 0's shard is the digested C2 genome); before the BW leg reuses the buffers
    fingerprint = None
    if rank == 0:
        kl = nwarm + args.steps - 1
        ln = lanes[kl % nlanes]
        _, _, d_so, d_score, d_iout, d_icnt = ln["dec"][kl % ndl]
        _, ecnt_l, lcnt_l = ln["recs"][kl % len(ln["recs"])]
        fingerprint = c2_fingerprint(fx, d_so, d_score, d_iout, d_icnt, ecnt_l, lcnt_l, ndec,
                                     nsplit)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    islands_found = int(lanes[0]["icnt"].item()) + sum(int(p["icnt"].item()) for p in lanes[0]["parts"])
    bw = None
    if args.bw_iters > 0:
        ln0 = lanes[0]
        bw = bw_iteration_leg(
            ctx, lambda m: D.bw_estep(ctx, m, dp, N, TRAIN, out=ln0["ecnt"]),
            lambda m: decode_step(ctx, m, dp, N, ln0["so"], ln0["score"], ln0["iout"], ln0["icnt"],
                                  fused_decode, first_chunk),
            N * world, args.bw_iters, dist, dev, backend)
    cold = None
    if args.cold_steps > 0 and not dist and not args.flush_mb:
        cold = cold_cache_steps(lanes[0], dp, ds, N, model0, model1, args.cold_steps, main_s, dev,
                                first_chunk, fused=fused, fused_decode=fused_decode)
    # N = 1: the C3 strong-scaling workload (the one the N > 1 lines run) on this one GPU, a
    # short leg after the headline, plus the count kernel over its HBM-resident genome
    c3_leg = None
    if not dist and args.c3_steps > 0:
        import copy
        a3 = copy.copy(args)
        a3.steps, a3.warmup, a3.bases = args.c3_steps, 3, C3_BASES
        c3_leg = run_c3(a3, 1, 0, local, False, backend, dev, emit=False)
        if c3_leg is not None:
            c3_leg = {k: c3_leg[k] for k in ("value", "unit", "ms_per_step", "steps",
                                              "warmup_steps_run", "scaling", "config",
                                              "phases_ms", "roofline", "roofline_count",
                                              "fingerprint", "bw_iteration")
                      if k in c3_leg}
    steps = args.steps
    ms_per_step = elapsed * 1e3 / steps
    value = N * world * steps / elapsed
    phases = {k: (v / nrec[k] if nrec[k] else 0.0) for k, v in acc.items()}
    if flush is not None:
        phases_total = sum(phases.values())
        ms_per_step = phases_total   # exclude the cache-flush writes from the step time
        value = N * world / (phases_total / 1e3)

    if rank == 0:
        # dominant kernel (rocprof, profiles/): the E-step chunk kernel.  achieved = its
        # algorithmic bytes per launch / the phase's mean duration (HIP events on its stream;
        # the phase is k_estep_chunk + the ~4 us one-workgroup final kernel).
        # (fused: the phase is the training pass, whose one kernel also reads the label bits)
        dom = "estep"
        bpb = BYTES_PER_BASE[dom] + (0.125 if fused else 0.0)
        alg_bytes = bpb * N
        ach = alg_bytes / (phases[dom] / 1e3) / 1e9 if phases[dom] > 0 else 0.0
        roof = {"bound": "hbm",
                "kernel": (ESTEP_KERNEL + " (training pass: E-step + labelled counts)"
                           if fused else ESTEP_KERNEL), "phase": dom,
                "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                "algorithmic_bytes": alg_bytes, "bytes_per_base": bpb}
        pmc = _pmc_traffic(ESTEP_KERNEL, N)
        if pmc:
            roof["traffic"] = pmc["traffic_bytes"]
            roof["traffic_source"] = ("stored PMC profile, not this run: " + pmc["source"])
        # "bound" names the roof the kernel is priced against (the contract's HBM roofline);
        # what actually limits it is measured by the PMC passes and reported beside it
        # with pipeline lanes, launches of consecutive steps overlap: `achieved` is per launch
        # (its own duration, shared GPU), the kernel's delivered rate over the timed region is
        # one launch's algorithmic bytes per step time
        roof["concurrent_launches"] = nlanes
        roof["aggregate_achieved"] = round(alg_bytes / (ms_per_step / 1e3) / 1e9, 1)
        roof["limiter"] = "fp64 VALU issue + dependency latency, not HBM (PMC: profiles/*pmc*)"
        roof["note"] = ("exact fp64 forward-backward: ~50 VALU instructions per base against "
                        "0.25 B/base of HBM traffic; DESIGN.md 5")
        # the limiter named above, priced: algorithmic fp64 flops per launch / the same phase
        # time, against the fp64 vector peak
        fl = ESTEP_FLOPS_PER_BASE * N / (phases[dom] / 1e3) / 1e12 if phases[dom] > 0 else 0.0
        roof_fp64 = {"bound": "valu-fp64", "kernel": ESTEP_KERNEL, "phase": dom,
                     "achieved": round(fl, 2), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(fl / FP64_PEAK_TFLOPS, 4),
                     "flops_per_base": ESTEP_FLOPS_PER_BASE}
        vit = phases["decode"] if "decode" in phases else phases["viterbi"] + phases["islands"]
        dbpb = (BYTES_PER_BASE["decode_fused"] if fused_decode else
                BYTES_PER_BASE["viterbi"] + BYTES_PER_BASE["islands"])
        roof_decode = {"bound": "hbm", "phase": "viterbi+islands", "achieved": round(
            dbpb * N / (vit / 1e3) / 1e9 if vit > 0 else 0.0, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None, "bytes_per_base": dbpb,
            "algorithmic_bytes": dbpb * N}
        roof_decode["frac"] = round(roof_decode["achieved"] / HBM_PEAK_GBS, 4)
        roof_decode_valu = _decode_valu(N, vit)
        out = {"metric": METRIC, "value": value, "unit": "bases/s", "n_gpus": world,
               "steps": steps, "warmup": args.warmup, "warmup_steps_run": nwarm,
               "settle_ms": args.settle_ms, "ms_per_step": ms_per_step,
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
               "dtype": "f64", "data": "synthetic (counter-based planted-island genome, "
                                        f"seed {SEED})",
               "config": {"workload": "C2: 46 Mbp chr21-sized per GPU; BW E-step + labelled "
                                      "counts + RCCL reduce + exact Viterbi + islands",
                          "streams": 1 if args.serial else 2,
                          "train_pass": ("fused: cpg_train_pass_d, E-step + labelled counts in "
                                         "one launch" if fused else "separate launches"),
                          "decode": ("fused: cpg_decode_d, traceback writes the island run "
                                     "records" if fused_decode else "separate calls"),
                          "decode_priority": "high" if (args.prio and not args.serial) else "normal",
                          "step_overlap": not (args.no_overlap or args.serial),
                          "pipeline_lanes": nlanes,
                          "train_lanes": ntl,
                          "decode_lanes": ndl,
                          "decode_cus_from": args.decode_cus_from,
                          "phase_events": ("all" if full_ev else
                                           f"estep every {args.estep_event_every}, decode every {args.decode_event_every}"),
                          "train_cus": len(tr_cus) if tr_cus else ncu,
                          "bases_per_gpu": N, "train_chunk": TRAIN, "decode_chunk": DECODE,
                          "decode_chunks_per_gpu": ndec, "parallelism": f"dp{world}",
                          "decode_parts": nsplit,
                          "conditions": ("warm cache: the 11.5 MB packed shard stays in the "
                                         "256 MB Infinity Cache between steps (cold_cache: "
                                         "1 GiB flush before each step); fixed models: "
                                         "E-step on the reference's initial model, Viterbi on "
                                         "the model after one BW iteration, per-model tables "
                                         "built before the timed region"),
                          "collectives": (("rccl" if backend == "nccl" else backend)
                                          if dist else None),
                          "islands_found": islands_found},
               "phases_ms": {k: round(v, 4) for k, v in phases.items()},
               "host_issue_ms_per_step": round(issue * 1e3 / steps, 4),
               "roofline": roof, "roofline_fp64": roof_fp64, "roofline_decode": roof_decode,
               "roofline_decode_valu": roof_decode_valu, "cold_cache": cold,
               "fingerprint": fingerprint, "bw_iteration": bw}
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(SEED, args.cpu_sample,
                                                min(args.cpu_threads, os.cpu_count() or 1))
        else:
            out["cpu_baseline"] = None
        out["c3_single_gpu"] = c3_leg
        if c3_leg is not None:
            out["roofline_count"] = c3_leg.pop("roofline_count", None)
        print(json.dumps(out), flush=True)
    for ln in lanes:
        for cx3, st in ln["tr"]:
            if tr_cus:
                D.cu_stream_destroy(st)
            if cx3 is not ln["ctx"]:
                cx3.close()
        for dl in ln["dec"][1:]:
            dl[0].close()
        if args.decode_cus_from > 0 and not args.serial:
            D.cu_stream_destroy(ln["s_dec"])
        for part in ln["parts"]:
            part["ctx"].close()
        ln["ctx"].close()
    if dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
