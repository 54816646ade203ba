"""BASELINE config C4 on one MI355X: a batch of ragged contigs (log-uniform 150 bp - 50 kbp,
default 10M contigs ~ 86 Gbases) resident in HBM.  The bases come from a 2^30-base synthetic
genome tiled over the batch span (device copies; the content statistics are the synthetic
genome's).  Times, with HIP events on the launching streams: the length schedule (radix
sort), labelled counts, E-step, exact Viterbi, island scan; a "step" = train (E-step +
counts) and decode (Viterbi + islands) on two streams.  Prints one JSON line."""
import argparse
import json
import os
import sys
import time

os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("CPG_DEV_PKG"):   # a variant tree from tools/build_variant.sh
    sys.path.insert(0, os.environ["CPG_DEV_PKG"])
from cpgisland_amd import Context, HmmModel  # noqa: E402
from cpgisland_amd import device as D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--contigs", type=int, default=10_000_000)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(20251019)
    n = args.contigs
    lens = np.exp(rng.uniform(np.log(150), np.log(50000), n)).astype(np.int64)
    offs, span = D.contig_layout(lens)
    nbases = int(lens.sum())
    t0 = time.perf_counter()
    tile = 1 << 30
    p1, s1 = D.synth_host(20251019, 0, tile, 16)
    wp, ws = tile // 16, tile // 32
    words_p, words_s = D.words16(span) + 8, D.words32(span) + 8
    dp = torch.empty(words_p, dtype=torch.int32, device=dev)
    ds = torch.empty(words_s, dtype=torch.int32, device=dev)
    tp = D.to_device(p1[:wp], dev)
    tsg = D.to_device(s1[:ws], dev)
    for i in range(0, words_p, wp):
        k = min(wp, words_p - i)
        dp[i:i + k].copy_(tp[:k])
    for i in range(0, words_s, ws):
        k = min(ws, words_s - i)
        ds[i:i + k].copy_(tsg[:k])
    del tp, tsg
    d_offs = torch.from_numpy(offs).to(dev)
    d_lens = torch.from_numpy(lens.astype(np.int32)).to(dev)
    so = torch.zeros(words_s, dtype=torch.int32, device=dev)
    score = torch.empty(n, dtype=torch.float64, device=dev)
    ecnt = torch.empty(105, dtype=torch.float64, device=dev)
    lcnt = torch.empty(124, dtype=torch.int64, device=dev)
    icap = 1 << 24
    iout = torch.empty((icap, 32), dtype=torch.uint8, device=dev)
    icnt = torch.zeros(1, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    t_setup = time.perf_counter() - t0
    ctx = Context(0)
    m = HmmModel.initial()
    order = torch.empty(n, dtype=torch.int32, device=dev)
    s_tr, s_dec = torch.cuda.Stream(), torch.cuda.Stream(priority=-1)
    main_s = torch.cuda.current_stream()

    def ev():
        return torch.cuda.Event(enable_timing=True)

    def phase(fn):
        a, b = ev(), ev()
        a.record()
        fn()
        b.record()
        return a, b

    res = {k: [] for k in ("order", "counts", "estep", "viterbi", "islands", "step")}
    for rep in range(args.reps + 1):
        marks = {}
        marks["order"] = phase(lambda: D.contigs_order(ctx, d_lens, n, out=order))
        marks["counts"] = phase(lambda: D.contigs_count_labelled(ctx, dp, ds, span, d_offs, d_lens,
                                                                 order, n, out=lcnt))
        marks["estep"] = phase(lambda: D.contigs_estep(ctx, m, dp, span, d_offs, d_lens, order, n,
                                                       out=ecnt))
        marks["viterbi"] = phase(lambda: D.contigs_viterbi(ctx, m, dp, span, d_offs, d_lens, order,
                                                           n, sign_out=so, score=score))
        marks["islands"] = phase(lambda: D.contigs_islands(ctx, dp, so, span, d_offs, d_lens, order,
                                                           n, cap=icap, out=iout, count=icnt))
        # the step: schedule, then train and decode concurrently
        a = ev()
        a.record()
        D.contigs_order(ctx, d_lens, n, out=order)
        s_tr.wait_stream(main_s)
        s_dec.wait_stream(main_s)
        with torch.cuda.stream(s_tr):
            D.contigs_estep(ctx, m, dp, span, d_offs, d_lens, order, n, out=ecnt)
            D.contigs_count_labelled(ctx, dp, ds, span, d_offs, d_lens, order, n, out=lcnt)
        with torch.cuda.stream(s_dec):
            D.contigs_viterbi(ctx, m, dp, span, d_offs, d_lens, order, n, sign_out=so,
                              score=score)
            D.contigs_islands(ctx, dp, so, span, d_offs, d_lens, order, n, cap=icap, out=iout,
                              count=icnt)
        main_s.wait_stream(s_tr)
        main_s.wait_stream(s_dec)
        b = ev()
        b.record()
        marks["step"] = (a, b)
        torch.cuda.synchronize()
        ctx.sync()
        if rep > 0:
            for k, (x, y) in marks.items():
                res[k].append(x.elapsed_time(y))
    ms = {k: min(v) for k, v in res.items()}
    out = {"metric": "bases/sec train+Viterbi, ragged contig batch (C4, one GPU)",
           "value": nbases / (ms["step"] / 1e3), "unit": "bases/s", "n_gpus": 1,
           "contigs": n, "bases": nbases, "span": span, "ms": ms,
           "rates_bases_per_s": {k: nbases / (v / 1e3) for k, v in ms.items()},
           "islands": int(icnt.item()), "setup_seconds": t_setup,
           "data": "log-uniform 150-50000 bp lengths; bases tiled from a 2^30-base synthetic "
                   "genome"}
    print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
