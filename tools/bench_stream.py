"""BASELINE config C5 on one MI355X: a 3.1 Gbp (hg38-sized) synthetic genome in PINNED host
DRAM, streamed through cpg_genome_run (H2D windows overlapped with the E-step + labelled
counts + exact Viterbi + island scan, D2H of the decoded path).  The multi-genome batch runs
one genome per GPU (8 x 3.1 Gbp on 8 GPUs), so the per-GPU figure is this one.  Throughput
is PCIe-inclusive (host memory in, host memory out).  Prints one JSON line."""
import argparse
import ctypes as C
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
from cpgisland_amd import Context, HmmModel, _lib  # noqa: E402
from cpgisland_amd import device as D  # noqa: E402


def pinned(nwords):
    t = torch.empty(nwords, dtype=torch.int32, pin_memory=True)
    return t, t.numpy().view(np.uint32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bases", type=int, default=3_100_000_000)
    ap.add_argument("--window", type=int, default=64 << 20)
    ap.add_argument("--nbuf", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-labels", action="store_true")
    args = ap.parse_args()
    n = args.bases
    torch.cuda.init()
    tp, packed = pinned(D.words16(n) + 4)
    ts, sign = pinned(D.words32(n) + 4)
    to, sign_out = pinned(D.words32(n) + 4)
    t0 = time.perf_counter()
    _lib.check(_lib.lib.cpg_synth(C.c_uint64(20251015 + 5), 0, n, _lib.ptr(packed),
                                  _lib.ptr(sign), 16))
    t_synth = time.perf_counter() - t0
    ctx = Context(0)
    m0 = HmmModel.initial()
    m1 = m0
    ndec = n // (1 << 20)
    est = np.zeros(105)
    cnt = np.zeros(124, np.int64)
    sc = np.zeros(max(ndec, 1))
    cap = 1 << 22
    isl = np.zeros(cap, _lib.ISLAND_DTYPE)
    icount = C.c_int64()
    opts = np.zeros(3, np.int64)
    opts[0], opts[1] = args.window, args.nbuf
    lab = None if args.no_labels else sign

    def run():
        _lib.check(_lib.lib.cpg_genome_run(
            ctx.handle, _lib.ptr(m0.to_struct()), _lib.ptr(m1.to_struct()), _lib.ptr(packed),
            _lib.ptr(lab) if lab is not None else None, n, _lib.ptr(opts), _lib.ptr(est),
            _lib.ptr(cnt) if lab is not None else None, _lib.ptr(sign_out), _lib.ptr(sc),
            _lib.ptr(isl), cap, C.byref(icount)))

    run()   # warm-up (workspace allocation, code objects)
    times = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        run()
        times.append(time.perf_counter() - t0)
    best = min(times)
    h2d = D.words16(n) * 4 + (0 if lab is None else D.words32(n) * 4)
    d2h = D.words32(n) * 4
    print(json.dumps({
        "metric": "bases/sec train+Viterbi, genome streamed from pinned host DRAM (C5, per GPU)",
        "value": n / best, "unit": "bases/s", "n_gpus": 1, "bases": n,
        "seconds": best, "seconds_all": times, "window_bases": args.window, "nbuf": args.nbuf,
        "pcie_bytes_h2d": h2d, "pcie_bytes_d2h": d2h,
        "pcie_GBps_h2d_equiv": h2d / best / 1e9, "islands": icount.value,
        "labelled_counts": lab is not None, "synth_seconds": t_synth,
        "work": "E-step + labelled counts + exact Viterbi + islands + decoded path to host",
        "loglik": est[104]}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
