"""Load-shape ceilings for the count kernel (tools/loadshape.hip) on an HBM-resident buffer the
size of the C3 genome's packed bases + label bits, next to a plain read sweep of the same bytes
(tools/readsweep.hip).  Prints one JSON line per configuration, then the best of each shape.

usage: python tools/loadshape.py [--bases N]      (GPU; dev tool)
"""
import argparse
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def timed(fn, reps=10):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        ts.append((a, b))
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ts)
    return ms[len(ms) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bases", type=int, default=3_100_000_000)
    a = ap.parse_args()
    nblk = a.bases // 64 // 128 * 128
    dev = torch.device("cuda:0")
    packed = torch.randint(-2**31, 2**31 - 1, (nblk * 4,), dtype=torch.int32, device=dev)
    sign = torch.randint(-2**31, 2**31 - 1, (nblk * 2,), dtype=torch.int32, device=dev)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    ls = C.CDLL(os.path.join(ROOT, "tools", "libloadshape.so"))
    ls.loadshape.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_int,
                             C.c_int, C.c_int, C.c_void_p]
    rs = C.CDLL(os.path.join(ROOT, "tools", "libreadsweep.so"))
    rs.readsweep.argtypes = [C.c_void_p, C.c_int64, C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    nbytes = nblk * 24
    best = {}
    for grid in (1024, 2048, 4096, 8192):
        for inf in (2, 4, 8):
            def sw():
                rs.readsweep(C.c_void_p(packed.data_ptr()), nblk * 16, C.c_void_p(sink.data_ptr()), grid, inf, st)
                rs.readsweep(C.c_void_p(sign.data_ptr()), nblk * 8, C.c_void_p(sink.data_ptr()), grid, inf, st)
            sw()
            ms = timed(sw)
            r = {"kind": "readsweep", "grid": grid, "inflight": inf, "ms": ms, "TBps": nbytes / ms / 1e9}
            print(json.dumps(r), flush=True)
            if r["TBps"] > best.get("readsweep", {"TBps": 0})["TBps"]:
                best["readsweep"] = r
    for shape in (0, 1, 2):
        for depth in (1, 2, 4):
            for grid in (1024, 2048, 4096, 8192):
                for lds in (0, 40960):
                    def run():
                        rc = ls.loadshape(C.c_void_p(packed.data_ptr()), C.c_void_p(sign.data_ptr()),
                                          nblk, C.c_void_p(sink.data_ptr()), shape, depth, grid, lds, st)
                        assert rc == 0, rc
                    run()
                    ms = timed(run)
                    r = {"kind": f"shape{shape}", "depth": depth, "grid": grid,
                         "waves_per_simd": "max" if lds == 0 else 4, "ms": ms,
                         "TBps": nbytes / ms / 1e9}
                    print(json.dumps(r), flush=True)
                    k = f"shape{shape}/{r['waves_per_simd']}"
                    if r["TBps"] > best.get(k, {"TBps": 0})["TBps"]:
                        best[k] = r
    print(json.dumps({"best": best}), flush=True)


if __name__ == "__main__":
    main()
