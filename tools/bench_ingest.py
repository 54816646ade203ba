"""Device-side reader throughput (cpg_ingest_d): FASTA-like text (width 60, header) of the
bench genome, resident in HBM; HIP events on the launching stream.  Prints one JSON line."""
import argparse
import json
import os
import sys

os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("CPG_DEV_PKG"):   # a variant tree from tools/build_variant.sh
    sys.path.insert(0, os.environ["CPG_DEV_PKG"])
from cpgisland_amd import Context  # noqa: E402
from cpgisland_amd import device as D  # noqa: E402
from oracle import pyref as pr  # noqa: E402


def make_text(nbases, width=60, seed=20251016):
    packed, _ = D.synth_host(seed, 0, nbases)
    seq = np.frombuffer(b"ACGT", np.uint8)[pr.unpack(packed, nbases)]
    nl = nbases // width
    body = np.empty((nl, width + 1), np.uint8)
    body[:, :width] = seq[: nl * width].reshape(nl, width)
    body[:, width] = ord("\n")
    return b">chr21 synthetic\n" + body.tobytes() + bytes(seq[nl * width:])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bases", type=int, default=46_000_000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--mode", type=int, default=0)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    txt = make_text(args.bases)
    n = len(txt)
    dt = D.text_to_device(txt, dev)
    ctx = Context(0)
    out, res = D.ingest(ctx, dt, n, args.mode, True)
    torch.cuda.synchronize()
    r = res.cpu().numpy()
    assert r[1] in (0, -5), r     # -5: the decode reader would throw (FASTA cadence)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.reps)]
    for a, b in ev:
        a.record()
        D.ingest(ctx, dt, n, args.mode, True, out=out, result=res)
        b.record()
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ev)
    med = ms[len(ms) // 2]
    nb = int(r[3])
    alg = n + nb / 4.0                     # read every byte once, write 2 bits per base
    print(json.dumps({"kernel": "k_ingest", "bytes_in": n, "bases": nb, "mode": args.mode,
                      "status": int(r[1]), "extra_chunks": int(r[4]),
                      "ms_median": med, "ms_min": ms[0], "GBps_alg": alg / med / 1e6,
                      "frac_of_8TBps": alg / med / 1e6 / 8000.0,
                      "bytes_per_s_text": n / med * 1e3}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
