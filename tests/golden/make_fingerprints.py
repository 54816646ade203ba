"""Generate tests/golden/fingerprints.json — the oracle's results over the WHOLE bench genomes.

TEST INFRASTRUCTURE (the checker): runs oracle/cpg_oracle.c over every chunk of the two bench
workloads and records digests that the GPU tests (tests/test_gpu_fingerprints.py) and
bench.py's `fingerprint.oracle_match` compare the HIP path's results with:

  C2  configs[1]  46 Mbp chr21-sized, seed 20251016, bases [0, 46e6):  701 training chunks,
                  43 decode chunks
  C3  configs[2]  3.1 Gbp hg38-sized, seed 20251017, bases [0, 3.1e9): 47,302 training chunks,
                  2,956 decode chunks (chunks 2,048.. carry the int32-wrapped coordinates of
                  CpGIslandFinder.java:287)

Per config:
  genome   SHA-256 of the packed bases and the truth (label) bits cpg_synth produced
  train    the labelled int64 counts (orc_count_labelled) and the E-step sum (orc_estep8,
           the Rabiner-scaled forward-backward restated for the unvendored mapper called at
           :200) of every whole 65,536-base chunk (:130-141) under the reference's initial
           model (:155-173), plus the per-entry absolute bound of the GPU's fixed-point grid
           (k_estep.hip; tests/test_gpu_parity.py estep_grid_bound)
  decode   the decode model — the reducer's row normalisation (orc_normalize) of that E-step,
           i.e. one Baum-Welch iteration, committed as IEEE-754 bit patterns so the GPU and
           the oracle decode with identical constants — and, under it, the Mahout-order
           8-state Viterbi (orc_viterbi8, HmmEvaluator.decode(model, obs, true) :260) of every
           whole 1,048,576-base chunk (:256-259): SHA-256 of the sign path (32 bases per
           uint32, '+' = state < 4), a 64-bit digest per chunk, the per-chunk best scores,
           and SHA-256 of the island records (orc_islands, :262-339, int32 coordinates :287)
           in chunk order

PARITY UNPINNED: the oracle is this build's restatement of the reference (no
JDK, Mahout/MAHOUT-627 unvendored, no reference fixtures).

    python tests/golden/make_fingerprints.py [C2] [C3]      (all cores; C3 takes minutes)
"""
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import coracle as co  # noqa: E402
from cpgisland_amd import device as D  # noqa: E402  (host-only: cpg_synth)
from cpgisland_amd import fingerprint as F  # noqa: E402

TRAIN = 65536
DECODE = 1 << 20
CONFIGS = {"C2": {"seed": 20251015 + 1, "start": 0, "nbases": 46_000_000,
                  "bench": "bench.py (N = 1 headline line: rank 0's shard)"},
           "C3": {"seed": 20251015 + 2, "start": 0, "nbases": 3_100_000_000,
                  "bench": "bench.py c3_single_gpu / --workload c3 (every N: rank-order merge)"}}
TRAIN_JOB = 64          # training chunks per worker job


def unpack(words):
    sh = (np.arange(16, dtype=np.uint32) * 2)[None, :]
    return ((words[:, None] >> sh) & 3).astype(np.uint8).ravel()


def unpack_bits(words):
    sh = np.arange(32, dtype=np.uint32)[None, :]
    return ((words[:, None] >> sh) & 1).astype(np.uint8).ravel()


def grid_bound(nd, nch):
    """Per-entry absolute bound of the GPU E-step's fixed-point sums (k_estep.hip), from the
    16 within-chunk dinucleotide class counts nd (previous base | current base << 2)."""
    b = np.zeros(105)
    b[:8] = nch * 2.0 ** -63
    for i in range(8):
        for j in range(8):
            b[8 + 8 * i + j] = nd[(i & 3) | ((j & 3) << 2)] * 2.0 ** -47
    for j in range(8):
        b[72 + 4 * j + (j & 3)] = b[j] + sum(b[8 + 8 * i + j] for i in range(8))
    b[104] = nch * 2.0 ** -25
    return b


def run_config(name, cfg, threads):
    seed, start, n = cfg["seed"], cfg["start"], cfg["nbases"]
    t0 = time.time()
    packed, sign = D.synth_host(seed, start, n)
    packed, sign = packed[: D.words16(n)], sign[: D.words32(n)]
    print(f"{name}: synthesised {n} bases in {time.time() - t0:.1f} s", flush=True)
    m0 = co.initial_model()
    ntr = n // TRAIN
    wpt, spt = TRAIN // 16, TRAIN // 32

    def train_job(c0):
        c1 = min(ntr, c0 + TRAIN_JOB)
        obs = unpack(packed[c0 * wpt:c1 * wpt])
        truth = unpack_bits(sign[c0 * spt:c1 * spt])
        e = co.estep(m0, obs, TRAIN)
        c = co.count_labelled(obs, truth, TRAIN)
        o = obs.reshape(c1 - c0, TRAIN).astype(np.int64)
        nd = np.bincount((o[:, :-1] | (o[:, 1:] << 2)).ravel(), minlength=16)
        return e, c, nd

    t1 = time.time()
    est = np.zeros(co.COUNTS_F64_N)
    cnt = np.zeros(co.COUNTS_I64_N, np.int64)
    nd = np.zeros(16, np.int64)
    with ThreadPoolExecutor(threads) as ex:
        for e, c, d in ex.map(train_job, range(0, ntr, TRAIN_JOB)):
            est += e               # job order = chunk order
            cnt += c
            nd += d
    print(f"{name}: E-step + counts over {ntr} chunks in {time.time() - t1:.1f} s", flush=True)
    m1 = co.normalize(est)

    nde = n // DECODE
    wpd = DECODE // 16

    def decode_job(c):
        obs = unpack(packed[c * wpd:(c + 1) * wpd])
        st, best = co.viterbi8(m1, obs)
        words = np.packbits((st < 4).astype(np.uint8), bitorder="little").view(np.uint32)
        return words, best, co.islands(st, start // DECODE + c)

    t2 = time.time()
    words, scores, recs = [], [], []
    with ThreadPoolExecutor(threads) as ex:
        for w, s, r in ex.map(decode_job, range(nde)):
            words.append(w)
            scores.append(s)
            recs.append(r)
    sw = np.concatenate(words) if words else np.zeros(0, np.uint32)
    rec = np.concatenate(recs) if recs else np.zeros(0, co.ISLAND_DTYPE)
    dd = F.decode_digest(sw, np.array(scores), rec, nde, DECODE, per_chunk=True)
    print(f"{name}: Viterbi + islands over {nde} chunks in {time.time() - t2:.1f} s "
          f"({dd['islands']} islands)", flush=True)
    return {"seed": seed, "start": start, "nbases": n, "bench": cfg["bench"],
            "genome": {"packed_sha256": F.sha256(packed), "sign_sha256": F.sha256(sign)},
            "train": {"chunk_len": TRAIN, "chunks": ntr, "model": "initial (:155-173)",
                      "estep_hex": F.f64_to_hex(est),
                      "estep_bound_hex": F.f64_to_hex(grid_bound(nd, ntr)),
                      "counts": [int(x) for x in cnt],
                      "dinuc_classes": [int(x) for x in nd]},
            "decode": dict({"chunk_len": DECODE, "first_chunk": start // DECODE,
                            "model_hex": F.f64_to_hex(m1),
                            "model": "orc_normalize(train.estep): one Baum-Welch iteration"},
                           **dd),
            "oracle_seconds": round(time.time() - t0, 1)}


def main():
    names = [a for a in sys.argv[1:] if a in CONFIGS] or list(CONFIGS)
    threads = os.cpu_count() or 8
    try:
        out = F.load()
    except OSError:
        out = {}
    out["_about"] = ("oracle/cpg_oracle.c over every chunk of the bench genomes; written by "
                     "tests/golden/make_fingerprints.py; compared by "
                     "cpgisland_amd/fingerprint.py (tests/test_gpu_fingerprints.py, bench.py). "
                     "PARITY UNPINNED: the oracle restates the reference (SURVEY.md 8c).")
    for name in names:
        out[name] = run_config(name, CONFIGS[name], threads)
        with open(F.FILE, "w") as f:
            json.dump(out, f, indent=1)
        print(f"{name}: written to {F.FILE}", flush=True)


if __name__ == "__main__":
    main()
