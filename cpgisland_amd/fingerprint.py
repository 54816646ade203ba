"""Whole-genome result digests: what a run of the hot path over one of the bench genomes
produced, in a form that compares with the oracle's digests of the same genome.

`tests/golden/fingerprints.json` holds the oracle's digests of the two bench workloads
(C2: the 46 Mbp chr21-sized sequence, C3: the 3.1 Gbp hg38-sized genome), written by
`tests/golden/make_fingerprints.py` from oracle/cpg_oracle.c over EVERY training and decode
chunk (the Mahout-order 8-state Viterbi of `CpGIslandFinder.java:260`, the island scan of
`:262-339` with the int32 coordinates of `:287`, the labelled int64 counts, the fp64 E-step of
the mapper called at `:200`).  This module only reads that data file and hashes device
results; it never imports or runs anything under oracle/.

Digests:
  path     SHA-256 of the sign-bit words of the decoded chunks (32 bases per uint32, bit
           k = base k is '+', i.e. state < 4), plus one 64-bit digest per chunk to name the
           first chunk that differs
  scores   the best log-probability per chunk, as IEEE-754 bit patterns
  records  SHA-256 of the cpg_island records in chunk order (32 B each), and their count
  counts   the 124 labelled int64 counts (cpg_counts_i64), exact
  estep    the 105 E-step doubles (cpg_counts_f64), within 1e-9 relative plus the
           fixed-point grid bound the fixture states per entry (k_estep.hip)
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

from . import _lib

FILE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "tests", "golden", "fingerprints.json")
ESTEP_RTOL = 1e-9        # north_star: fp64 within 1e-9 relative


def load(path: str = FILE) -> dict:
    with open(path) as f:
        return json.load(f)


def f64_to_hex(a) -> list[str]:
    return [f"{int(x):016x}" for x in np.ascontiguousarray(a, np.float64).view(np.uint64)]


def hex_to_f64(h) -> np.ndarray:
    return np.array([int(x, 16) for x in h], np.uint64).view(np.float64)


def sha256(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).view(np.uint8).tobytes())
    return h.hexdigest()


def chunk_digests(sign_words: np.ndarray, nchunks: int, chunk_len: int) -> list[str]:
    """One 64-bit digest (16 hex digits of SHA-256) per decode chunk of the sign path."""
    w = chunk_len // 32
    return [hashlib.sha256(np.ascontiguousarray(sign_words[c * w:(c + 1) * w]).tobytes())
            .hexdigest()[:16] for c in range(nchunks)]


def decode_digest(sign_words: np.ndarray, scores: np.ndarray, records: np.ndarray,
                  nchunks: int, chunk_len: int = _lib.DECODE_CHUNK,
                  per_chunk: bool = False) -> dict:
    """Digest of a decode's outputs: sign words (uint32) of at least nchunks whole chunks,
    the per-chunk scores, the island records (cpg_island array or raw bytes)."""
    sw = np.ascontiguousarray(np.asarray(sign_words).view(np.uint32)[: nchunks * chunk_len // 32])
    sc = np.ascontiguousarray(np.asarray(scores, np.float64)[:nchunks])
    rec = np.ascontiguousarray(records)
    nrec = rec.size if rec.dtype == _lib.ISLAND_DTYPE else rec.size // _lib.ISLAND_DTYPE.itemsize
    d = {"chunks": int(nchunks), "path_sha256": sha256(sw), "scores_sha256": sha256(sc),
         "records_sha256": sha256(rec), "islands": int(nrec)}
    if per_chunk:
        d["chunk_path_digests"] = chunk_digests(sw, nchunks, chunk_len)
        d["scores_hex"] = f64_to_hex(sc)
    return d


def estep_close(got, ref_hex, bound_hex) -> tuple[bool, float]:
    """|got - oracle| <= grid bound + 1e-9 |oracle| on every entry, zeros where the oracle's
    are; returns (ok, the largest relative error over the non-zero entries)."""
    got = np.asarray(got, np.float64)
    ref, bound = hex_to_f64(ref_hex), hex_to_f64(bound_hex)
    err = np.abs(got - ref)
    ok = bool(np.array_equal(got == 0, ref == 0) and
              (err <= bound + ESTEP_RTOL * np.abs(ref)).all())
    nz = ref != 0
    rel = float(np.max(err[nz] / np.abs(ref[nz]))) if nz.any() else 0.0
    return ok, rel


def compare(fx: dict, estep=None, counts=None, decode: dict | None = None) -> dict:
    """Compare one run with the fixture entry `fx` (one config of fingerprints.json).
    Returns {"oracle_match": bool, per-part booleans, the first differing chunk if any}."""
    r = {}
    if counts is not None:
        r["counts"] = bool(np.array_equal(np.asarray(counts, np.int64),
                                          np.asarray(fx["train"]["counts"], np.int64)))
    if estep is not None:
        ok, rel = estep_close(estep, fx["train"]["estep_hex"], fx["train"]["estep_bound_hex"])
        r["estep"] = ok
        r["estep_max_rel_err"] = rel
    if decode is not None:
        fd = fx["decode"]
        r["path"] = decode["path_sha256"] == fd["path_sha256"]
        r["scores"] = decode["scores_sha256"] == fd["scores_sha256"]
        r["records"] = (decode["records_sha256"] == fd["records_sha256"] and
                        decode["islands"] == fd["islands"])
        if not r["path"] and "chunk_path_digests" in decode:
            bad = [c for c, (a, b) in enumerate(zip(decode["chunk_path_digests"],
                                                     fd["chunk_path_digests"])) if a != b]
            r["path_chunks_differing"] = bad[:16]
    parts = [k for k in ("counts", "estep", "path", "scores", "records") if k in r]
    r["oracle_match"] = bool(parts) and all(r[k] for k in parts)
    r["checked"] = parts
    return r
