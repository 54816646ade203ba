"""Baum-Welch training — the host side of BaumWelchDriver.runBaumWelchMR (called at
/root/reference/CpGIslandFinder.java:200-201; MAHOUT-627 MapReduce classes, unvendored).

  mapper   -> estep()      the fp64 expected-count stripes of every 65,536-base chunk
                           (GPU kernel, cpg_bw_estep_d)
  reducer  -> normalize()  sum of stripes + row normalisation (cpg_bw_normalize)
  driver   -> run()        iterate until converged or max_iter (convergence rule:
                           Mahout HmmTrainer's — the MAHOUT-627 rule is unpinned)
Multi-GPU: each rank runs the mapper on its shard; the stripes are all-gathered and summed
in rank order (dist.merge_counts_f64: deterministic), then every rank normalises identically
(no broadcast).
"""
from __future__ import annotations

import math

import numpy as np

from . import _lib, dist
from ._lib import check, lib, ptr
from .hmm import Context, HmmModel


def normalize(counts) -> HmmModel:
    """The reducer: counts (cpg_counts_f64 layout, 105 doubles) -> row-normalised model."""
    c = np.ascontiguousarray(counts, dtype=np.float64)
    assert c.size == _lib.COUNTS_F64_N
    m = np.zeros(_lib.MODEL_N, np.float64)
    check(lib.cpg_bw_normalize(ptr(c), ptr(m)))
    return HmmModel.from_struct(m)


def normalize_labelled(counts) -> HmmModel:
    """M-step of the labelled (hard-label) counts, cpg_counts_i64 layout."""
    c = np.ascontiguousarray(counts, dtype=np.int64)
    m = np.zeros(_lib.MODEL_N, np.float64)
    check(lib.cpg_counts_normalize(ptr(c), ptr(m)))
    return HmmModel.from_struct(m)


def converged(old: HmmModel, new: HmmModel, epsilon: float) -> bool:
    """Mahout HmmTrainer.checkConvergence: sqrt(sum (dA)^2) + sqrt(sum (dB)^2) < eps, the sums
    taken element by element in row-major order as the Java loops do (not numpy's pairwise
    summation, which rounds differently)."""
    def norm(x, y):
        acc = 0.0
        for u, v in zip(np.ravel(x).tolist(), np.ravel(y).tolist()):
            d = u - v
            acc += d * d
        return math.sqrt(acc)
    return norm(old.a, new.a) + norm(old.b, new.b) < epsilon


def estep(ctx: Context, model: HmmModel, packed, nbases: int,
          chunk_len: int = _lib.TRAIN_CHUNK, group=None, distributed: bool = False):
    """The mapper over one shard (device tensor) -> host counts (105 doubles).  With
    `distributed`, the stripes of all ranks are summed in rank order (dist.merge_counts_f64):
    every rank gets the same bits."""
    from . import device as D
    out = D.bw_estep(ctx, model, packed, nbases, chunk_len)
    if distributed:
        dist.merge_counts_f64(out, group)
    return out.cpu().numpy()


def run(ctx: Context | None, packed, nbases: int, model: HmmModel | None = None,
        convergence: float = 0.005, max_iter: int = 10,
        chunk_len: int = _lib.TRAIN_CHUNK, distributed: bool = False, group=None,
        mapper=None):
    """runBaumWelchMR(conf, input, modelIn, output, ..., convergence, "rescaling", numIter).
    `mapper(model) -> torch tensor of 105 doubles` overrides the shard's E-step (default:
    the GPU kernel over `packed`); the reducer merge and the loop are the same either way.
    Returns (trained model, iterations run, log-likelihood of the last E-step)."""
    import torch
    from . import device as D
    if mapper is None:
        def mapper(m):
            return D.bw_estep(ctx, m, packed, nbases, chunk_len)
    model = model or HmmModel.initial()
    ll = -math.inf
    it = 0
    for it in range(1, max_iter + 1):
        t = mapper(model)
        if not isinstance(t, torch.Tensor):
            t = torch.as_tensor(np.asarray(t, dtype=np.float64))
        if distributed:
            dist.merge_counts_f64(t, group)
        counts = t.cpu().numpy()
        ll = float(counts[-1])
        new = normalize(counts)
        done = converged(model, new, convergence)
        model = new
        if done:
            break
    return model, it, ll
