"""End to end: the reference's command line (CpGIslandFinder.main, :346-357) on the GPU path
(cpgisland_amd.cli) against the oracle pipeline on small synthetic FASTA files with a header
line, 60-column lines and N runs: ingest (:112-145, :238-259) -> Baum-Welch iterations
(:200-203, convergence args[4], <= args[5] iterations) -> trained-model file (:207-224) ->
decode (:260) -> islands (:262-339) -> island file (:287-288).

  * island file: byte for byte equal to the oracle pipeline's (its own BW-trained model);
  * trained-model file: byte for byte equal to the Java formatter restatement of the model the
    GPU trained (oracle/pyref.format_model); the model itself within 1e-9 relative of the
    oracle's (the E-step is a tolerance-bound fp64 sum: tests/test_gpu_parity.py), with the
    same number of iterations;
  * a decode reader crash (:257-258) -> exit status 1, the islands decoded before it written.
"""
import math
import os

import numpy as np
import pytest

from oracle import coracle as co
from oracle import pyref as pr

pytestmark = pytest.mark.gpu
TRAIN, DECODE = 65536, 1 << 20


def _fasta(seed, n, header=b">chr_test synthetic island genome\n", nrun=(5000, 700)):
    from cpgisland_amd import device as D
    packed, _ = D.synth_host(seed, 0, n)
    body = pr.unpack(packed, n).tobytes().translate(bytes.maketrans(b"\0\1\2\3", b"ACGT"))
    at, ln = nrun
    body = body[:at] + b"N" * ln + body[at:]
    lines = [body[i:i + 60] for i in range(0, len(body), 60)]
    return header + b"\n".join(lines) + b"\n"


def _oracle_pipeline(train_txt, test_txt, eps, num_iter):
    obs = co.ingest_train(train_txt)
    m = co.initial_model()
    it = 0
    for it in range(1, num_iter + 1):
        new = co.normalize(co.estep(m, obs, TRAIN))
        pi0, a0, b0 = co.model_split(m)
        pi1, a1, b1 = co.model_split(new)
        na = math.sqrt(sum((u - v) ** 2 for u, v in zip(a0.ravel().tolist(), a1.ravel().tolist())))
        nb = math.sqrt(sum((u - v) ** 2 for u, v in zip(b0.ravel().tolist(), b1.ravel().tolist())))
        m = new
        if na + nb < eps:
            break
    sd, crash = co.ingest_decode(test_txt)
    _, isl, _ = co.decode_chunks(m, sd, DECODE)
    return m, it, "".join(co.format_island(r) for r in isl).encode(), crash


@pytest.fixture(scope="module")
def files(tmp_path_factory):
    d = tmp_path_factory.mktemp("cli")
    tr = _fasta(31, 24 * TRAIN + 777)
    te = _fasta(32, 3 * DECODE + 4321)
    (d / "train.fa").write_bytes(tr)
    (d / "test.fa").write_bytes(te)
    return d, tr, te


@pytest.mark.parametrize("eps,num_iter", [(".005", 3), ("1e-12", 2)])
def test_cli_matches_oracle_pipeline(files, eps, num_iter):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cpgisland_amd import baumwelch, cli
    d, tr, te = files
    isl_out, hmm_out = d / f"islands_{num_iter}.txt", d / f"model_{num_iter}.txt"
    rc = cli.main([str(d / "train.fa"), str(d / "test.fa"), str(isl_out), str(hmm_out), eps,
                   str(num_iter)])
    assert rc == 0
    m_ref, it_ref, isl_ref, crash = _oracle_pipeline(tr, te, float(eps), num_iter)
    assert not crash
    got_isl = isl_out.read_bytes()
    assert got_isl == isl_ref and len(got_isl) > 0
    # the trained-model file: Double.toString lines of the GPU-trained model
    text = hmm_out.read_text()
    rows = [ln for ln in text.split("\n")]
    assert len(rows) == 25 and rows[-1] == ""
    vals = np.array([float(v) for r in rows[:-1] for v in r.split()], np.float64)
    m_gpu = np.concatenate([vals[[13 * i for i in range(8)]],
                            np.concatenate([vals[13 * i + 1:13 * i + 9] for i in range(8)]),
                            np.concatenate([vals[13 * i + 9:13 * i + 13] for i in range(8)])])
    assert text.encode() == pr.format_model(m_gpu).encode()
    nz = m_ref != 0
    assert np.array_equal(m_gpu == 0, m_ref == 0)
    assert np.max(np.abs(m_gpu[nz] - m_ref[nz]) / np.abs(m_ref[nz])) < 1e-9
    # the same number of iterations as the oracle's loop
    _, it_gpu, _ = baumwelch.run(None, None, 0, mapper=_gpu_mapper(tr), convergence=float(eps),
                                 max_iter=num_iter)
    assert it_gpu == it_ref


def _gpu_mapper(train_txt):
    import torch
    from cpgisland_amd import Context
    from cpgisland_amd import device as D
    obs = co.ingest_train(train_txt)
    ctx = Context(0)
    dp = D.to_device(np.concatenate([pr.pack(obs), np.zeros(8, np.uint32)]), torch.device("cuda:0"))
    return lambda m: D.bw_estep(ctx, m, dp, len(obs))


def test_cli_decode_reader_crash(files, tmp_path):
    """A newline read while the decode reader's count sits on 2^20 (:256-258): the reference
    throws; the driver writes the islands decoded before and exits 1."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cpgisland_amd import cli
    d, tr, _ = files
    body = _fasta(33, 2 * DECODE, header=b"", nrun=(0, 0)).replace(b"\n", b"")
    te = body[:DECODE] + b"\n" + body[DECODE:]
    (tmp_path / "crash.fa").write_bytes(te)
    isl_out, hmm_out = tmp_path / "isl.txt", tmp_path / "model.txt"
    rc = cli.main([str(d / "train.fa"), str(tmp_path / "crash.fa"), str(isl_out), str(hmm_out),
                   ".005", "1"])
    assert rc == 1
    sd, crash = co.ingest_decode(te)
    assert crash and len(sd) == DECODE
    m = np.array([float(v) for v in hmm_out.read_text().split()], np.float64)
    assert len(m) == 104
