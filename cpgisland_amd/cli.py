"""The reference's command line on the GPU path — CpGIslandFinder.main (/root/reference/
CpGIslandFinder.java:346-357):

    python -m cpgisland_amd.cli trainingFile testFile islandsOut trainedHmmFile convergence numIter

  trainModel (:102-225)
    ingest       raw training text -> HBM -> packed 65,536-base chunks, with the reader's quirks
                 (the extra all-A chunk, header letters counted, tail dropped): cpg_ingest_d
    Baum-Welch   runBaumWelchMR(..., convergence, "rescaling", numIter) (:200-201): the GPU
                 E-step per iteration (cpg_bw_estep_d), reducer cpg_bw_normalize, Mahout
                 HmmTrainer's convergence rule (baumwelch.run)
    model file   Double.toString lines of :207-224 (cpg_format_model)
  testModel (:227-344)
    ingest       raw test text -> packed 1 Mi chunks (cpg_ingest_d, mode 1); a non-ACGT byte
                 read while the base count sits on a chunk multiple makes the reference throw
                 IndexOutOfBoundsException at :258 (CPG_E_REF_CRASH)
    decode       HmmEvaluator.decode (:260) + the island scan / filter (:262-339) of every
                 whole chunk in one call (cpg_decode_d)
    island file  "%d %d %d %f %f\\n" lines of :287-288 (cpg_format_islands)

Where the reference throws, this driver writes the islands of the chunks decoded before the
throw and exits with status 1 and the exception's name (the Java process would also exit 1;
how much of its unflushed BufferedWriter reached the file is not emulated).  Logging follows
the reference's two slf4j lines (:147, :228) on stderr.
"""
from __future__ import annotations

import sys


from . import _lib, baumwelch
from .hmm import Context, HmmModel, format_islands, format_model


def _java_int(x: int) -> int:
    """Java int arithmetic (the reference's `count` is an int, :107, :236)."""
    return (x + (1 << 31)) % (1 << 32) - (1 << 31)


def _ingest(ctx: Context, path: str, mode: int):
    """The reader of :112-145 (mode 0) / :238-259 (mode 1) on the device: returns (packed
    device tensor, committed bases, result row as python ints)."""
    import torch
    from . import device as D
    with open(path, "rb") as f:
        txt = f.read()
    dev = torch.device("cuda", ctx.device)
    d_txt = D.text_to_device(txt, dev)
    chunk = _lib.TRAIN_CHUNK if mode == 0 else _lib.DECODE_CHUNK
    cap = None
    for _ in range(2):
        packed, res = D.ingest(ctx, d_txt, len(txt), mode, True, cap_bases=cap)
        torch.cuda.synchronize()
        ctx.sync()
        r = [int(v) for v in res.cpu().tolist()]
        if r[1] != _lib.CPG_E_CAPACITY:
            break
        # the training reader's extra all-A chunks outnumbered the default slack: size exactly
        # (valid bases + extra chunks, both reported by the first pass)
        cap = ((r[3] // chunk) + r[4] + 2) * chunk
    if r[1] not in (_lib.CPG_OK, _lib.CPG_E_REF_CRASH):
        raise _lib.CpgError(r[1], f"device ingest of {path} failed (status {r[1]})")
    return packed, r[0], r


def train_model(ctx: Context, training_path: str, trained_hmm_file: str, num_iter: int,
                convergence: str, log=print):
    """trainModel (:102-225): returns (trained model, iterations run)."""
    packed, nbases, r = _ingest(ctx, training_path, 0)
    log(f"INFO: Size of input file:{_java_int(r[3])}")          # :147 (ACGT bytes read)
    model, iters, _ = baumwelch.run(ctx, packed, nbases, model=HmmModel.initial(),
                                    convergence=float(convergence), max_iter=num_iter)
    with open(trained_hmm_file, "wb") as f:
        f.write(format_model(model))
    return model, iters


def test_model(ctx: Context, model: HmmModel, test_path: str, islands_out: str, log=print):
    """testModel (:227-344): returns (island records, crashed)."""
    import torch
    from . import device as D
    log("INFO: testing")                                         # :228
    packed, nbases, r = _ingest(ctx, test_path, 1)
    cap = 1 << 16
    for _ in range(2):   # (a second pass sized by the first pass's exact count)
        _, _, out, cnt = D.decode(ctx, model, packed, nbases, _lib.DECODE_CHUNK, cap=cap)
        torch.cuda.synchronize()
        ctx.sync()
        n = int(cnt.item())
        if n <= cap:
            break
        cap = n
    recs = D.islands_to_numpy(out, cnt)
    with open(islands_out, "wb") as f:
        f.write(format_islands(recs))
    return recs, r[1] == _lib.CPG_E_REF_CRASH


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if len(argv) < 6:
        print("usage: python -m cpgisland_amd.cli trainingFile testFile islandsOut "
              "trainedHmmFile convergence numIter", file=sys.stderr)
        return 2
    training_file, test_file, islands_file, trained_hmm_file, convergence = argv[:5]
    num_iter = int(argv[5])                                      # Integer.parseInt (:352)

    def log(msg):
        print(msg, file=sys.stderr, flush=True)

    with Context(0) as ctx:
        model, _ = train_model(ctx, training_file, trained_hmm_file, num_iter, convergence, log)
        _, crashed = test_model(ctx, model, test_file, islands_file, log)
    if crashed:
        log('Exception in thread "main" java.lang.IndexOutOfBoundsException '
            "(CpGIslandFinder.java:258: a non-ACGT byte read while the base count sits on a "
            "1 Mi multiple)")
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
