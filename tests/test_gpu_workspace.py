"""Workspace growth while another stream still reads the old buffer (regression for the
streamed-genome illegal-address fault fixed in 68bacec: ws_get freed a slot that a kernel
queued on another stream had not read yet).

Deterministic ordering: stream A is held behind a ~1 ms spin kernel, then queues a Viterbi
call that sizes the context's Viterbi slots for 4 chunks.  Stream B waits for A's event (the
caller orders the two launches, as cpg.h asks) and queues a 43-chunk call on the same
context, whose host-side ws_get grows the slots while A's kernels have not even started.
The growth must wait for the device before freeing; A's path and scores must equal an
independent context's.  Every call goes through the C-ABI (libcpg.so).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DECODE = 1 << 20


def test_workspace_growth_while_another_stream_reads():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cpgisland_amd import Context, HmmModel
    from cpgisland_amd import device as D
    dev = torch.device("cuda:0")
    n1, n2 = 4 * DECODE, 43 * DECODE
    packed, _ = D.synth_host(20251016, 0, n2)
    dp = D.to_device(np.concatenate([packed, np.zeros(8, np.uint32)]), dev)
    m = HmmModel.initial()
    ref = Context(0)
    try:
        rso, rsc = D.viterbi(ref, m, dp, n1)
        torch.cuda.synchronize()
        ref.sync()
        want_sign, want_score = D.sign_to_numpy(rso, n1), rsc.cpu().numpy()
    finally:
        ref.close()
    ctx = Context(0)          # fresh: its slots are sized by the first call below
    try:
        sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
        so1 = torch.empty(D.words32(n1) + 4, dtype=torch.int32, device=dev)
        sc1 = torch.empty(4, dtype=torch.float64, device=dev)
        so2 = torch.empty(D.words32(n2) + 4, dtype=torch.int32, device=dev)
        sc2 = torch.empty(43, dtype=torch.float64, device=dev)
        torch.cuda.synchronize()
        with torch.cuda.stream(sa):
            torch.cuda._sleep(2_000_000)                   # A's Viterbi queued behind ~1 ms
            D.viterbi(ctx, m, dp, n1, sign_out=so1, score=sc1)
            ev = torch.cuda.Event()
            ev.record(sa)
        with torch.cuda.stream(sb):
            sb.wait_event(ev)
            D.viterbi(ctx, m, dp, n2, sign_out=so2, score=sc2)   # grows the slots now
        torch.cuda.synchronize()
        ctx.sync()
        assert np.array_equal(D.sign_to_numpy(so1, n1), want_sign)
        assert np.array_equal(sc1.cpu().numpy(), want_score)
        assert np.array_equal(D.sign_to_numpy(so2, n2)[:n1], want_sign)
    finally:
        ctx.close()


def test_reserve_chunk_covers_its_chunk_length():
    """ cpg_reserve_chunk sizes the workspace for ONE decode chunk length: after
    it, the training pass, the fused decode and the island call at that length over up to
    nbases bases allocate nothing (the context's workspace does not grow), and the reservation
    is smaller than cpg_reserve's, which covers every multiple of 256."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cpgisland_amd import Context, HmmModel
    from cpgisland_amd import device as D
    dev = torch.device("cuda:0")
    n = 43 * DECODE
    p, s = D.synth_host(20251016, 0, n)
    dp, ds = D.to_device(p, dev), D.to_device(s, dev)
    a, b = Context(0), Context(0)
    try:
        a.reserve(n, chunk_len=DECODE)
        b.reserve(n)
        wa = a.workspace_bytes()
        assert wa < b.workspace_bytes()
        m = HmmModel.initial()
        D.train_pass(a, m, dp, ds, n)
        so, sc, io, ic = D.decode(a, m, dp, n, DECODE)
        D.islands(a, dp, so, n, DECODE)
        torch.cuda.synchronize()
        a.sync()
        assert a.workspace_bytes() == wa
        so2, sc2, io2, ic2 = D.decode(b, m, dp, n, DECODE)
        torch.cuda.synchronize()
        b.sync()
        assert np.array_equal(D.islands_to_numpy(io, ic), D.islands_to_numpy(io2, ic2))
    finally:
        a.close()
        b.close()
