"""Two pipeline lanes (bench.py's default since round 6): consecutive steps on their own
contexts and streams, so two decodes and two training passes of the same genome run on the GPU
at once.  Every lane's outputs must equal one context's serial results, bitwise — the decode
kernels wait on no other workgroup and share nothing between contexts.  Every call goes
through the C-ABI (libcpg.so)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DECODE = 1 << 20
TRAIN = 65536


def test_two_lanes_concurrent_equal_serial():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cpgisland_amd import Context, HmmModel
    from cpgisland_amd import device as D
    dev = torch.device("cuda:0")
    n = 24 * DECODE
    packed, sign = D.synth_host(20251016, 0, n)
    dp = D.to_device(np.concatenate([packed, np.zeros(8, np.uint32)]), dev)
    ds = D.to_device(np.concatenate([sign, np.zeros(8, np.uint32)]), dev)
    m0 = HmmModel.initial()
    ref = Context(0)
    try:
        est0, cnt0 = D.train_pass(ref, m0, dp, ds, n, TRAIN)
        so0, sc0, io0, ic0 = D.decode(ref, m0, dp, n, DECODE)
        torch.cuda.synchronize()
        ref.sync()
        want = (est0.cpu().numpy(), cnt0.cpu().numpy(), D.sign_to_numpy(so0, n),
                sc0.cpu().numpy(), D.islands_to_numpy(io0, ic0))
    finally:
        ref.close()
    lanes = [Context(0), Context(0)]
    try:
        for cx in lanes:
            cx.reserve(n)
        outs = []
        s_dec = [torch.cuda.Stream(priority=-1), torch.cuda.Stream(priority=-1)]
        s_tr = [torch.cuda.Stream(), torch.cuda.Stream()]
        torch.cuda.synchronize()
        for step in range(6):   # three steps per lane, nothing joined between them
            k = step % 2
            with torch.cuda.stream(s_dec[k]):
                d = D.decode(lanes[k], m0, dp, n, DECODE)
            with torch.cuda.stream(s_tr[k]):
                t = D.train_pass(lanes[k], m0, dp, ds, n, TRAIN)
            outs.append((t, d))
        torch.cuda.synchronize()
        for cx in lanes:
            cx.sync()
        for (est, cnt), (so, sc, io, ic) in outs:
            assert np.array_equal(est.cpu().numpy(), want[0])
            assert np.array_equal(cnt.cpu().numpy(), want[1])
            assert np.array_equal(D.sign_to_numpy(so, n), want[2])
            assert np.array_equal(sc.cpu().numpy(), want[3])
            assert np.array_equal(D.islands_to_numpy(io, ic), want[4])
    finally:
        for cx in lanes:
            cx.close()
