"""Subprocess body of tests/test_gpu_fuse57.py: the fused forward + traceback Viterbi kernel
(k_vit_fwdtrace, selected once per process by CPG_VIT_FUSE57=1 before the library's first
decode) against the oracle's decode loop (:256-340) and bitwise against the single calls."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cpgisland_amd import Context, HmmModel  # noqa: E402
from cpgisland_amd import device as D  # noqa: E402
from oracle import coracle as co  # noqa: E402
from oracle import pyref as pr  # noqa: E402

assert os.environ.get("CPG_VIT_FUSE57") == "1"
dev = torch.device("cuda:0")
ctx = Context(0)
C = 1 << 20   # the segment path (16 segments per chunk) with the fused island scan
pi, a, b = co.model_split(co.initial_model())
a2 = a.copy()
a2[:4, 4:] *= 40.0
a2[4:, :4] *= 40.0
a2 /= a2.sum(axis=1, keepdims=True)
models = {"initial": co.initial_model(), "switchy": co.model_flat(pi, a2, b)}
for seed, nch in [(5, 3), (6, 2)]:
    N = nch * C + 777
    packed, _ = D.synth_host(seed, 0, N)
    obs = pr.unpack(packed, N)
    dp = D.to_device(np.concatenate([packed.astype(np.uint32), np.zeros(8, np.uint32)]), dev)
    for name, m in models.items():
        hm = HmmModel.from_struct(m)
        so, sc, out, cnt = D.decode(ctx, hm, dp, N, C, cap=1 << 18)
        torch.cuda.synchronize()
        ctx.sync()
        states, isl_ref, score = co.decode_chunks(m, obs, C)
        nd = len(states)
        sg = D.sign_to_numpy(so, N)
        assert np.array_equal(sg[:nd], (states < 4).astype(np.uint8)), (seed, name, "path")
        assert not sg[nd:].any(), (seed, name, "tail")
        assert np.array_equal(sc.cpu().numpy()[:nch], score), (seed, name, "score")
        assert np.array_equal(D.islands_to_numpy(out, cnt), isl_ref), (seed, name, "islands")
        # bitwise the single Viterbi call (the two-kernel K5 / K7 path)
        so3, sc3 = D.viterbi(ctx, hm, dp, N, C)
        torch.cuda.synchronize()
        ctx.sync()
        w = (N + 31) // 32
        assert np.array_equal(so.cpu().numpy()[:w], so3.cpu().numpy()[:w]), (seed, name, "single")
        assert np.array_equal(sc.cpu().numpy()[:nch], sc3.cpu().numpy()[:nch]), (seed, name)
ctx.close()
print("fuse57 ok")
