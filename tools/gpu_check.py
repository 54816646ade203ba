"""Quick GPU correctness probe against the C oracle (development tool)."""
import sys, time
import numpy as np
sys.path.insert(0, "/root/repo")
import torch
from cpgisland_amd import HmmModel, Context, HmmEvaluator
from cpgisland_amd import device as D
from oracle import coracle as co, pyref as pr

dev = torch.device("cuda:0")
ctx = Context(0)
model = HmmModel.initial()
m = model.to_struct()

def unpack(p, n): return pr.unpack(p.view(np.uint32), n)

# 1) small decode_states vs oracle viterbi8
rng = np.random.default_rng(5)
for T in [1, 2, 3, 17, 255, 256, 257, 1000, 4096, 70000]:
    obs = rng.integers(0, 4, T).astype(np.int32)
    st = HmmEvaluator.decode(model, obs, ctx=ctx)
    ref, _ = co.viterbi8(m, obs.astype(np.uint8))
    print("decode_states T=%d match=%s" % (T, np.array_equal(st, ref)), flush=True)

# 2) synthetic genome: 4 decode chunks
N = 4 * 1048576 + 12345
packed, sign = D.synth_host(20251015, 0, N)
obs = unpack(packed, N)
sg = pr.unpack_bits(sign, N)
dp = D.to_device(packed, dev); ds = D.to_device(sign, dev)
t0 = time.time()
so, sc = D.viterbi(ctx, model, dp, N)
torch.cuda.synchronize(); ctx.sync()
print("viterbi gpu %.3fs" % (time.time() - t0))
gsign = D.sign_to_numpy(so, N)
t0 = time.time()
states, isl, scores = co.decode_chunks(m, obs, 1048576)
print("oracle %.3fs" % (time.time() - t0))
nd = len(states)
print("viterbi path match:", np.array_equal(gsign[:nd], (states < 4).astype(np.uint8)),
      "mismatches", int(np.sum(gsign[:nd] != (states < 4))))
print("scores", sc.cpu().numpy()[:4], scores)
out, cnt = D.islands(ctx, dp, so, N)
gi = D.islands_to_numpy(out, cnt)
print("islands gpu", len(gi), "oracle", len(isl), "equal", len(gi) == len(isl) and all(
    tuple(a) == tuple(b) for a, b in zip(gi, isl)))
# 3) labelled counts
cnt = D.count_labelled(ctx, dp, ds, N, 65536)
ref = co.count_labelled(obs, sg, 65536)
print("counts match:", np.array_equal(cnt.cpu().numpy(), ref))
# 4) estep
e = D.bw_estep(ctx, model, dp, N, 65536)
torch.cuda.synchronize()
eref = co.estep(m, obs, 65536)
g = e.cpu().numpy()
rel = np.abs(g - eref) / np.maximum(np.abs(eref), 1e-300)
print("estep max rel err", rel[np.abs(eref) > 0].max(), "loglik", g[-1], eref[-1])
ctx.sync()
print("OK")
