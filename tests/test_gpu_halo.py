"""Unaligned shards on the GPU (cpgisland_amd/dist.py HaloShardRunner): a genome split at
multiples of 64 bases, not at chunk boundaries, over 3 emulated ranks on one device (each
rank's next-rank head handed over directly, as halo_exchange's all-gather delivers it).
Every chunk runs whole on the rank that holds its first base: labelled counts, island
records and decoded paths equal the unsharded run's bit for bit; the E-step sums to it
within rounding of the fp64 rank sum."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
TRAIN = 65536
DECODE = 1 << 20


def test_halo_shards_equal_unsharded(gpu_ctx):
    import torch
    from cpgisland_amd import HmmModel
    from cpgisland_amd import device as D
    from cpgisland_amd import dist as cd
    dev = torch.device("cuda:0")
    seed, N, world = 77, 5 * DECODE + 12345, 3
    m = HmmModel.initial()
    full_p, full_s = D.synth_host(seed, 0, N)
    fp, fs = D.to_device(full_p, dev), D.to_device(full_s, dev)
    ref_i = D.count_labelled(gpu_ctx, fp, fs, N).cpu().numpy()
    ref_e = D.bw_estep(gpu_ctx, m, fp, N).cpu().numpy()
    ref_sg, _ = D.viterbi(gpu_ctx, m, fp, N)
    out, cnt = D.islands(gpu_ctx, fp, ref_sg, N)
    ref_isl = D.islands_to_numpy(out, cnt)
    ref_bits = D.sign_to_numpy(ref_sg, N)
    spans = [cd.shard_bounds(N, world, r, align=cd.HALO_ALIGN) for r in range(world)]
    assert any(s % DECODE for s, _ in spans)
    tot_i = np.zeros_like(ref_i)
    tot_e = np.zeros_like(ref_e)
    isl, halos = [], []
    for r, (start, n) in enumerate(spans):
        p, s = D.synth_host(seed, start, n)          # the rank's own words
        heads = (None, None, 0)
        if r + 1 < world:                             # the next rank's first 2^20 bases
            s1, n1 = spans[r + 1]
            hp, hs = D.synth_host(seed, s1, min(n1, DECODE))
            hp = np.concatenate([hp, np.zeros(DECODE // 16, np.uint32)])[:DECODE // 16]
            hs = np.concatenate([hs, np.zeros(DECODE // 32, np.uint32)])[:DECODE // 32]
            heads = (D.to_device(hp, dev), D.to_device(hs, dev), n1)
        run = cd.HaloShardRunner(gpu_ctx, D.to_device(p, dev), D.to_device(s, dev), start, n,
                                 N, heads=heads)
        halos.append(run.plan.halo)
        tot_i += run.labelled_counts().cpu().numpy()
        tot_e += run.estep(m)
        sg, _, rec = run.decode(m)
        isl.append(rec)
        pl = run.plan
        nb = (pl.d1 - pl.d0) * DECODE
        assert np.array_equal(D.sign_to_numpy(sg, nb),
                              ref_bits[pl.d0 * DECODE:pl.d0 * DECODE + nb])
    assert any(h > 0 for h in halos)
    assert np.array_equal(tot_i, ref_i)
    nz = ref_e != 0
    assert np.max(np.abs(tot_e[nz] - ref_e[nz]) / np.abs(ref_e[nz])) < 1e-12
    assert np.array_equal(np.concatenate(isl), ref_isl)
