// k_count.hip — labelled int64 counts on gfx950.
//
// Training-side counterpart of the BW mapper stripes (init / transition / emission rows,
// CpGIslandFinder.java:200) computed from hard labels: state s_t = base_t + (sign_t?0:4).
// Streams 2-bit packed bases (16 B per lane = 64 bases) and sign bits (8 B per lane),
// builds per-lane dinucleotide bitmasks and counts them with v_bcnt (popcount+add), so a
// base costs a few VALU ops and no LDS traffic.  Sign classes ride a uniform fast path:
// inside an island or background run every transition is ++ or --, and only lane-blocks
// that straddle an island boundary take the general four-class path.
//
// Per-workgroup partial counts (and the init states of the chunks starting in the
// workgroup) are added to 72 global 64-bit accumulators (integer atomics: exact and
// order-independent, one per counter per workgroup); the last workgroup to finish derives the
// emission/dinucleotide/mono counts from the transition + init counts (exact integer
// identities) and re-zeroes the accumulators.  One launch per call (a separate one-workgroup
// finalize launch for the streamed genome, which accumulates every window first).

#include "cpg_internal.h"

namespace cpg {
namespace {

constexpr int kCountThreads = 256;
constexpr int kRaw = 72;        // tot[16] pp[16] pm[16] mp[16] init[8]
// workgroups add into kCntRep replicated accumulator sets (blockIdx % kCntRep) so that the
// workgroups do not serialise on 72 device-scope atomic addresses; the finalize sums them
#ifndef CNT_REP
#define CNT_REP 16
#endif
#ifndef CNT_GRID
#define CNT_GRID 512   // measured: 2048 / 1024 / 512 workgroups 19.0 / 14.6 / 12.9 us at 46 Mbp
#endif
constexpr int kCntRep = CNT_REP;
constexpr uint32_t M55 = 0x55555555u;

struct Masks {
    uint32_t e[4];   // bit 2k set iff base k == b
};

__device__ __forceinline__ Masks base_masks(uint32_t w) {
    uint32_t h = w >> 1;
    Masks m;
    m.e[0] = ~(w | h) & M55;
    m.e[1] = w & ~h & M55;
    m.e[2] = h & ~w & M55;
    m.e[3] = w & h & M55;
    return m;
}

// spread 16 bits (bit k) to even bit positions (bit 2k)
__device__ __forceinline__ uint32_t spread16(uint32_t x) {
    x &= 0xFFFFu;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x;
}

__device__ void final_counts(const uint64_t* raw, int t, int64_t* __restrict__ out);
template <bool kAgent>
__device__ void finalize(unsigned long long* gacc, uint64_t* raw, int64_t* out);

// done != nullptr: the last workgroup to finish also finalizes (one launch per call)
__global__ __launch_bounds__(kCountThreads) void k_count_main(
    const uint4* __restrict__ packed4, const uint2* __restrict__ sign2,
    const uint32_t* __restrict__ packed, const uint32_t* __restrict__ sign, int64_t nblk,
    int64_t blk_per_chunk, unsigned long long* __restrict__ gacc, unsigned int* done,
    int64_t* __restrict__ out) {
    uint32_t tot[16], pp[16], pm[16], mp[16];
#pragma unroll
    for (int d = 0; d < 16; ++d) tot[d] = pp[d] = pm[d] = mp[d] = 0u;
    __shared__ uint32_t sinit[8];   // states of the chunks' first bases (rare: LDS atomics)
    if (threadIdx.x < 8) sinit[threadIdx.x] = 0u;
    __syncthreads();

    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nblk; i += stride) {
        const uint4 w = packed4[i];
        const uint2 s = sign2[i];
        const bool cstart = (i % blk_per_chunk) == 0;
        uint32_t wprev = 0, sprev = 0;
        if (cstart) atomicAdd(&sinit[(w.x & 3u) + ((s.x & 1u) ? 0u : 4u)], 1u);
        if (!cstart) {
            wprev = packed[4 * i - 1];
            sprev = sign[2 * i - 1] >> 31;
        }
        const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
        Masks cur[4], prv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) cur[k] = base_masks(ww[k]);
        {
            uint32_t wp = __builtin_amdgcn_alignbit(ww[0], wprev, 30);
            prv[0] = base_masks(wp);
        }
#pragma unroll
        for (int k = 1; k < 4; ++k)
#pragma unroll
            for (int b = 0; b < 4; ++b)
                prv[k].e[b] = __builtin_amdgcn_alignbit(cur[k].e[b], cur[k - 1].e[b], 30);
        if (cstart) {
#pragma unroll
            for (int b = 0; b < 4; ++b) prv[0].e[b] &= ~1u;   // no transition into pos 0
        }
        const bool all_minus = (s.x == 0u) && (s.y == 0u) && (cstart || sprev == 0u);
        const bool all_plus = (s.x == ~0u) && (s.y == ~0u) && (cstart || sprev == 1u);
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int p = 0; p < 4; ++p)
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    tot[p * 4 + b] += __popc(prv[k].e[p] & cur[k].e[b]);
        if (!all_minus) {
            if (all_plus) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
#pragma unroll
                    for (int p = 0; p < 4; ++p)
#pragma unroll
                        for (int b = 0; b < 4; ++b)
                            pp[p * 4 + b] += __popc(prv[k].e[p] & cur[k].e[b]);
            } else {
                // general path: per word spread sign masks
                const uint32_t sw[4] = {s.x & 0xFFFFu, s.x >> 16, s.y & 0xFFFFu, s.y >> 16};
                uint32_t sprv = sprev;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    uint32_t S = spread16(sw[k]);
                    uint32_t Sp = (S << 2) | (sprv & 1u);
                    sprv = sw[k] >> 15;
                    uint32_t SS = Sp & S, SN = Sp & ~S, NS = ~Sp & S;
#pragma unroll
                    for (int p = 0; p < 4; ++p)
#pragma unroll
                        for (int b = 0; b < 4; ++b) {
                            uint32_t D = prv[k].e[p] & cur[k].e[b];
                            pp[p * 4 + b] += __popc(D & SS);
                            pm[p * 4 + b] += __popc(D & SN);
                            mp[p * 4 + b] += __popc(D & NS);
                        }
                }
            }
        }
    }

    // wave reduction by recursive halving: after 6 levels lane L holds the wave sum of
    // counter L (63 shuffles instead of 64 x 6)
    uint32_t v[64];
#pragma unroll
    for (int d = 0; d < 16; ++d) {
        v[d] = tot[d];
        v[16 + d] = pp[d];
        v[32 + d] = pm[d];
        v[48 + d] = mp[d];
    }
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int lvl = 0; lvl < 6; ++lvl) {
        const int o = 32 >> lvl;
        const bool up = (lane & o) != 0;
#pragma unroll
        for (int i = 0; i < o; ++i) {
            uint32_t send = up ? v[i] : v[i + o];
            uint32_t keep = up ? v[i + o] : v[i];
            v[i] = keep + (uint32_t)__shfl_xor((int)send, o);
        }
    }
    __shared__ uint32_t wsum[kCountThreads / 64][64];
    wsum[threadIdx.x >> 6][lane] = v[0];
    __syncthreads();
    if (threadIdx.x < kRaw) {
        uint64_t acc = 0;
        if (threadIdx.x < 64) {
#pragma unroll
            for (int w = 0; w < kCountThreads / 64; ++w) acc += wsum[w][threadIdx.x];
        } else {
            acc = sinit[threadIdx.x - 64];
        }
#ifdef CNT_NOATOM   // measurement only: wrong counts
        if (acc == 0x123456789ull)
#else
        if (acc)
#endif
            atomicAdd(gacc + (blockIdx.x % kCntRep) * kRaw + threadIdx.x,
                           (unsigned long long)acc);
    }
    __shared__ int s_last;
    __shared__ uint64_t raw[kRaw];
    if (done && last_workgroup(done, &s_last)) {
        finalize<true>(gacc, raw, out);
        reset_done(done);
    }
}

// the cpg_counts_i64 assembly from the 72 accumulators (replicas summed), which it re-zeroes;
// kAgent: the accumulators were written by workgroups of the same launch
template <bool kAgent>
__device__ void finalize(unsigned long long* gacc, uint64_t* raw, int64_t* out) {
    const int t = threadIdx.x;
    if (t < kRaw) {
        uint64_t v = 0;
        for (int r = 0; r < kCntRep; ++r)
            v += kAgent ? load_agent(gacc + r * kRaw + t) : gacc[r * kRaw + t];
        raw[t] = v;
    }
    __syncthreads();
    for (int i = t; i < kRaw * kCntRep; i += blockDim.x) gacc[i] = 0ull;
    for (int i = t; i < 124; i += blockDim.x) final_counts(raw, i, out);
}

// One workgroup: the cpg_counts_i64 assembly from the 72 accumulators, which it re-zeroes.
__global__ __launch_bounds__(128) void k_count_final(unsigned long long* __restrict__ gacc,
                                                     int64_t* __restrict__ out) {
    __shared__ uint64_t raw[kRaw];
    finalize<false>(gacc, raw, out);
}

// cpg_counts_i64 from the 72 raw sums (tot | pp | pm | mp | init); thread t < 124
__device__ void final_counts(const uint64_t* raw, int t, int64_t* __restrict__ out) {
    // cpg_counts_i64 layout: init[8] trans[8][8] emit[8][4] dinuc[4][4] mono[4]; one
    // output word per thread
    int64_t v = 0;
    if (t < 8) {
        v = (int64_t)raw[64 + t];
    } else if (t < 72) {
        const int i = (t - 8) >> 3, j = (t - 8) & 7;      // trans[i][j]
        const int d = (i & 3) * 4 + (j & 3), si = i >> 2, sj = j >> 2;
        const int64_t tt = (int64_t)raw[d], ppv = (int64_t)raw[16 + d],
                      pmv = (int64_t)raw[32 + d], mpv = (int64_t)raw[48 + d];
        v = si == 0 ? (sj == 0 ? ppv : pmv) : (sj == 0 ? mpv : tt - ppv - pmv - mpv);
    } else if (t < 104) {
        const int s = (t - 72) >> 2, k = (t - 72) & 3;     // emit[s][k]
        if (k == (s & 3)) {
            v = (int64_t)raw[64 + s];
            for (int r = 0; r < 8; ++r) {
                const int d = (r & 3) * 4 + (s & 3), si = r >> 2, sj = s >> 2;
                const int64_t tt = (int64_t)raw[d], ppv = (int64_t)raw[16 + d],
                              pmv = (int64_t)raw[32 + d], mpv = (int64_t)raw[48 + d];
                v += si == 0 ? (sj == 0 ? ppv : pmv) : (sj == 0 ? mpv : tt - ppv - pmv - mpv);
            }
        }
    } else if (t < 120) {
        const int p = (t - 104) >> 2, b = (t - 104) & 3;    // dinuc[p][b]
        v = (int64_t)raw[p * 4 + b];
    } else {
        const int b = t - 120;                               // mono[b] = sum_p dinuc + inits
        // every base at a chunk position > 0 is the cur base of one transition; position 0
        // is counted by init
        for (int p = 0; p < 4; ++p) v += (int64_t)raw[p * 4 + b];
        v += (int64_t)raw[64 + b] + (int64_t)raw[64 + b + 4];
    }
    out[t] = v;
}

}  // namespace

hipError_t launch_count(const uint32_t* packed, const uint32_t* sign, int64_t nchunks,
                        int64_t chunk_len, uint64_t* ws, int64_t* out, hipStream_t s, int parts) {
    const int64_t nblk = nchunks * chunk_len / 64;
    if (nblk <= 0 && parts == PART_ALL) return hipMemsetAsync(out, 0, 124 * sizeof(int64_t), s);
    if ((parts & PART_ACC) && nblk > 0) {
        int grid = CNT_GRID;
        if ((int64_t)grid * kCountThreads > nblk)
            grid = (int)((nblk + kCountThreads - 1) / kCountThreads);
        // the whole call in one launch: its last workgroup finalizes
        unsigned int* done = parts == PART_ALL ? (unsigned int*)(ws + kRaw * kCntRep) : nullptr;
        hipLaunchKernelGGL(k_count_main, dim3(grid), dim3(kCountThreads), 0, s,
                           (const uint4*)packed, (const uint2*)sign, packed, sign, nblk,
                           chunk_len / 64, (unsigned long long*)ws, done, out);
        if (done) return hipGetLastError();
    }
    if (parts & PART_FINAL)
        hipLaunchKernelGGL(k_count_final, dim3(1), dim3(128), 0, s, (unsigned long long*)ws, out);
    return hipGetLastError();
}

// + the done counters
size_t count_ws_bytes(int64_t) { return (size_t)kRaw * 8 * kCntRep + 4 * kDoneWords; }

}  // namespace cpg
