// k_vit_general.hip — HmmEvaluator.decode(model, obs, true) (CpGIslandFinder.java:260) for ANY
// model the reference accepts: zero transition probabilities (log 0 = -inf, legal in Mahout's
// loop), emission rows that are not deterministic, pi with zeros.  The exact parallel scan of
// k_viterbi.hip needs the deterministic emission matrix (2 live states per position) and
// finite log constants; this path runs Mahout's 8-state recurrence itself:
//
//   delta_0(i) = log(pi_i * b_i(o_0))
//   delta_t(i) = max_j [delta_{t-1}(j) + log a_ji] + log b_i(o_t)   (candidate j = 0 first,
//                strict '>' : the lowest j wins ties)
//   final: argmax from -inf with strict '>' (state 0 when every delta is -inf), backtrack phi
//
// in IEEE fp64 with the same operations in the same order (no contraction: -ffp-contract=off),
// with the log constants computed once on the host by the C library (shared with the oracle).
// Chunks are independent (:256-260), so the parallelism is across chunks: a wave decodes 8
// chunks, lane 8g + i holding delta(i) of chunk g; the 8 deltas of the previous step come from
// the lane group by shuffles.  The backpointers of a step are 3 wave ballots (bit b of every
// lane's argmax) = 24 B per step per wave; the traceback walks them one chunk per wave in
// batches of 64 steps (scalar walk, lane-distributed state registers, coalesced byte stores).
// Throughput is bounded by the step's dependent shuffle + compare chain (~1 Gbase/s): the
// correctness path for models outside the fast path's contract, not the benchmark path.

#include "cpg_internal.h"

namespace cpg {
namespace {

constexpr int kGL = 64;   // lanes per workgroup (one wave): 8 chunks x 8 states

__global__ __launch_bounds__(kGL) void k_vitg_forward(GenConsts gc, const uint32_t* __restrict__ packed,
                                                       int64_t nchunks, int64_t C,
                                                       unsigned long long* __restrict__ rec,
                                                       double* __restrict__ score,
                                                       uint8_t* __restrict__ last) {
    const int lane = threadIdx.x, g = lane >> 3, i = lane & 7;
    const int64_t c = (int64_t)blockIdx.x * 8 + g;
    const bool live = c < nchunks;
    const uint32_t* pk = packed + (live ? c : 0) * (C / 16);
    double Lc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) Lc[j] = gc.L[j][i];   // log a[j][i]: the lane's column
    const double lb0 = gc.LB[i][0], lb1 = gc.LB[i][1], lb2 = gc.LB[i][2], lb3 = gc.LB[i][3];
    uint32_t w = pk[0];
    double d = gc.LP[i][w & 3u];                       // log(pi_i * b_i(o_0))
    unsigned long long* r = rec + (int64_t)blockIdx.x * (C - 1) * 3;
    for (int64_t t = 1; t < C; ++t) {
        if ((t & 15) == 0) w = pk[t >> 4];
        const uint32_t o = (w >> (2 * (t & 15))) & 3u;
        double dj[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) dj[j] = __shfl(d, j, 8);
        double mp = dj[0] + Lc[0];
        int ms = 0;
#pragma unroll
        for (int j = 1; j < 8; ++j) {
            const double p = dj[j] + Lc[j];
            if (p > mp) {
                mp = p;
                ms = j;
            }
        }
        d = mp + (o == 0 ? lb0 : o == 1 ? lb1 : o == 2 ? lb2 : lb3);
        const unsigned long long b0 = __ballot(ms & 1), b1 = __ballot(ms & 2),
                                 b2 = __ballot(ms & 4);
        if (lane < 3) r[(t - 1) * 3 + lane] = lane == 0 ? b0 : lane == 1 ? b1 : b2;
    }
    double dj[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) dj[j] = __shfl(d, j, 8);
    if (live && i == 0) {
        double best = -INFINITY;
        int s = 0;                                     // Java int[] starts zeroed
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (dj[j] > best) {
                best = dj[j];
                s = j;
            }
        if (score) score[c] = best;
        last[c] = (uint8_t)s;
    }
}

// one wave per chunk: path[C-1] = last, path[t] = phi_t(path[t+1]) for t = C-2 .. 0
__global__ __launch_bounds__(kGL) void k_vitg_trace(const unsigned long long* __restrict__ rec,
                                                     int64_t C, const uint8_t* __restrict__ last,
                                                     uint8_t* __restrict__ states) {
    const int64_t c = blockIdx.x;
    const int lane = threadIdx.x;
    const int sh = 8 * (int)(c & 7);
    const unsigned long long* r = rec + (c >> 3) * (C - 1) * 3;
    uint8_t* so = states + c * C;
    int s = last[c];
    if (lane == 0) so[C - 1] = (uint8_t)s;
    for (int64_t hi = C - 2; hi >= 0; hi -= kGL) {
        const int64_t lo = hi - (kGL - 1) > 0 ? hi - (kGL - 1) : 0;
        const int n = (int)(hi - lo) + 1;
        unsigned long long m0 = 0, m1 = 0, m2 = 0;
        if (lane < n) {
            const unsigned long long* q = r + (lo + lane) * 3;
            m0 = q[0];
            m1 = q[1];
            m2 = q[2];
        }
        int st = 0;
        for (int k = n - 1; k >= 0; --k) {
            const unsigned long long a0 = __shfl(m0, k), a1 = __shfl(m1, k), a2 = __shfl(m2, k);
            const int b = sh + s;
            s = (int)((a0 >> b) & 1ull) | ((int)((a1 >> b) & 1ull) << 1) |
                ((int)((a2 >> b) & 1ull) << 2);
            if (lane == k) st = s;
        }
        if (lane < n) so[lo + lane] = (uint8_t)st;
    }
}

// states -> sign bits (state < 4) and "state packed" words (state & 3, the packed layout): the
// island scan over them is the :262-339 loop over the states themselves (it reads only state
// values: C+ = 1, G+ = 2, '+' = 0..3).  One lane per 32 positions of the whole chunks; with
// check != nullptr a position whose state is not its base's (state & 3 != base) sets
// ST_GEN_NOT_SIGN (the path is not representable as sign bits).
__global__ __launch_bounds__(256) void k_vitg_pack(const uint8_t* __restrict__ states, int64_t n,
                                                    const uint32_t* __restrict__ packed,
                                                    uint32_t* __restrict__ sign_out,
                                                    uint32_t* __restrict__ spk,
                                                    uint32_t* __restrict__ status) {
    const int64_t wi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // sign word
    if (wi * 32 >= n) return;
    uint32_t sg = 0u, p0 = 0u, p1 = 0u;
    for (int k = 0; k < 32; ++k) {
        const int64_t p = wi * 32 + k;
        if (p >= n) break;
        const uint32_t s = states[p];
        sg |= (s < 4u ? 1u : 0u) << k;
        if (k < 16) p0 |= (s & 3u) << (2 * k);
        else p1 |= (s & 3u) << (2 * (k - 16));
    }
    if (sign_out) sign_out[wi] = sg;
    if (spk) {
        spk[2 * wi] = p0;
        if (wi * 32 + 16 < n) spk[2 * wi + 1] = p1;
    }
    if (status && packed) {
        const int64_t m = n - wi * 32 < 32 ? n - wi * 32 : 32;
        const uint32_t b0 = packed[2 * wi], b1 = m > 16 ? packed[2 * wi + 1] : 0u;
        const uint32_t mk0 = m >= 16 ? 0xFFFFFFFFu : ((1u << (2 * m)) - 1u);
        const uint32_t mk1 = m >= 32 ? 0xFFFFFFFFu : m > 16 ? ((1u << (2 * (m - 16))) - 1u) : 0u;
        if (((b0 ^ p0) & mk0) | ((b1 ^ p1) & mk1)) atomicOr(status, ST_GEN_NOT_SIGN);
    }
}

}  // namespace

size_t vitg_ws_bytes(int64_t nchunks, int64_t C) {
    const int64_t nw = (nchunks + 7) / 8;
    const size_t rec = (size_t)nw * (size_t)(C > 1 ? C - 1 : 1) * 24;
    const size_t st = (size_t)nchunks * C + 64;
    const size_t words = (size_t)((nchunks * C + 31) / 32) * 12 + 64;   // sign + state-packed
    return rec + st + words + (size_t)nchunks + 256;
}

hipError_t launch_vitg(const GenConsts& gc, const uint32_t* packed, int64_t nchunks, int64_t C,
                       void* ws, size_t ws_bytes, uint8_t* states_out, double* score,
                       uint32_t* sign_out, uint32_t** spk_out, uint32_t* status,
                       bool check_sign, hipStream_t s) {
    if (nchunks <= 0) return hipSuccess;
    if (vitg_ws_bytes(nchunks, C) > ws_bytes || (nchunks > 1 && C % 16)) return hipErrorInvalidValue;
    const int64_t nw = (nchunks + 7) / 8;
    unsigned char* p = static_cast<unsigned char*>(ws);
    auto* rec = reinterpret_cast<unsigned long long*>(p);
    p += (size_t)nw * (size_t)(C > 1 ? C - 1 : 1) * 24;
    uint8_t* st = states_out ? states_out : p;
    p += (size_t)nchunks * C + 64;
    p = reinterpret_cast<unsigned char*>((reinterpret_cast<uintptr_t>(p) + 255) & ~uintptr_t(255));
    auto* spk = reinterpret_cast<uint32_t*>(p);
    p += (size_t)((nchunks * C + 31) / 32) * 8 + 64;
    uint8_t* last = p;
    hipLaunchKernelGGL(k_vitg_forward, dim3((unsigned)nw), dim3(kGL), 0, s, gc, packed, nchunks, C,
                       rec, score, last);
    hipLaunchKernelGGL(k_vitg_trace, dim3((unsigned)nchunks), dim3(kGL), 0, s, rec, C, last, st);
    const int64_t n = nchunks * C, nwords = (n + 31) / 32;
    if (sign_out || spk_out || check_sign)
        hipLaunchKernelGGL(k_vitg_pack, dim3((unsigned)((nwords + 255) / 256)), dim3(256), 0, s, st,
                           n, packed, sign_out, spk_out ? spk : nullptr,
                           check_sign ? status : nullptr);
    if (spk_out) *spk_out = spk;
    return hipGetLastError();
}

}  // namespace cpg
