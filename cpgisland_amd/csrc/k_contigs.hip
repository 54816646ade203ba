// k_contigs.hip — ragged contig batches (BASELINE config C4: ~10M contigs of 150 bp - 50 kbp)
// on gfx950.  Every contig is an independent observation sequence, exactly as every whole
// chunk is in the reference (training :130-141 -> BW mapper :200; decode :256-260 ->
// HmmEvaluator.decode; islands :262-339 per chunk): the batch applies the reference's
// per-chunk semantics per contig.
//
// Layout: one packed buffer (16 bases / uint32); contig c occupies bases
// [offs[c], offs[c] + lens[c]) with offs[c] % 64 == 0, so each lane reads its contig with
// aligned 16-B loads (64 bases) and owns whole sign-bit words.  The wavefront schedule is the
// contig order sorted by decreasing length (cpg_contigs_order_d, a device radix sort): the 64
// lanes of a wave walk 64 contigs of nearly equal length in lockstep, so divergence at the
// ends costs little ("load-balanced per wavefront").  One lane = one contig:
//   * labelled counts : per 64-base block, dinucleotide x sign-class bit masks and popcounts
//                       (k_count's scheme), per-lane registers, wave butterfly, WG atomics;
//   * Viterbi         : the reference step (Mahout order, '>' tie-break, fp64) sequentially
//                       per lane — bit-exact by construction, no scan needed at this
//                       granularity — 2-bit backpointers to a scratch that mirrors the packed
//                       layout (its own 16 B per 64 bases), then the traceback in the same
//                       kernel -> sign bits at the contig's own bit offsets;
//   * E-step          : scaled forward pass with alpha checkpoints every 64 positions (scratch
//                       mirroring the packed layout), then backward per 64-block from its
//                       checkpoint with 16-position alpha windows in registers; pair
//                       posteriors in unsigned fixed point 2^-38 into per-wave replicated LDS
//                       bins (integer atomics: exact, order-independent), flushed to the same
//                       128-bit accumulators the chunk E-step uses (finalized by k_estep_final);
//   * islands         : the :262-339 scan per lane with 32-position word fast paths (whole
//                       background words skipped; whole island words by popcounts), two passes
//                       around a device scan so records come out in contig order.

#include <hipcub/hipcub.hpp>

#include <cmath>

#include "cpg_internal.h"

namespace cpg {
namespace {

constexpr int kCT = 256;                 // lanes per workgroup
constexpr int kCtgGrid = 2048;           // persistent grid (grid-stride over the schedule)
constexpr uint32_t M55 = 0x55555555u;

struct Ctg {
    const uint32_t* packed;
    const uint32_t* sign;
    const int64_t* offs;
    const int32_t* lens;
    const int32_t* order;   // schedule (NULL: identity)
    int64_t n;
    int64_t nbases;         // span of the packed buffer
    uint32_t* status;
};

// contig of schedule slot g, with the layout contract checked (status bit, skipped if broken)
__device__ __forceinline__ bool ctg_get(const Ctg& a, int64_t g, int64_t& c, int64_t& off,
                                        int64_t& len, int64_t maxlen) {
    c = a.order ? (int64_t)a.order[g] : g;
    off = a.offs[c];
    len = a.lens[c];
    if (off < 0 || (off & 63) || len < 1 || len > maxlen || off + len > a.nbases) {
        atomicOr(a.status, ST_CONTIG_LAYOUT);
        return false;
    }
    return true;
}

// ------------------------------------------------------------------ labelled counts
struct Masks {
    uint32_t e[4];   // bit 2k set iff base k == b
};
__device__ __forceinline__ Masks base_masks(uint32_t w) {
    const uint32_t h = w >> 1;
    Masks m;
    m.e[0] = ~(w | h) & M55;
    m.e[1] = w & ~h & M55;
    m.e[2] = h & ~w & M55;
    m.e[3] = w & h & M55;
    return m;
}
__device__ __forceinline__ uint32_t spread16(uint32_t x) {
    x &= 0xFFFFu;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x;
}
__device__ __forceinline__ uint32_t pext_even(uint32_t x) {   // bits 0,2,..,30 -> 0..15
    x &= M55;
    x = (x | (x >> 1)) & 0x33333333u;
    x = (x | (x >> 2)) & 0x0F0F0F0Fu;
    x = (x | (x >> 4)) & 0x00FF00FFu;
    x = (x | (x >> 8)) & 0x0000FFFFu;
    return x;
}

__global__ __launch_bounds__(kCT) void k_ctg_count(Ctg a, unsigned long long* __restrict__ gacc) {
    __shared__ unsigned long long wacc[72];
    if (threadIdx.x < 72) wacc[threadIdx.x] = 0ull;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const uint4* pk4 = reinterpret_cast<const uint4*>(a.packed);
    const uint2* sg2 = reinterpret_cast<const uint2*>(a.sign);
    const int64_t stride = (int64_t)gridDim.x * kCT;
    for (int64_t g0 = (int64_t)blockIdx.x * kCT; g0 < a.n; g0 += stride) {
        uint32_t tot[16], pp[16], pm[16], mp[16];
#pragma unroll
        for (int d = 0; d < 16; ++d) tot[d] = pp[d] = pm[d] = mp[d] = 0u;
        const int64_t g = g0 + threadIdx.x;
        int64_t c, off, len;
        if (g < a.n && ctg_get(a, g, c, off, len, 0x7FFFFFFF)) {
            const int64_t nblk = (len + 63) / 64;
            uint32_t wprev = 0u, sprev = 0u;
            for (int64_t i = 0; i < nblk; ++i) {
                const uint4 w = pk4[off / 64 + i];
                const uint2 s = sg2[off / 64 + i];
                if (i == 0)
                    atomicAdd(&wacc[64 + (w.x & 3u) + ((s.x & 1u) ? 0u : 4u)], 1ull);
                const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
                const uint32_t sw[4] = {s.x & 0xFFFFu, s.x >> 16, s.y & 0xFFFFu, s.y >> 16};
                const int64_t left = len - 64 * i;   // valid positions in this block
                Masks cur[4], prv[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) cur[k] = base_masks(ww[k]);
                prv[0] = base_masks(__builtin_amdgcn_alignbit(ww[0], wprev, 30));
#pragma unroll
                for (int k = 1; k < 4; ++k)
#pragma unroll
                    for (int b = 0; b < 4; ++b)
                        prv[k].e[b] = __builtin_amdgcn_alignbit(cur[k].e[b], cur[k - 1].e[b], 30);
                uint32_t sprv = sprev;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int64_t nv = left - 16 * k;
                    uint32_t vm = nv >= 16 ? 0xFFFFu : (nv <= 0 ? 0u : ((1u << nv) - 1u));
                    if (i == 0 && k == 0) vm &= ~1u;   // no transition into position 0
                    const uint32_t VM = spread16(vm);
                    const uint32_t S = spread16(sw[k]);
                    const uint32_t Sp = (S << 2) | (sprv & 1u);
                    sprv = sw[k] >> 15;
                    const uint32_t SS = Sp & S & VM, SN = Sp & ~S & VM, NS = ~Sp & S & VM;
#pragma unroll
                    for (int p = 0; p < 4; ++p)
#pragma unroll
                        for (int b = 0; b < 4; ++b) {
                            const uint32_t D = prv[k].e[p] & cur[k].e[b];
                            tot[p * 4 + b] += __popc(D & VM);
                            pp[p * 4 + b] += __popc(D & SS);
                            pm[p * 4 + b] += __popc(D & SN);
                            mp[p * 4 + b] += __popc(D & NS);
                        }
                }
                wprev = ww[3];
                sprev = s.y >> 31;
            }
        }
        // wave butterfly (recursive halving): lane L ends with the wave sum of counter L
        uint32_t v[64];
#pragma unroll
        for (int d = 0; d < 16; ++d) {
            v[d] = tot[d];
            v[16 + d] = pp[d];
            v[32 + d] = pm[d];
            v[48 + d] = mp[d];
        }
#pragma unroll
        for (int lvl = 0; lvl < 6; ++lvl) {
            const int o = 32 >> lvl;
            const bool up = (lane & o) != 0;
#pragma unroll
            for (int i = 0; i < o; ++i) {
                const uint32_t send = up ? v[i] : v[i + o];
                const uint32_t keep = up ? v[i + o] : v[i];
                v[i] = keep + (uint32_t)__shfl_xor((int)send, o);
            }
        }
        if (v[0]) atomicAdd(&wacc[lane], (unsigned long long)v[0]);
    }
    __syncthreads();
    if (threadIdx.x < 72 && wacc[threadIdx.x])
        atomicAdd(gacc + threadIdx.x, wacc[threadIdx.x]);
}

// ------------------------------------------------------------------ Viterbi
// The reference step (see k_viterbi.hip ref_step): target '+' sees predecessor '+' first,
// so '-' wins only when strictly greater; the survivor value is the max either way.
__global__ __launch_bounds__(kCT) void k_ctg_viterbi(Ctg a, VitConsts vc,
                                                     uint32_t* __restrict__ bp,
                                                     uint32_t* __restrict__ sign_out,
                                                     double* __restrict__ score) {
    __shared__ double4 L[16];
    __shared__ double lpi[8];
    if (threadIdx.x < 16)
        L[threadIdx.x] = make_double4(vc.L[threadIdx.x][0], vc.L[threadIdx.x][1],
                                      vc.L[threadIdx.x][2], vc.L[threadIdx.x][3]);
    if (threadIdx.x < 8) lpi[threadIdx.x] = vc.logpi[threadIdx.x];
    __syncthreads();
    const uint4* pk4 = reinterpret_cast<const uint4*>(a.packed);
    uint4* bp4 = reinterpret_cast<uint4*>(bp);
    uint2* so2 = reinterpret_cast<uint2*>(sign_out);
    const int64_t stride = (int64_t)gridDim.x * kCT;
    for (int64_t g = (int64_t)blockIdx.x * kCT + threadIdx.x; g < a.n; g += stride) {
        int64_t c, off, len;
        if (!ctg_get(a, g, c, off, len, 0x7FFFFFFF)) continue;
        const int64_t nblk = (len + 63) / 64, b0 = off / 64;
        double P = 0.0, M = 0.0;
        uint32_t prev = 0u;
        for (int64_t i = 0; i < nblk; ++i) {
            const uint4 w = pk4[b0 + i];
            const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
            uint32_t bw[4] = {0u, 0u, 0u, 0u};
            const int64_t left = len - 64 * i;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
#pragma unroll 4
                for (int j = 0; j < 16; ++j) {
                    const int p = 16 * k + j;
                    if (p >= left) break;
                    const uint32_t cur = (ww[k] >> (2 * j)) & 3u;
                    if (i == 0 && p == 0) {
                        P = lpi[cur];
                        M = lpi[cur + 4];
                    } else {
                        const double4 l = L[prev | (cur << 2)];
                        const double cpp = P + l.x, cmp = M + l.y, cpm = P + l.z, cmm = M + l.w;
                        bw[k] |= ((cmp > cpp) ? 1u : 0u) << (2 * j);
                        bw[k] |= ((cmm > cpm) ? 2u : 0u) << (2 * j);
                        P = fmax(cpp, cmp);
                        M = fmax(cpm, cmm);
                    }
                    prev = cur;
                }
            }
            bp4[b0 + i] = make_uint4(bw[0], bw[1], bw[2], bw[3]);
        }
        // final argmax (Mahout: states 0..7 in order, strict '>': '-' only if greater)
        uint32_t s = (M > P) ? 0u : 1u;   // 1 = '+'
        if (score) score[c] = fmax(P, M);
        // traceback: state at t-1 = backpointer of the state at t
        for (int64_t i = nblk - 1; i >= 0; --i) {
            const uint4 q = bp4[b0 + i];
            const uint32_t qq[4] = {q.x, q.y, q.z, q.w};
            uint32_t out[2] = {0u, 0u};
            const int64_t left = len - 64 * i;
#pragma unroll
            for (int k = 3; k >= 0; --k) {
#pragma unroll 4
                for (int j = 15; j >= 0; --j) {
                    const int p = 16 * k + j;
                    if (p >= left) continue;
                    out[k >> 1] |= s << (p & 31);
                    const uint32_t b = (qq[k] >> (2 * j + (s ? 0 : 1))) & 1u;   // 1: pred '-'
                    s = b ? 0u : 1u;
                }
            }
            so2[b0 + i] = make_uint2(out[0], out[1]);
        }
    }
}

// ------------------------------------------------------------------ E-step
constexpr double kFixC = 274877906944.0;            // 2^38 (contig bins; see header)
constexpr double kMagic = 6755399441055744.0;       // 1.5 * 2^52
// xi bins: 64 rows (k * 16 + d) x 16 lane columns (column = lane % 16): the 16 lanes of an
// LDS 64-bit pass hit 16 columns = 32 distinct banks whatever their classes (no conflicts,
// no same-address collisions); a column sums <= kCT / 16 lanes' contigs of <= 2^20 bases
// in 2^-38 units: below 2^62 for kCT <= 256
constexpr int kLogFix = 24;
__device__ __forceinline__ unsigned long long to_fixed_scaled(double y) {
    return (unsigned long long)__double_as_longlong(y + kMagic) -
           (unsigned long long)__double_as_longlong(kMagic);
}
__device__ __forceinline__ double rcp_nr(double z) {
    double r = __builtin_amdgcn_rcp(z);
    double e = fma(-z, r, 1.0);
    r = fma(r, e, r);
    e = fma(-z, r, 1.0);
    return fma(r, e, r);
}
__device__ __forceinline__ int vnorm(double& x, double& y) {
    const double mx = fmax(x, y);
    int k = 0;
    if (mx > 0.0) {
        k = ilogb(mx);
        x = ldexp(x, -k);
        y = ldexp(y, -k);
    }
    return k;
}
// a 128-bit addend (lo, hi) into the E-step's split accumulators (acc_split_add,
// cpg_internal.h; finalized by k_estep_final)
__device__ __forceinline__ void acc128_add2(unsigned long long* lohi, unsigned long long lo,
                                            unsigned long long hi) {
    acc_split_add(lohi, lo, hi);
}

constexpr int kCtgEstWaves = 3;   // min waves per SIMD (VGPR budget 512 / this; 2..4 measured)
__global__ __launch_bounds__(kCT, kCtgEstWaves) void k_ctg_estep(Ctg a, cpg_model model,
                                                   double2* __restrict__ ck,
                                                   unsigned long long* __restrict__ acc) {
    __shared__ double2 TA[16], TB[16];   // rows of M_d: (M(+,+), M(+,-)), (M(-,+), M(-,-))
    __shared__ unsigned long long bins[64 * 16];
    static_assert(kCT <= 256, "bin column capacity");
    __shared__ unsigned long long sinit[8];
    __shared__ long long sll;
    __shared__ double2 sent[3][kCT];     // alpha entering mini-blocks 1..3, per lane
    const int t = threadIdx.x, lane = t & 63;
    if (t < 16) {
        const int p = t & 3, b = t >> 2;
        TA[t] = make_double2(model.a[p][b], model.a[p][b + 4]);
        TB[t] = make_double2(model.a[p + 4][b], model.a[p + 4][b + 4]);
    }
    const uint4* pk4 = reinterpret_cast<const uint4*>(a.packed);
    unsigned long long* wb = bins + (lane & 15);
    const int64_t stride = (int64_t)gridDim.x * kCT;
    for (int64_t g0 = (int64_t)blockIdx.x * kCT; g0 < a.n; g0 += stride) {
        for (int i = t; i < 64 * 16; i += kCT) bins[i] = 0ull;
        if (t < 8) sinit[t] = 0ull;
        if (t == 0) sll = 0;
        __syncthreads();
        const int64_t g = g0 + t;
        int64_t c, off, len;
        if (g < a.n && ctg_get(a, g, c, off, len, 1 << 20)) {
            const int64_t nblk = (len + 63) / 64, b0 = off / 64;
            const uint32_t o0 = a.packed[off / 16] & 3u;
            // forward: alpha with power-of-two rescaling, checkpoints at every block start
            double aP = model.pi[o0], aM = model.pi[o0 + 4];
            int64_t E = 0;
            uint32_t prev = o0;
            for (int64_t i = 0; i < nblk; ++i) {
                if (i > 0) ck[b0 + i] = make_double2(aP, aM);   // alpha at position 64 i - 1
                const uint4 w = pk4[b0 + i];
                const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
                const int64_t left = len - 64 * i;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
#pragma unroll 4
                    for (int j = 0; j < 16; ++j) {
                        const int p = 16 * k + j;
                        if (p >= left) break;
                        const uint32_t cur = (ww[k] >> (2 * j)) & 3u;
                        if (i > 0 || p > 0) {
                            const double2 ma = TA[prev | (cur << 2)], mb = TB[prev | (cur << 2)];
                            const double nP = aP * ma.x + aM * mb.x, nM = aP * ma.y + aM * mb.y;
                            aP = nP;
                            aM = nM;
                            if ((j & 3) == 3) E += vnorm(aP, aM);
                        }
                        prev = cur;
                    }
                }
            }
            const double loglik = log(aP + aM) + (double)E * 0.69314718055994530942;
            atomicAdd((unsigned long long*)&sll, (unsigned long long)llrint(ldexp(loglik, kLogFix)));
            // backward, last block first; beta at the last position = (1, 1)
            double yP = 1.0, yM = 1.0;
            for (int64_t i = nblk - 1; i >= 0; --i) {
                const uint4 w = pk4[b0 + i];
                const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
                const uint32_t wprev = i > 0 ? a.packed[off / 16 + 4 * i - 1] : 0u;
                const int64_t left = len - 64 * i;
                // alpha entering the block (position 64 i - 1) and, in LDS, entering its
                // mini-blocks 1..3 (positions 16 k - 1): registers stay for the alpha window
                double xP0, xM0;
                if (i > 0) {
                    const double2 e = ck[b0 + i];
                    xP0 = e.x;
                    xM0 = e.y;
                } else {
                    xP0 = model.pi[o0];
                    xM0 = model.pi[o0 + 4];
                }
                {
                    double xP = xP0, xM = xM0;
                    uint32_t pv = wprev >> 30;
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
#pragma unroll 4
                        for (int j = 0; j < 16; ++j) {
                            const uint32_t cur = (ww[k] >> (2 * j)) & 3u;
                            if (16 * k + j < left && (i > 0 || k > 0 || j > 0)) {
                                const double2 ma = TA[pv | (cur << 2)], mb = TB[pv | (cur << 2)];
                                const double nP = xP * ma.x + xM * mb.x, nM = xP * ma.y + xM * mb.y;
                                xP = nP;
                                xM = nM;
                                if ((j & 3) == 3) vnorm(xP, xM);
                            }
                            pv = cur;
                        }
                        sent[k][t] = make_double2(xP, xM);
                    }
                }
#pragma unroll 1
                for (int k = 3; k >= 0; --k) {
                    if (16 * k >= left) continue;
                    // the mini-block's word and the base before it (select chains: no
                    // register indexing)
                    const uint32_t wk = k == 0 ? ww[0] : k == 1 ? ww[1] : k == 2 ? ww[2] : ww[3];
                    const uint32_t pk = (k == 0 ? wprev : k == 1 ? ww[0] : k == 2 ? ww[1] : ww[2]) >> 30;
                    double eP = xP0, eM = xM0;
                    if (k > 0) {
                        const double2 e = sent[k - 1][t];
                        eP = e.x;
                        eM = e.y;
                    }
                    // alpha at the 16 positions of the mini-block (registers)
                    double alP[16], alM[16];
                    {
                        double xP = eP, xM = eM;
                        uint32_t pv = pk;
#pragma unroll
                        for (int j = 0; j < 16; ++j) {
                            const uint32_t cur = (wk >> (2 * j)) & 3u;
                            if (16 * k + j < left && (i > 0 || k > 0 || j > 0)) {
                                const double2 ma = TA[pv | (cur << 2)], mb = TB[pv | (cur << 2)];
                                const double nP = xP * ma.x + xM * mb.x, nM = xP * ma.y + xM * mb.y;
                                xP = nP;
                                xM = nM;
                                if ((j & 3) == 3) vnorm(xP, xM);
                            }
                            alP[j] = xP;
                            alM[j] = xM;
                            pv = cur;
                        }
                    }
#pragma unroll
                    for (int j = 15; j >= 0; --j) {
                        const int p = 16 * k + j;
                        if (p >= left) continue;
                        if (i == 0 && p == 0) {   // gamma_0 -> init counts
                            // (2^-54 units: <= kCT contigs per round stay below 2^62)
                            const double gp = alP[0] * yP, gm = alM[0] * yM, z = gp + gm;
                            const double r = rcp_nr(z) * 18014398509481984.0;   // 2^54
                            atomicAdd(&sinit[o0], __double2ull_rn(gp * r));
                            atomicAdd(&sinit[o0 + 4], __double2ull_rn(gm * r));
                            continue;
                        }
                        const double uP = j > 0 ? alP[j - 1] : eP;
                        const double uM = j > 0 ? alM[j - 1] : eM;
                        const uint32_t d = (j > 0 ? ((wk >> (2 * j - 2)) & 3u) : pk) |
                                           (((wk >> (2 * j)) & 3u) << 2);
                        const double2 ma = TA[d], mb = TB[d];
                        const double t00 = ma.x * yP, t01 = ma.y * yM, t10 = mb.x * yP,
                                     t11 = mb.y * yM;
                        const double x00 = uP * t00, x01 = uP * t01, x10 = uM * t10,
                                     x11 = uM * t11;
                        const double r = rcp_nr((x00 + x01) + (x10 + x11)) * kFixC;
                        atomicAdd(wb + (0 * 16 + d) * 16, to_fixed_scaled(x00 * r));
                        atomicAdd(wb + (1 * 16 + d) * 16, to_fixed_scaled(x01 * r));
                        atomicAdd(wb + (2 * 16 + d) * 16, to_fixed_scaled(x10 * r));
                        atomicAdd(wb + (3 * 16 + d) * 16, to_fixed_scaled(x11 * r));
                        yP = t00 + t01;
                        yM = t10 + t11;
                        if ((j & 3) == 0) vnorm(yP, yM);
                    }
                }
            }
        }
        __syncthreads();
        // flush: bins (2^-38) -> the 128-bit accumulators (2^-47; init rows 2^-54 -> 2^-62)
        if (t < 64) {   // t = k * 16 + d  ->  slab row d * 4 + k
            unsigned long long s = 0;
#pragma unroll
            for (int col = 0; col < 16; ++col) s += bins[t * 16 + ((col + t) & 15)];
            if (s) acc128_add2(acc + 2 * ((t & 15) * 4 + (t >> 4)), s << 9, s >> 55);
        } else if (t < 72) {   // init rows: 2^-54 -> 2^-62 (k_estep.hip kFixInit): shift by 8
            const unsigned long long s = sinit[t - 64];
            if (s) acc128_add2(acc + 2 * t, s << 8, s >> 56);
        } else if (t == 72) {
            const long long L = sll;
            if (L) acc128_add2(acc + 2 * 72, (unsigned long long)L, L < 0 ? ~0ull : 0ull);
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ islands
struct IslState {
    bool in;
    bool atC;
    bool atC0;                          // atC just before the current island started
    int32_t beg, len, C, G, CG;
};
struct IslOut {
    cpg_island* out;
    int64_t cap;
    int64_t base;       // first record index of this contig (pass 2)
    int64_t nk;         // kept so far
    int64_t c;
    int32_t first_beg;  // pass 1: the first kept island's start, atC before it
    bool first_atC;
    int32_t last_close; // pass 1: the position whose '-' closed the last kept island
};
__device__ __forceinline__ void isl_close(const IslState& st, int32_t close, IslOut& o,
                                          bool write) {
    const double ccnt = (double)st.C, gcnt = (double)st.G;
    const double cg = (ccnt + gcnt) / (double)st.len;                        // :280
    double oe = 0.0;
    if (st.C != 0 && st.G != 0) {                                             // :282-283
        const int32_t prod = (int32_t)((uint32_t)st.CG * (uint32_t)st.len);   // int wraps
        oe = (double)prod / (ccnt * gcnt);
    }
    if (cg > 0.5 && oe > 0.6) {                                               // :285
        if (write) {
            const int64_t dst = o.base + o.nk;
            if (dst < o.cap) {
                cpg_island r;
                r.beg1 = st.beg + 1;
                r.end1 = close;                  // end = close - 1, 1-based
                r.len = st.len;
                r.chunk = (int32_t)o.c;
                r.cg = cg;
                r.oe = oe;
                o.out[dst] = r;
            }
        } else {
            if (o.nk == 0) {
                o.first_beg = st.beg;
                o.first_atC = st.atC0;
            }
            o.last_close = close;
        }
        ++o.nk;
    }
}
// The scan of :262-339 over one word of 32 positions from position j (sign bits s, C / G
// masks of the bases), jumping whole runs: a background run is skipped, an island run is
// added by popcounts (CpG = G whose predecessor is C inside the island; the first position's
// predecessor flag is atC, including the reference's stale carry across islands).
__device__ __forceinline__ void isl_word(IslState& st, uint32_t s, uint32_t Cm, uint32_t Gm,
                                         int32_t p0, int j, int jn, IslOut& o, bool write) {
    const uint32_t valid = jn >= 32 ? ~0u : ((1u << jn) - 1u);
    while (j < jn) {
        if (!st.in) {
            const uint32_t rest = s & valid & (~0u << j);
            if (!rest) return;
            j = __builtin_ctz(rest);                     // island starts here (:318-331)
            const bool isC = (Cm >> j) & 1u;
            st.in = true;
            st.len = 1;
            st.CG = 0;
            st.beg = p0 + j;
            st.atC0 = st.atC;
            st.C = isC ? 1 : 0;
            st.G = (int32_t)((Gm >> j) & 1u);
            if (isC) st.atC = true;                      // stale otherwise
            ++j;
        } else {
            const uint32_t minus = ~s & valid & (j < 32 ? (~0u << j) : 0u);
            const int e = minus ? __builtin_ctz(minus) : jn;
            if (e > j) {                                 // island positions j .. e-1
                const uint32_t seg = (e >= 32 ? ~0u : ((1u << e) - 1u)) & ~((1u << j) - 1u);
                const uint32_t prevC = ((Cm << 1) & seg & ~(1u << j)) | (st.atC ? (1u << j) : 0u);
                st.len += e - j;
                st.C += __popc(Cm & seg);
                st.G += __popc(Gm & seg);
                st.CG += __popc(Gm & seg & prevC);
                st.atC = (Cm >> (e - 1)) & 1u;
            }
            j = e;
            if (j < jn) {                                // '-' at j closes it (atC kept)
                st.in = false;
                isl_close(st, p0 + j, o, write);
                ++j;
            }
        }
    }
}

// pass 1 (kWrite = false): kept islands per contig + the window [first kept start, last kept
// close] and the stale atC before it; pass 2 rescans only that window, writing records
template <bool kWrite>
__global__ __launch_bounds__(kCT) void k_ctg_islands(Ctg a, int64_t* __restrict__ cnt,
                                                     int64_t* __restrict__ win,
                                                     const int64_t* __restrict__ base,
                                                     cpg_island* __restrict__ out,
                                                     int64_t cap) {
    const uint2* pk2 = reinterpret_cast<const uint2*>(a.packed);
    const int64_t stride = (int64_t)gridDim.x * kCT;
    for (int64_t g = (int64_t)blockIdx.x * kCT + threadIdx.x; g < a.n; g += stride) {
        int64_t c, off, len;
        if (!ctg_get(a, g, c, off, len, 0x7FFFFFFF)) {   // c is set even when invalid
            if (!kWrite) cnt[c] = 0;
            continue;
        }
        IslState st{false, false, false, 0, 0, 0, 0, 0};
        IslOut o{out, cap, 0, 0, c, 0, false, 0};
        int64_t k0 = 0, k1 = (len + 31) / 32;
        int j0 = 0;
        int64_t stop = len;              // positions processed: [.., stop)
        if (kWrite) {
            if (cnt[c] == 0) continue;
            const int64_t wv = win[c];
            const int32_t fb = (int32_t)(wv & 0x7FFFFFFF);
            st.atC = ((wv >> 31) & 1) != 0;
            stop = (wv >> 32) + 1;       // through the closing '-'
            k0 = fb / 32;
            j0 = fb % 32;
            k1 = (stop + 31) / 32;
            o.base = base[c];
        }
        for (int64_t k = k0; k < k1; ++k) {
            const uint32_t s = a.sign[off / 32 + k];
            const int64_t left = stop - 32 * k;
            const int jn = left >= 32 ? 32 : (int)left;
            if (!st.in && (s & (jn >= 32 ? ~0u : ((1u << jn) - 1u))) == 0u) continue;
            const uint2 pw = pk2[off / 32 + k];
            const Masks m0 = base_masks(pw.x), m1 = base_masks(pw.y);
            const uint32_t Cm = pext_even(m0.e[1]) | (pext_even(m1.e[1]) << 16);
            const uint32_t Gm = pext_even(m0.e[2]) | (pext_even(m1.e[2]) << 16);
            isl_word(st, s, Cm, Gm, (int32_t)(32 * k), k == k0 ? j0 : 0, jn, o, kWrite);
        }
        // an island still open at the contig end is dropped (as at a chunk end)
        if (!kWrite) {
            cnt[c] = o.nk;
            if (o.nk)
                win[c] = (int64_t)o.first_beg | ((int64_t)(o.first_atC ? 1 : 0) << 31) |
                         ((int64_t)o.last_close << 32);
        }
    }
}

__global__ void k_ctg_iota(int32_t* __restrict__ v, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (int32_t)i;
}
__global__ void k_ctg_total(const int64_t* __restrict__ cnt, const int64_t* __restrict__ base,
                            int64_t n, int64_t* __restrict__ total) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *total = n > 0 ? base[n - 1] + cnt[n - 1] : 0;
}

unsigned grid_for(int64_t n) {
    const int64_t wg = (n + kCT - 1) / kCT;
    return (unsigned)(wg < kCtgGrid ? (wg > 0 ? wg : 1) : kCtgGrid);
}

}  // namespace

// ---- launchers -----------------------------------------------------------------------
size_t contigs_sort_ws_bytes(int64_t n) {
    size_t tmp = 0;
    (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tmp, (const int32_t*)nullptr,
                                                 (int32_t*)nullptr, (const int32_t*)nullptr,
                                                 (int32_t*)nullptr, (int)n, 0, 32);
    size_t scan = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan, (const int64_t*)nullptr, (int64_t*)nullptr,
                                     (int)n);
    const size_t a = tmp > scan ? tmp : scan;
    return ((a + 255) & ~(size_t)255) + (size_t)n * 8 * 3 + 512;
}

hipError_t launch_contigs_order(const int32_t* lens, int64_t n, int32_t* order, void* ws,
                                size_t ws_bytes, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    if (n >= (1ll << 31)) return hipErrorInvalidValue;
    char* w = static_cast<char*>(ws);
    size_t tmp = 0;
    (void)hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tmp, lens, (int32_t*)nullptr,
                                                 (const int32_t*)nullptr, order, (int)n, 0, 32);
    const size_t need = ((tmp + 255) & ~(size_t)255) + (size_t)n * 8;
    if (need > ws_bytes) return hipErrorInvalidValue;
    int32_t* keys_out = reinterpret_cast<int32_t*>(w + ((tmp + 255) & ~(size_t)255));
    int32_t* iota = keys_out + n;
    hipLaunchKernelGGL(k_ctg_iota, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, iota, n);
    return hipcub::DeviceRadixSort::SortPairsDescending(w, tmp, lens, keys_out, iota, order,
                                                        (int)n, 0, 32, s);
}

static Ctg make_ctg(const uint32_t* packed, const uint32_t* sign, int64_t nbases,
                    const int64_t* offs, const int32_t* lens, const int32_t* order, int64_t n,
                    uint32_t* status) {
    return Ctg{packed, sign, offs, lens, order, n, nbases, status};
}

hipError_t launch_contigs_count(const uint32_t* packed, const uint32_t* sign, int64_t nbases,
                                const int64_t* offs, const int32_t* lens, const int32_t* order,
                                int64_t n, uint64_t* ws, int64_t* out, uint32_t* status,
                                hipStream_t s) {
    if (n > 0)
        hipLaunchKernelGGL(k_ctg_count, dim3(grid_for(n)), dim3(kCT), 0, s,
                           make_ctg(packed, sign, nbases, offs, lens, order, n, status),
                           (unsigned long long*)ws);
    return launch_count(nullptr, nullptr, 0, CPG_TRAIN_CHUNK, ws, out, s, PART_FINAL);
}

hipError_t launch_contigs_viterbi(const VitConsts& vc, const uint32_t* packed, int64_t nbases,
                                  const int64_t* offs, const int32_t* lens, const int32_t* order,
                                  int64_t n, uint32_t* bp, uint32_t* sign_out, double* score,
                                  uint32_t* status, hipStream_t s) {
    if (n > 0)
        hipLaunchKernelGGL(k_ctg_viterbi, dim3(grid_for(n)), dim3(kCT), 0, s,
                           make_ctg(packed, nullptr, nbases, offs, lens, order, n, status), vc,
                           bp, sign_out, score);
    return hipGetLastError();
}

hipError_t launch_contigs_estep(const cpg_model& model, const uint32_t* packed, int64_t nbases,
                                const int64_t* offs, const int32_t* lens, const int32_t* order,
                                int64_t n, void* ck, unsigned long long* acc, double* out,
                                uint32_t* status, hipStream_t s) {
    if (n > 0)
        hipLaunchKernelGGL(k_ctg_estep, dim3(grid_for(n)), dim3(kCT), 0, s,
                           make_ctg(packed, nullptr, nbases, offs, lens, order, n, status), model,
                           static_cast<double2*>(ck), acc);
    return launch_estep(model, nullptr, 0, CPG_TRAIN_CHUNK, acc, out, s, PART_FINAL);
}

hipError_t launch_contigs_islands(const uint32_t* packed, const uint32_t* sign, int64_t nbases,
                                  const int64_t* offs, const int32_t* lens, const int32_t* order,
                                  int64_t n, void* ws, size_t ws_bytes, cpg_island* out,
                                  int64_t cap, int64_t* count, uint32_t* status, hipStream_t s) {
    if (n <= 0) return hipMemsetAsync(count, 0, sizeof(int64_t), s);
    char* w = static_cast<char*>(ws);
    size_t tmp = 0;
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, (const int64_t*)nullptr, (int64_t*)nullptr,
                                     (int)n);
    const size_t tmpa = (tmp + 255) & ~(size_t)255;
    if (tmpa + (size_t)n * 24 > ws_bytes) return hipErrorInvalidValue;
    int64_t* cnt = reinterpret_cast<int64_t*>(w + tmpa);
    int64_t* base = cnt + n;
    int64_t* win = base + n;
    const Ctg a = make_ctg(packed, sign, nbases, offs, lens, order, n, status);
    hipLaunchKernelGGL(k_ctg_islands<false>, dim3(grid_for(n)), dim3(kCT), 0, s, a, cnt, win,
                       (const int64_t*)nullptr, out, cap);
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(w, tmp, cnt, base, (int)n, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_ctg_islands<true>, dim3(grid_for(n)), dim3(kCT), 0, s, a, cnt, win,
                       base, out, cap);
    hipLaunchKernelGGL(k_ctg_total, dim3(1), dim3(64), 0, s, cnt, base, n, count);
    return hipGetLastError();
}

}  // namespace cpg
