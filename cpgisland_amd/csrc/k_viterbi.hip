// k_viterbi.hip — exact parallel Viterbi for the CpG-island HMM on gfx950.
//
// Replaces HmmEvaluator.decode(trainedModel, testSequence, true)
// (/root/reference/CpGIslandFinder.java:260; Mahout HmmAlgorithms.viterbiAlgorithm,
// scaled=true) applied to every whole chunk (:256-260).  Result: the state path, bit-for-bit
// the one the sequential fp64 recurrence produces (Mahout operation order, '>' tie-break),
// not an approximation of it.
//
// Why a parallel scan can be exact here:
//   With the deterministic emission matrix only the two states (o_t,+) and (o_t,-) are live,
//   so the recurrence is a 2x2 max-plus product per step with constants L[dinucleotide].
//   fp64 addition is not associative in general — but while every value of a stretch of the
//   recurrence lies in one binade [2^e, 2^(e+1)) (values are negative: in magnitude), every
//   double there is a multiple of u_e = 2^(e-52), so fl(x + L) = x + RN_e(L) exactly (RN_e
//   = round to a multiple of u_e; host checks that no constant sits on a rounding tie).
//   Within a binade the recurrence is therefore EXACT max-plus arithmetic over the rounded
//   constants, which is associative: sub-block composites can be combined in any order.
//
// Pipeline (one lane = one 256-position sub-block "block"):
//   K1 approx composite   int32 fixed-point 2x2 composite per block
//   K2 plan               per chunk: scan of K1 composites -> approximate values at every
//                         block boundary (error <= eps, bounded on the host); classify each
//                         block (same kernel): REGULAR (inside one binade), SPLIT (one binade crossing:
//                         exact prefix composite + short sequential window + exact suffix
//                         composite), SEQ (sequential), DEGEN (pi = 0 for both live states)
//   K3/K3b exact composite fp64 composites with the binade-rounded constants (exact)
//   K4 chain              per chunk: segmented scan of exact composites; ONE lane walks the
//                         few barriers (windows / SEQ blocks) sequentially with the original
//                         constants; exact entry value of every block
//   K5 re-forward         per block from its exact entry with the ORIGINAL constants, the
//                         reference's own step (same rounding, same '>' tie-break): 2-bit
//                         backpointers; the exit value must equal the next block's entry
//                         bit-for-bit (self-check -> status word)
//   K6 trace scan         per chunk: final argmax + suffix scan of block origin maps
//   K7 traceback          per block: state path -> sign bits
//
// Layout: packed bases (16/uint32, base k at bits 2k), sign bits (32/uint32), all in HBM.
// Dinucleotide code d = prev | cur << 2 (one bfe of the packed word).

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>

#include "cpg_internal.h"

#include "isl_dev.h"

namespace cpg {
namespace {

constexpr int kThreads = 256;
constexpr int kMaxSeg = 16;   // segment path: 256-block segments per chunk (chunks up to 1 Mi)
constexpr int32_t kNeg32 = -(1 << 30);
constexpr int64_t kNeg64 = -(1ll << 60);

// 2x2 max-plus matrices: rows = start state (0 '+', 1 '-'), cols = end state.
struct C64 {
    double pp, pm, mp, mm;
};
struct CI {
    int64_t pp, pm, mp, mm;
};

__device__ __forceinline__ C64 c64_id() { return {0.0, -INFINITY, -INFINITY, 0.0}; }
__device__ __forceinline__ CI ci_id() { return {0, kNeg64, kNeg64, 0}; }

// one step of the composite with constants l = (+->+, -->+, +->-, -->-)
__device__ __forceinline__ void c64_step(C64& c, double l0, double l1, double l2, double l3) {
    double npp = fmax(c.pp + l0, c.pm + l1);
    double npm = fmax(c.pp + l2, c.pm + l3);
    double nmp = fmax(c.mp + l0, c.mm + l1);
    double nmm = fmax(c.mp + l2, c.mm + l3);
    c = {npp, npm, nmp, nmm};
}
__device__ __forceinline__ C64 c64_mul(const C64& a, const C64& b) {
    return {fmax(a.pp + b.pp, a.pm + b.mp), fmax(a.pp + b.pm, a.pm + b.mm),
            fmax(a.mp + b.pp, a.mm + b.mp), fmax(a.mp + b.pm, a.mm + b.mm)};
}
__device__ __forceinline__ double2 c64_apply(double2 v, const C64& c) {
    return make_double2(fmax(v.x + c.pp, v.y + c.mp), fmax(v.x + c.pm, v.y + c.mm));
}
__device__ __forceinline__ int64_t cl(int64_t x) { return x < kNeg64 ? kNeg64 : x; }
__device__ __forceinline__ int64_t mx(int64_t a, int64_t b) { return a > b ? a : b; }
__device__ __forceinline__ CI ci_mul(const CI& a, const CI& b) {
    return {cl(mx(a.pp + b.pp, a.pm + b.mp)), cl(mx(a.pp + b.pm, a.pm + b.mm)),
            cl(mx(a.mp + b.pp, a.mm + b.mp)), cl(mx(a.mp + b.pm, a.mm + b.mm))};
}
__device__ __forceinline__ CI shfl_up_ci(const CI& x, int d) {
    return {__shfl_up(x.pp, d), __shfl_up(x.pm, d), __shfl_up(x.mp, d), __shfl_up(x.mm, d)};
}
__device__ __forceinline__ void ci_apply(int64_t& P, int64_t& M, const CI& c) {
    int64_t nP = cl(mx(P + c.pp, M + c.mp)), nM = cl(mx(P + c.pm, M + c.mm));
    P = nP;
    M = nM;
}

// The reference step (Mahout order): target '+' sees predecessor '+' first, so '-' wins
// only when strictly greater; + log(1.0) = +0.0 is exact and omitted.
struct Step {
    double P, M;
    uint32_t bP, bM;   // 1: predecessor is '-'
};
__device__ __forceinline__ Step ref_step(double P, double M, double l0, double l1, double l2,
                                         double l3) {
    double cpp = P + l0, cmp = M + l1, cpm = P + l2, cmm = M + l3;
    Step s;
    s.bP = cmp > cpp;
    s.bM = cmm > cpm;
    // the survivor value is the max either way: on a tie both candidates are the same
    // double (sums of finite values or -inf never give NaN or -0), so v_max_f64 replaces
    // two 32-bit selects per state
    s.P = fmax(cpp, cmp);
    s.M = fmax(cpm, cmm);
    return s;
}

__device__ __forceinline__ uint32_t base_at(const uint32_t* __restrict__ pk, int64_t pos) {
    return (pk[pos >> 4] >> ((pos & 15) * 2)) & 3u;
}

// Walk the steps of block k (positions k*256 .. k*256+255 of the chunk, position 0 and
// positions >= C excluded).  f(d, q, jj): d = dinucleotide code, q = quad (64 positions),
// jj = position within the quad (compile-time).
template <bool kFull, class F>
__device__ __forceinline__ void walk_block(const uint32_t* __restrict__ pk, int64_t k, int64_t C,
                                           F&& f) {
    const int64_t wbase = k * kSBWords;
    const int64_t nwords = (C + 15) >> 4;
    uint32_t prev = (k > 0) ? pk[wbase - 1] : 0u;
    uint4 cur;
    if (kFull) cur = *reinterpret_cast<const uint4*>(pk + wbase);   // next quad prefetched below
#pragma unroll 1
    for (int q = 0; q < 4; ++q) {
        uint32_t w[4];
        if (kFull) {
            const uint4 nxt =
                q < 3 ? *reinterpret_cast<const uint4*>(pk + wbase + 4 * (q + 1)) : cur;
            w[0] = cur.x; w[1] = cur.y; w[2] = cur.z; w[3] = cur.w;
            cur = nxt;
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t wi = wbase + 4 * q + r;
                w[r] = wi < nwords ? pk[wi] : 0u;
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int jj = r * 16 + i;
                const uint32_t d = (i == 0) ? (__builtin_amdgcn_alignbit(w[r], prev, 30) & 15u)
                                            : ((w[r] >> (2 * i - 2)) & 15u);
                if (kFull) {
                    f(d, q, jj);
                } else {
                    const int64_t pos = k * kSB + q * 64 + jj;
                    if (pos >= 1 && pos < C) f(d, q, jj);
                }
            }
            prev = w[r];
        }
    }
}

// the 17 packed words a full block reads (its 16 + the one before), all loads in flight
struct BlockWords {
    uint32_t w[16], prev;
};
__device__ __forceinline__ BlockWords load_block(const uint32_t* __restrict__ pk, int64_t k) {
    const int64_t wbase = k * kSBWords;
    BlockWords b;
    const uint4* p4 = reinterpret_cast<const uint4*>(pk + wbase);
    const uint4 a0 = p4[0], a1 = p4[1], a2 = p4[2], a3 = p4[3];
    b.prev = k > 0 ? pk[wbase - 1] : 0u;   // block 0: no word before (its step 0 is skipped)
    b.w[0] = a0.x; b.w[1] = a0.y; b.w[2] = a0.z; b.w[3] = a0.w;
    b.w[4] = a1.x; b.w[5] = a1.y; b.w[6] = a1.z; b.w[7] = a1.w;
    b.w[8] = a2.x; b.w[9] = a2.y; b.w[10] = a2.z; b.w[11] = a2.w;
    b.w[12] = a3.x; b.w[13] = a3.y; b.w[14] = a3.z; b.w[15] = a3.w;
    return b;
}

// dinucleotide code of step j (compile-time) of a full block; j = 0 pairs with the word before
__device__ __forceinline__ uint32_t bw_code(const BlockWords& b, int j) {
    const int r = j >> 4, i = j & 15;
    const uint32_t lo = r == 0 ? b.prev : b.w[r - 1];
    return i == 0 ? (__builtin_amdgcn_alignbit(b.w[r], lo, 30) & 15u)
                  : ((b.w[r] >> (2 * i - 2)) & 15u);
}

// Software-pipelined table walk over NSTEP compile-time steps: the LDS lookup of step j + G
// is issued before step j is consumed, so G lookups are in flight behind the dependent
// recurrence (the blocks' lanes are few per SIMD: latency, not bandwidth, is the limit).
template <int G, int NSTEP, class Idx, class Fetch, class Use>
__device__ __forceinline__ void pipelined(Idx&& idx, Fetch&& fetch, Use&& use) {
    using V = decltype(fetch(0u));
    V ring[G];
#pragma unroll
    for (int j = 0; j < G; ++j) ring[j] = fetch(idx(j));
#pragma unroll
    for (int j = 0; j < NSTEP; ++j) {
        const V v = ring[j % G];
        if (j + G < NSTEP) ring[j % G] = fetch(idx(j + G));
        use(v, j);
    }
}

struct Geo {
    int64_t nchunks, C, nsb;
    __device__ __forceinline__ bool full(int64_t k) const { return k > 0 && (k + 1) * kSB <= C; }
    // all 256 positions inside the chunk (block 0 included: its step 0 is an identity)
    __device__ __forceinline__ bool whole(int64_t k) const { return (k + 1) * kSB <= C; }
    __device__ __forceinline__ int jfirst(int64_t k) const { return k == 0 ? 1 : 0; }
    __device__ __forceinline__ int jend(int64_t k) const {
        int64_t e = C - k * kSB;
        return (int)(e < kSB ? (e < 0 ? 0 : e) : kSB);
    }
};

__device__ __forceinline__ const uint32_t* chunk_ptr(const uint32_t* packed, const Geo& g,
                                                     int64_t c) {
    return packed + c * (g.C >> 4);   // C % 256 == 0 whenever nchunks > 1
}

// ---------------------------------------------------------------- K1: approx composite
__device__ __forceinline__ int4 i4_mul(const int4 a, const int4 b) {   // max-plus, int32
    return make_int4(max(a.x + b.x, a.y + b.z), max(a.x + b.y, a.y + b.w),
                     max(a.z + b.x, a.w + b.z), max(a.z + b.y, a.w + b.w));
}
// single-step matrix of dinucleotide d in the (pp, pm, mp, mm) layout from Q = (+->+,
// -->+, +->-, -->-)
__device__ __forceinline__ int4 q_mat(const int4 q) { return make_int4(q.x, q.z, q.y, q.w); }

// Block 0 of every chunk starts at the chunk's first base and crosses several binades
// (|delta| grows from ~2 to ~360 over its 256 steps), so it is always walked sequentially.
// That walk needs nothing but the bases and the model: extra "head" workgroups of K2's launch run it
// (one lane per chunk, the reference step with the original constants, pipelined table
// lookups) while the main workgroups build composites; K4 starts from its exit value.
__device__ void vit_head(const VitConsts& vc, const uint32_t* packed, const Geo& g,
                         int64_t c, double2* __restrict__ vhead) {
    __shared__ double2 HA[17], HB[17];   // (l0, l1) | (l2, l3); entry 16: identity step
    if (threadIdx.x < 16) {
        HA[threadIdx.x] = make_double2(vc.L[threadIdx.x][0], vc.L[threadIdx.x][1]);
        HB[threadIdx.x] = make_double2(vc.L[threadIdx.x][2], vc.L[threadIdx.x][3]);
    } else if (threadIdx.x == 16) {
        HA[16] = make_double2(0.0, -INFINITY);
        HB[16] = make_double2(-INFINITY, 0.0);
    }
    __syncthreads();
    if (c >= g.nchunks) return;
    const uint32_t* pk = chunk_ptr(packed, g, c);
    const uint32_t o0 = pk[0] & 3u;
    double P = vc.logpi[o0], M = vc.logpi[o0 + 4];
    if (g.whole(0)) {
        const BlockWords bw = load_block(pk, 0);
        pipelined<4, kSB>([&](int j) { return j == 0 ? 16u : bw_code(bw, j); },
                          [&](uint32_t d) { return C64{HA[d].x, HA[d].y, HB[d].x, HB[d].y}; },
                          [&](const C64& l, int) {
                              const Step st = ref_step(P, M, l.pp, l.pm, l.mp, l.mm);
                              P = st.P;
                              M = st.M;
                          });
    } else {
        walk_block<false>(pk, 0, g.C, [&](uint32_t d, int, int) {
            const Step st = ref_step(P, M, HA[d].x, HA[d].y, HB[d].x, HB[d].y);
            P = st.P;
            M = st.M;
        });
    }
    vhead[c] = make_double2(P, M);
}

// ---------------------------------------------------------------- model-derived tables
// K1's 4-step fixed-point products and K3's per-binade step / 2-step tables depend on the
// model only; k_vit_tables writes them once per model (vit_tables' cache) right after the
// VitTables in the same allocation, and every K1/K3 workgroup copies its part to LDS.
constexpr int kQ4 = 1280;   // 4-step products over 5-base windows [0, 1024), 3-step [1024, 1280)
constexpr int kW4 = 1024;   // 4-step composites over 5-base windows b0..b4 (bits 2k: b_k)
struct VitDerived {
    int4 Q4[kQ4];
    double2 sA[kMaxBinade * 16], sB[kMaxBinade * 16];    // single-step halves (l0,l1) | (l2,l3)
    double2 P2A[kMaxBinade * 64], P2B[kMaxBinade * 64];  // 2-step composites (pp,pm) | (mp,mm)
    double2 P4A[kMaxBinade * kW4], P4B[kMaxBinade * kW4];   // 4-step composites, same halves
};
__device__ __forceinline__ const VitDerived* derived(const VitTables* vt) {
    return reinterpret_cast<const VitDerived*>(vt + 1);
}

// Waves per SIMD a kernel is compiled for (VGPR budget 512 / n).  On a training CU the
// E-step holds 4 waves x 96 VGPRs per SIMD, leaving 128: a decode kernel of <= 64 VGPRs gets
// two wave slots there instead of one.  K5 (the longest decode kernel under overlap) is built
// for 8 (64 VGPRs; its few spills are outside the step loop): bench +2 % with the 2-deep
// lookup ring below (profiles/r02_v10/ab_k5_occupancy*.log).  K3 at 8 (spills) and K7 at 8 (75
// spills) were slower; K1 cannot reach 64 at its LDS (the slim-LDS variant at 64 lost 1.5 %).
constexpr int kK5WavesPerEU = 8;
// the fused form (K6 inside: decodes of <= 256 chunks, tail_fusion_pays) runs ~3 waves per
// SIMD — too few to cover a step's table-lookup latency with one another — so its lookups are
// issued kK5LookFused steps ahead (the registers for them: 2 ahead fits the 64 of 8 waves per
// SIMD that the long decodes' form keeps)
constexpr int kK5LookFused = 4;
constexpr int kK5WavesPerEUFused = 6;
__global__ __launch_bounds__(kThreads) void k_vit_tables(VitConsts vc, VitTables* vt) {
    VitDerived* dv = reinterpret_cast<VitDerived*>(vt + 1);
    const int n = kQ4 + kMaxBinade * 16 + kMaxBinade * 64 + kMaxBinade * kW4;
    for (int i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads) {
        if (i < kQ4) {   // i >= 1024: 3-step entries (block 0's first window; b0 unused)
            const bool three = i >= 1024;
            const int w = three ? (i - 1024) << 2 : i;
            auto qd = [&](int d) {
                return q_mat(make_int4(vc.Q[d][0], vc.Q[d][1], vc.Q[d][2], vc.Q[d][3]));
            };
            int4 m = three ? make_int4(0, kNeg32, kNeg32, 0) : qd((w & 3) | (((w >> 2) & 3) << 2));
            for (int k = 1; k < 4; ++k) {
                const int p = (w >> (2 * k)) & 3, b = (w >> (2 * k + 2)) & 3;
                m = i4_mul(m, qd(p | (b << 2)));
            }
            dv->Q4[i] = m;
        } else if (i < kQ4 + kMaxBinade * 16) {
            const int j = i - kQ4;
            const double* l = vt->Le[j / 16][j % 16];
            dv->sA[j] = make_double2(l[0], l[1]);
            dv->sB[j] = make_double2(l[2], l[3]);
        } else if (i >= kQ4 + kMaxBinade * 16 + kMaxBinade * 64) {
            // 4-step composite of window w: steps with dinucleotides (w >> 2k) & 15, k = 0..3
            const int j = i - kQ4 - kMaxBinade * 16 - kMaxBinade * 64, e = j / kW4, w = j % kW4;
            const double* l = vt->Le[e][w & 15];
            C64 m{l[0], l[2], l[1], l[3]};
            for (int k = 1; k < 4; ++k) {
                const double* lk = vt->Le[e][(w >> (2 * k)) & 15];
                c64_step(m, lk[0], lk[1], lk[2], lk[3]);
            }
            dv->P4A[j] = make_double2(m.pp, m.pm);
            dv->P4B[j] = make_double2(m.mp, m.mm);
        } else {
            const int j = i - kQ4 - kMaxBinade * 16, e = j / 64, w = j % 64;
            const double* l1 = vt->Le[e][(w & 3) | (((w >> 2) & 3) << 2)];          // x -> y
            const double* l2 = vt->Le[e][((w >> 2) & 3) | (((w >> 4) & 3) << 2)];   // y -> z
            // composite of one step: (pp, pm, mp, mm) = (l0, l2, l1, l3)
            C64 m{l1[0], l1[2], l1[1], l1[3]};
            c64_step(m, l2[0], l2[1], l2[2], l2[3]);
            dv->P2A[j] = make_double2(m.pp, m.pm);
            dv->P2B[j] = make_double2(m.mp, m.mm);
        }
    }
}

// Segment path of K1 (chunks of whole 256-block segments): each workgroup (one segment) also
// stores its segment's ordered product of the approximate composites; the next launch,
// k_vit_segplan (K2's work per segment), reads the products of the chunk's earlier segments
// from it — a kernel boundary, so no workgroup waits for another.
struct ApproxSeg {
    CI* segprod;               // [segment]: product of the segment's block composites (K1)
    longlong2* aent;
    uint8_t* degen;
    VitPlan* plan;
    int32_t* irrlist;          // [segment][256]
    int32_t* irrseg;           // [segment]: irregular blocks listed
};
__device__ __forceinline__ int64_t fix_of(double x, int f);
__device__ __forceinline__ VitPlan classify(const VitConsts& vc, const Geo& g, int64_t k,
                                            longlong2 en, longlong2 ex, bool& irregular);

__global__ __launch_bounds__(kThreads) void k_vit_approx(VitConsts vc, const uint32_t* packed,
                                                         Geo g, const VitTables* vt,
                                                         int4* __restrict__ comp, ApproxSeg as) {
    __shared__ int4 Q[16];
    // 4-step products over 5-base windows b0..b4 (exact: integers) [0, 1024), then the
    // 3-step products of steps 1..3 over b1..b4 [1024, 1280): block 0's first window (the
    // chunk's position 0 carries no step) — copied from the per-model tables (k_vit_tables)
    __shared__ int4 Q4[kQ4];
    if (threadIdx.x < 16)
        Q[threadIdx.x] = make_int4(vc.Q[threadIdx.x][0], vc.Q[threadIdx.x][1],
                                   vc.Q[threadIdx.x][2], vc.Q[threadIdx.x][3]);
    const int4* gq = derived(vt)->Q4;
#pragma unroll
    for (int i = 0; i < kQ4 / kThreads; ++i) Q4[threadIdx.x + i * kThreads] = gq[threadIdx.x + i * kThreads];
    __syncthreads();
    const int64_t gid = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (gid >= g.nchunks * g.nsb) return;   // (segment path: every lane is valid)
    const int64_t c = gid / g.nsb, k = gid - c * g.nsb;
    const uint32_t* pk = chunk_ptr(packed, g, c);
    if (g.whole(k)) {
        int4 acc = make_int4(0, kNeg32, kNeg32, 0);
        const BlockWords bw = load_block(pk, k);
        const bool first = k == 0;
        pipelined<4, 64>(
            [&](int j) {   // 5-base window of steps 4j .. 4j+3
                const int r = j >> 2, s = j & 3;
                const uint32_t lo = r == 0 ? bw.prev : bw.w[r - 1];
                const uint32_t wi = s == 0 ? (__builtin_amdgcn_alignbit(bw.w[r], lo, 30) & 0x3FFu)
                                           : ((bw.w[r] >> (8 * s - 2)) & 0x3FFu);
                return (j == 0 && first) ? 1024u + (wi >> 2) : wi;
            },
            [&](uint32_t wi) { return Q4[wi]; }, [&](const int4 q, int) { acc = i4_mul(acc, q); });
        comp[gid] = acc;
        if (as.segprod) {   // segment path (whole blocks only): the segment's ordered product,
                            // a butterfly over the wave (the lower lane's factor first), then
                            // the four wave products in order
            CI x{acc.x, acc.y, acc.z, acc.w};
            const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const CI y{__shfl_xor(x.pp, off), __shfl_xor(x.pm, off), __shfl_xor(x.mp, off),
                           __shfl_xor(x.mm, off)};
                x = (lane & off) ? ci_mul(y, x) : ci_mul(x, y);
            }
            __shared__ CI sW[kThreads / 64];
            if (lane == 0) sW[wv] = x;
            __syncthreads();
            if (threadIdx.x == 0)
                as.segprod[blockIdx.x] = ci_mul(ci_mul(sW[0], sW[1]), ci_mul(sW[2], sW[3]));
        }
        return;
    }
    int32_t a = 0, b = kNeg32, e = kNeg32, f = 0;
    auto step = [&](uint32_t d, int, int) {
        const int4 q = Q[d];
        int32_t na = max(a + q.x, b + q.y), nb = max(a + q.z, b + q.w);
        int32_t ne = max(e + q.x, f + q.y), nf = max(e + q.z, f + q.w);
        a = na; b = nb; e = ne; f = nf;
    };
    walk_block<false>(pk, k, g.C, step);
    comp[gid] = make_int4(a, b, e, f);
}

// ---------------------------------------------------------------- K2: plan
__device__ __forceinline__ int64_t fix_of(double x, int f) {
    if (!(x > -INFINITY)) return kNeg64;
    return (int64_t)llrint(ldexp(x, f));
}
__device__ __forceinline__ bool binade_ok(const VitConsts& vc, int e) {
    return e >= vc.emin && e <= vc.emax && !((vc.tie_mask >> e) & 1ull);
}

// K2 (one workgroup of 1024 lanes per chunk): scan of the K1 composites -> approximate
// value entering every block (fixed point, int64; stored for the irregular blocks),
// then every block is classified from its entry/exit estimates: REGULAR (inside one
// binade) or irregular (listed for K3b); block 0 is always sequential; DEGEN chunks (pi = 0
// for both live states) skip everything.
constexpr int kScanT = 1024;
__device__ __forceinline__ VitPlan classify(const VitConsts& vc, const Geo& g, int64_t k,
                                            longlong2 en, longlong2 ex, bool& irregular) {
    const double invS = ldexp(1.0, -vc.qshift);
    VitPlan p{PLAN_SEQ, 0, 0, 0, 0, 0};
    const int j0 = g.jfirst(k), jend = g.jend(k);
    irregular = false;
    if (k > 0 && jend > j0) {
        const double hi = (double)mx(en.x, en.y) * invS + vc.eps;
        const double lo = (double)mx(ex.x, ex.y) * invS - vc.eps - vc.spread;
        const int e = hi < 0.0 ? ilogb(-hi) : -1;
        if (e >= 0 && binade_ok(vc, e) && lo > -ldexp(1.0, e + 1))
            p = VitPlan{PLAN_REGULAR, (int8_t)e, 0, 0, (uint16_t)jend, (uint16_t)jend};
        else
            irregular = hi < 0.0;
    }
    return p;
}

__global__ __launch_bounds__(kScanT) void k_vit_scan(VitConsts vc, const uint32_t* packed, Geo g,
                                                     const int4* __restrict__ comp,
                                                     longlong2* __restrict__ aent,
                                                     uint8_t* __restrict__ degen,
                                                     VitPlan* __restrict__ plan,
                                                     int32_t* __restrict__ irrlist,
                                                     int32_t* __restrict__ irrcount,
                                                     double2* __restrict__ vhead) {
    if (blockIdx.x >= g.nchunks) {   // workgroup-uniform: the head workgroups (vit_head)
        vit_head(vc, packed, g, (int64_t)(blockIdx.x - g.nchunks) * kScanT + threadIdx.x, vhead);
        return;
    }
    const int64_t c = blockIdx.x;
    const int t = threadIdx.x;
    const uint32_t* pk = chunk_ptr(packed, g, c);
    const int4* cc = comp + c * g.nsb;
    longlong2* ae = aent + c * (g.nsb + 1);
    VitPlan* pl = plan + c * g.nsb;
    __shared__ CI buf[kScanT / 64];   // wave products
    __shared__ int sIrr;
    const int64_t per = (g.nsb + kScanT - 1) / kScanT;
    const int64_t b0 = min((int64_t)t * per, g.nsb), b1 = min(b0 + per, g.nsb);
    const uint32_t o0 = base_at(pk, 0);
    const double lp = vc.logpi[o0], lm = vc.logpi[o0 + 4];
    const bool dg = !(lp > -INFINITY) && !(lm > -INFINITY);   // uniform per workgroup
    if (t == 0) {
        degen[c] = dg ? 1 : 0;
        sIrr = 0;
    }
    if (dg) {
        for (int64_t k = b0; k < b1; ++k) pl[k] = VitPlan{PLAN_DEGEN, 0, 0, 0, 0, 0};
        if (t == 0) irrcount[c] = 0;
        return;
    }
    // a lane's (<= kPre2 for chunks up to 1 Mi) composites are loaded up front, all in flight,
    // and kept in registers for the classification pass (no second, dependent read per block)
    constexpr int kPre2 = 4;
    const int cnt = (int)(b1 - b0);
    const bool pre = cnt <= kPre2;
    CI xs[kPre2];
    CI prod = ci_id();
    if (pre) {
#pragma unroll
        for (int i = 0; i < kPre2; ++i) {
            const int4 x = cc[cnt > 0 ? b0 + (i < cnt ? i : 0) : 0];
            xs[i] = CI{x.x, x.y, x.z, x.w};
        }
#pragma unroll
        for (int i = 0; i < kPre2; ++i)
            if (i < cnt) prod = ci_mul(prod, xs[i]);
    } else {
        for (int64_t k = b0; k < b1; ++k) {
            const int4 x = cc[k];
            prod = ci_mul(prod, CI{x.x, x.y, x.z, x.w});
        }
    }
    // exclusive scan of the lanes' products: shuffles inside each wave, then the wave totals
    const int lane = t & 63, wv = t >> 6;
    CI x = prod;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const CI y = shfl_up_ci(x, off);
        if (lane >= off) x = ci_mul(y, x);
    }
    const CI up1 = shfl_up_ci(x, 1);
    if (lane == 63) buf[wv] = x;
    __syncthreads();
    CI excl = ci_id();
    for (int w = 0; w < wv; ++w) excl = ci_mul(excl, buf[w]);
    if (lane > 0) excl = ci_mul(excl, up1);
    const int f = vc.qshift;
    int64_t P = fix_of(lp, f), M = fix_of(lm, f);
    if (t > 0) ci_apply(P, M, excl);
    auto block = [&](int64_t k, const CI& x) {
        const longlong2 en = make_longlong2(P, M);
        ci_apply(P, M, x);
        bool irregular;
        pl[k] = classify(vc, g, k, en, make_longlong2(P, M), irregular);
        if (irregular) {   // only K3b reads the entry estimates (one workgroup writes a
                           // chunk's records at one CU's share of the memory system)
            ae[k] = en;
            irrlist[c * g.nsb + atomicAdd(&sIrr, 1)] = (int32_t)k;
        }
    };
    if (pre) {
#pragma unroll
        for (int i = 0; i < kPre2; ++i)
            if (i < cnt) block(b0 + i, xs[i]);
    } else {
        for (int64_t k = b0; k < b1; ++k) {
            const int4 x = cc[k];
            block(k, CI{x.x, x.y, x.z, x.w});
        }
    }
    __syncthreads();
    if (t == 0) irrcount[c] = sIrr;
}

// K2 of the segment path, one workgroup per segment: the segment's entry estimate (the chunk's
// start times the products of its earlier segments, stored by K1), the exclusive scan of its
// blocks' composites (exact integer max-plus), the classification of its blocks; irregular
// blocks go to the segment's list.
__global__ __launch_bounds__(kThreads) void k_vit_segplan(VitConsts vc, const uint32_t* packed,
                                                          Geo g, const int4* __restrict__ comp,
                                                          ApproxSeg as) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int64_t gid = (int64_t)blockIdx.x * kThreads + t;
    const int64_t c = gid / g.nsb, k = gid - c * g.nsb;
    const int sidx = (int)(k / kThreads);   // segment within the chunk (workgroup-uniform)
    const uint32_t* pk = chunk_ptr(packed, g, c);
    const uint32_t o0 = base_at(pk, 0);
    const double lp = vc.logpi[o0], lm = vc.logpi[o0 + 4];
    if (!(lp > -INFINITY) && !(lm > -INFINITY)) {   // DEGEN chunk (uniform)
        as.plan[gid] = VitPlan{PLAN_DEGEN, 0, 0, 0, 0, 0};
        if (t == 0) {
            as.irrseg[blockIdx.x] = 0;
            if (sidx == 0) as.degen[c] = 1;
        }
        return;
    }
    if (t == 0 && sidx == 0) as.degen[c] = 0;
    const int4 x4 = comp[gid];
    const CI x{x4.x, x4.y, x4.z, x4.w};
    __shared__ CI sPre[kMaxSeg];
    __shared__ CI sW[kThreads / 64];
    __shared__ longlong2 sEnt;
    __shared__ int sIrr;
    if (t < sidx) sPre[t] = as.segprod[(int64_t)blockIdx.x - sidx + t];
    // inclusive scan of the segment's composites
    CI s = x;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const CI y = shfl_up_ci(s, off);
        if (lane >= off) s = ci_mul(y, s);
    }
    if (lane == 63) sW[wv] = s;
    if (t == 0) sIrr = 0;
    __syncthreads();
    CI before = ci_id();
    for (int w = 0; w < wv; ++w) before = ci_mul(before, sW[w]);
    const CI up = shfl_up_ci(s, 1);
    const CI excl = lane > 0 ? ci_mul(before, up) : before;
    if (t == 0) {   // the segment's entry estimate
        const int f = vc.qshift;
        int64_t P = fix_of(lp, f), M = fix_of(lm, f);
        for (int j = 0; j < sidx; ++j) ci_apply(P, M, sPre[j]);
        sEnt = make_longlong2(P, M);
    }
    __syncthreads();
    int64_t P = sEnt.x, M = sEnt.y;
    ci_apply(P, M, excl);
    const longlong2 en = make_longlong2(P, M);
    ci_apply(P, M, x);
    bool irregular;
    as.plan[gid] = classify(vc, g, k, en, make_longlong2(P, M), irregular);
    if (irregular) {
        as.aent[c * (g.nsb + 1) + k] = en;
        as.irrlist[(int64_t)blockIdx.x * kThreads + atomicAdd(&sIrr, 1)] = (int32_t)k;
    }
    __syncthreads();
    if (t == 0) as.irrseg[blockIdx.x] = sIrr;
}

// ---------------------------------------------------------------- K3: exact composites
// comp3: the pre composites of all blocks [nchunks * nsb], then the post composites [same];
// a block's post is written (and read) for SPLIT blocks only, so K4's one workgroup per chunk
// streams dense pre records, not every other 32 B of a 64-B pair
// largest finite magnitude (the identity's -inf entries carry no rounding)
__device__ __forceinline__ double fin(double x) { return x > -INFINITY ? fabs(x) : 0.0; }
__device__ __forceinline__ double c64_absmax(const C64& c) {
    return fmax(fmax(fin(c.pp), fin(c.pm)), fmax(fin(c.mp), fin(c.mm)));
}
__device__ __forceinline__ bool c64_exact(const C64& c, int e, double spread) {
    return c64_absmax(c) + spread < ldexp(1.0, e + 1);
}

__device__ void vit_irregular(const VitConsts& vc, const uint32_t* packed, const Geo& g,
                              const longlong2* __restrict__ aent, VitPlan* __restrict__ plan,
                              const int32_t* __restrict__ irrlist,
                              const int32_t* __restrict__ irrcount,
                              double4* __restrict__ comp3, int64_t c, const double2* sA,
                              const double2* sB, const int32_t* __restrict__ irrseg);

// Segment path (chunks of a multiple of 256 blocks, e.g. 1 Mi): each regular workgroup (256
// blocks of one chunk = one "segment") also runs a segmented scan of its exact composites,
// barriers (every non-REGULAR block) resetting it, and writes per block rx = the product of
// the REGULAR composites between the last barrier before it in the segment (or the segment
// start) and the block, plus a SegSum (barrier mask, lead = product before the first barrier,
// tail = product after the last).  K4 then touches only the barriers and 16 summaries per
// chunk, and K5 derives every block's entry from rx and its anchor (the last barrier before
// it, or the segment's entry): no per-chunk pass over every block's records.
struct SegSum {
    double4 lead, tail;
    unsigned long long mask[4];   // bit l: block (segment start + l) is a barrier
};
__device__ __forceinline__ C64 shfl_up_c64(const C64& x, int d) {
    return {__shfl_up(x.pp, d), __shfl_up(x.pm, d), __shfl_up(x.mp, d), __shfl_up(x.mm, d)};
}

__global__ __launch_bounds__(kThreads) void k_vit_exact(VitConsts vc, const VitTables* vt,
                                                        const uint32_t* packed, Geo g,
                                                        VitPlan* __restrict__ plan,
                                                        double4* __restrict__ comp3,
                                                        uint32_t* status, unsigned main_grid,
                                                        const longlong2* __restrict__ aent,
                                                        const int32_t* __restrict__ irrlist,
                                                        const int32_t* __restrict__ irrcount,
                                                        double4* __restrict__ rx,
                                                        SegSum* __restrict__ seg,
                                                        const int32_t* __restrict__ irrseg,
                                                        double2* __restrict__ vhead) {
    // per binade slot: single-step halves sA/sB [16] (one 256-B bank row each) and 2-step
    // composites over 3-base windows, halves P2A = (pp, pm), P2B = (mp, mm) [64].  Every
    // entry is a sum of binade-rounded constants: exact on the binade's grid.
    // LDS: single-step halves of every binade [emin, emax] (partial blocks, the irregular
    // blocks' workgroups), then a union: the 4-step composites of ONE binade (when every
    // full REGULAR block of the workgroup lies in it: 64 lookups and max-plus products per
    // block instead of 128) or the 2-step composites of every binade
    extern __shared__ __attribute__((aligned(16))) double2 sLe[];
    const int nb = vc.emax - vc.emin + 1;
    // segment path (no partial blocks): ONE 32 KB union holds the table the workgroup uses —
    // the single-step rows (irregular-block workgroups), the 4-step composites of one binade,
    // or the 2-step rows of the segment's binade range only — 4 workgroups per CU instead of
    // 3 (K3 1.23 -> 1.15 ms at 3.1 Gbp, profiles/r04_k3range/)
    const bool compact = seg != nullptr;
    double2* sA = sLe;
    double2* sB = sA + nb * 16;
    double2* P2A = compact ? sLe : sB + nb * 16;
    double2* P2B = P2A + nb * 64;
    double2* P4A = compact ? sLe : sB + nb * 16;
    double2* P4B = P4A + kW4;
    __shared__ int s_emin, s_emax, s_part;
    const VitDerived* dv = derived(vt);
    auto load_single = [&]() {   // the single-step halves of every binade
        for (int i = threadIdx.x; i < nb * 16; i += kThreads) {
            sA[i] = dv->sA[vc.emin * 16 + i];
            sB[i] = dv->sB[vc.emin * 16 + i];
        }
    };
    if (blockIdx.x >= main_grid + g.nchunks) {   // segment path: block 0's walk (K2's heads)
        vit_head(vc, packed, g,
                 (int64_t)(blockIdx.x - main_grid - g.nchunks) * kThreads + threadIdx.x, vhead);
        return;
    }
    if (blockIdx.x >= main_grid) {   // workgroup-uniform: the chunk's irregular blocks
        load_single();
        __syncthreads();
        vit_irregular(vc, packed, g, aent, plan, irrlist, irrcount, comp3,
                      (int64_t)(blockIdx.x - main_grid), sA, sB, irrseg);
        return;
    }
    if (threadIdx.x == 0) {
        s_emin = 1 << 30;
        s_emax = -(1 << 30);
        s_part = 0;
    }
    __syncthreads();
    const int64_t gid = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    const bool valid = gid < g.nchunks * g.nsb;
    const VitPlan p = valid ? plan[gid] : VitPlan{PLAN_SEQ, 0, 0, 0, 0, 0};
    const int64_t c = valid ? gid / g.nsb : 0, k = valid ? gid - c * g.nsb : 0;
    const bool reg = valid && p.type == PLAN_REGULAR;
    // a partial REGULAR block (the chunk's last, short one) walks single steps
    if (reg && !g.full(k)) s_part = 1;
    {   // binade range of the workgroup's full REGULAR blocks: wave reduction, one LDS atomic
        int lo = (reg && g.full(k)) ? (int)p.e_pre : (1 << 30);
        int hi = (reg && g.full(k)) ? (int)p.e_pre : -(1 << 30);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            lo = min(lo, __shfl_xor(lo, off));
            hi = max(hi, __shfl_xor(hi, off));
        }
        if ((threadIdx.x & 63) == 0) {
            atomicMin(&s_emin, lo);
            atomicMax(&s_emax, hi);
        }
    }
    __syncthreads();
    const bool four = s_emin == s_emax;   // workgroup-uniform
    if (s_part) load_single();   // (tables only where a workgroup uses them: ~11 KB each)
    if (four) {
        const double2* ga = dv->P4A + (size_t)s_emin * kW4;
        const double2* gb = dv->P4B + (size_t)s_emin * kW4;
        for (int i = threadIdx.x; i < kW4; i += kThreads) {
            P4A[i] = ga[i];
            P4B[i] = gb[i];
        }
    } else if (!compact) {
        for (int i = threadIdx.x; i < nb * 64; i += kThreads) {
            P2A[i] = dv->P2A[vc.emin * 64 + i];
            P2B[i] = dv->P2B[vc.emin * 64 + i];
        }
    }
    // compact: the 2-step rows of the segment's binade range only (<= 16 binades: 32 KB)
    const int nrange = s_emax - s_emin + 1;
    const bool glob2 = compact && !four && nrange > kW4 / 64;   // (rows from device memory)
    if (compact && !four && !glob2 && nrange > 0) {
        P2B = P2A + nrange * 64;
        for (int i = threadIdx.x; i < nrange * 64; i += kThreads) {
            P2A[i] = dv->P2A[(size_t)s_emin * 64 + i];
            P2B[i] = dv->P2B[(size_t)s_emin * 64 + i];
        }
    }
    __syncthreads();
    if (!reg && !seg) return;   // (segment path: every lane takes part in the scan below)
    const uint32_t* pk = chunk_ptr(packed, g, c);
    const int slot = p.e_pre - (compact ? s_emin : vc.emin);
    C64 acc = c64_id();
    if (!reg) {
    } else if (g.full(k) && four) {
        const BlockWords bw = load_block(pk, k);
        pipelined<4, 64>(
            [&](int j) {   // 5-base window of steps 4j .. 4j+3
                const int r = j >> 2, s = j & 3;
                const uint32_t lo = r == 0 ? bw.prev : bw.w[r - 1];
                return s == 0 ? (__builtin_amdgcn_alignbit(bw.w[r], lo, 30) & 0x3FFu)
                              : ((bw.w[r] >> (8 * s - 2)) & 0x3FFu);
            },
            [&](uint32_t wi) { return C64{P4A[wi].x, P4A[wi].y, P4B[wi].x, P4B[wi].y}; },
            [&](const C64& m, int) { acc = c64_mul(acc, m); });
    } else if (g.full(k) && glob2) {
        const double2* pa = dv->P2A + (size_t)p.e_pre * 64;
        const double2* pb = dv->P2B + (size_t)p.e_pre * 64;
        const BlockWords bw = load_block(pk, k);
        pipelined<4, 128>(
            [&](int j) {   // 3-base window of steps 2j, 2j+1
                const int r = j >> 3, s = j & 7;
                const uint32_t lo = r == 0 ? bw.prev : bw.w[r - 1];
                return s == 0 ? (__builtin_amdgcn_alignbit(bw.w[r], lo, 30) & 63u)
                              : ((bw.w[r] >> (4 * s - 2)) & 63u);
            },
            [&](uint32_t wi) { return C64{pa[wi].x, pa[wi].y, pb[wi].x, pb[wi].y}; },
            [&](const C64& m, int) { acc = c64_mul(acc, m); });
    } else if (g.full(k)) {
        const double2* pa = P2A + slot * 64;
        const double2* pb = P2B + slot * 64;
        const BlockWords bw = load_block(pk, k);
        pipelined<4, 128>(
            [&](int j) {   // 3-base window of steps 2j, 2j+1
                const int r = j >> 3, s = j & 7;
                const uint32_t lo = r == 0 ? bw.prev : bw.w[r - 1];
                return s == 0 ? (__builtin_amdgcn_alignbit(bw.w[r], lo, 30) & 63u)
                              : ((bw.w[r] >> (4 * s - 2)) & 63u);
            },
            [&](uint32_t wi) { return C64{pa[wi].x, pa[wi].y, pb[wi].x, pb[wi].y}; },
            [&](const C64& m, int) { acc = c64_mul(acc, m); });
    } else {
        const double2* ta = sA + slot * 16;
        const double2* tb = sB + slot * 16;
        walk_block<false>(pk, k, g.C, [&](uint32_t d, int, int) {
            const double2 a = ta[d], b = tb[d];
            c64_step(acc, a.x, a.y, b.x, b.y);
        });
    }
    const bool exact = reg && c64_exact(acc, p.e_pre, vc.spread);
    // exactness not guaranteed: K4 runs the block sequentially
    if (reg && !exact) plan[gid].type = PLAN_SEQ;
    if (!seg) {
        if (exact) comp3[gid] = make_double4(acc.pp, acc.pm, acc.mp, acc.mm);
        return;
    }
    // segmented inclusive scan (element: the composite, or a reset + identity at a barrier)
    const bool bar = !exact;   // (all lanes valid: nsb % 256 == 0)
    C64 m = exact ? acc : c64_id();
    int fl = bar ? 1 : 0;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const C64 ym = shfl_up_c64(m, off);
        const int yf = __shfl_up(fl, off);
        if (lane >= off) {
            if (!fl) m = c64_mul(ym, m);
            fl |= yf;
        }
    }
    __shared__ C64 sWm[kThreads / 64];
    __shared__ int sWf[kThreads / 64];
    __shared__ unsigned long long sMask[kThreads / 64];
    const unsigned long long bmask = __ballot(bar);
    if (lane == 63) {
        sWm[wv] = m;
        sWf[wv] = fl;
    }
    if (lane == 0) sMask[wv] = bmask;
    __syncthreads();
    C64 before = c64_id();   // the waves before this one
    for (int w = 0; w < wv; ++w) before = sWf[w] ? sWm[w] : c64_mul(before, sWm[w]);
    const C64 inc = fl ? m : c64_mul(before, m);
    C64 ex = shfl_up_c64(inc, 1);
    if (lane == 0) ex = before;
    rx[gid] = make_double4(ex.pp, ex.pm, ex.mp, ex.mm);
    SegSum& sg = seg[blockIdx.x];
    int fb = -1;   // the segment's first barrier
#pragma unroll
    for (int w = kThreads / 64 - 1; w >= 0; --w)
        if (sMask[w]) fb = w * 64 + (int)__builtin_ctzll(sMask[w]);
    if ((int)threadIdx.x == fb) sg.lead = make_double4(ex.pp, ex.pm, ex.mp, ex.mm);
    if (threadIdx.x == kThreads - 1) {
        sg.tail = make_double4(inc.pp, inc.pm, inc.mp, inc.mm);
        if (fb < 0) sg.lead = make_double4(inc.pp, inc.pm, inc.mp, inc.mm);
    }
    if (threadIdx.x < kThreads / 64) sg.mask[threadIdx.x] = sMask[threadIdx.x];
}

// K3b: irregular blocks, 16 lanes per block (lane i owns positions [16i, 16i+16)):
//   locate — fixed-point composites of the 16-position pieces, a 16-lane scan of them from
//            the block's approximate entry, then every lane checks its own 16 steps:
//            t1 = first step outside binade e, t2 = 1 + last step outside binade e+1;
//   split  — exact composites of the steps before t1 (binade e) and from t2 on (binade
//            e+1), per lane, multiplied in order by a 16-lane scan (exact max-plus).
// Result: SPLIT (pre composite, window [t1, t2), post composite) or SEQ.
__device__ __forceinline__ CI shfl_ci(const CI& x, int src) {
    return {__shfl(x.pp, src), __shfl(x.pm, src), __shfl(x.mp, src), __shfl(x.mm, src)};
}
__device__ __forceinline__ C64 shfl_c64(const C64& x, int src) {
    return {__shfl(x.pp, src), __shfl(x.pm, src), __shfl(x.mp, src), __shfl(x.mm, src)};
}

// the 16 steps of piece i of block k: f(d, j) with j the position offset in the block
template <class F>
__device__ __forceinline__ void walk_piece(const uint32_t* __restrict__ pk, int64_t k, int i,
                                           int j0, int jend, F&& f) {
    const int64_t wbase = k * kSBWords + i;
    const uint32_t w = (k * kSB + i * 16 < (int64_t)jend + k * kSB) ? pk[wbase] : 0u;
    const uint32_t prev = (k > 0 || i > 0) ? pk[wbase - 1] : 0u;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
        const int j = i * 16 + s;
        const uint32_t d = (s == 0) ? (__builtin_amdgcn_alignbit(w, prev, 30) & 15u)
                                    : ((w >> (2 * s - 2)) & 15u);
        if (j >= j0 && j < jend) f(d, j);
    }
}

// Runs in K3's launch as one extra workgroup per chunk (concurrently with the regular
// blocks' composites); sA/sB: K3's single-step binade tables [e - emin][16]
__device__ void vit_irregular(const VitConsts& vc, const uint32_t* packed, const Geo& g,
                              const longlong2* __restrict__ aent, VitPlan* __restrict__ plan,
                              const int32_t* __restrict__ irrlist,
                              const int32_t* __restrict__ irrcount,
                              double4* __restrict__ comp3, int64_t c, const double2* sA,
                              const double2* sB, const int32_t* __restrict__ irrseg) {
    __shared__ int4 Q[16];
    // segment path: the chunk's segments' lists (K1), concatenated through their offsets
    __shared__ int sOffI[kMaxSeg + 1];
    const int nseg = (int)(g.nsb / kThreads);
    if (irrseg) {
        if (threadIdx.x == 0) {
            int o = 0;
            for (int j = 0; j < nseg; ++j) {
                sOffI[j] = o;
                o += irrseg[c * nseg + j];
            }
            sOffI[nseg] = o;
        }
        __syncthreads();
    }
    const int n = irrseg ? sOffI[nseg] : irrcount[c];
    if (n == 0) return;   // workgroup-uniform
    const int nb = vc.emax - vc.emin + 1;
    if (threadIdx.x < 16)
        Q[threadIdx.x] = make_int4(vc.Q[threadIdx.x][0], vc.Q[threadIdx.x][1],
                                   vc.Q[threadIdx.x][2], vc.Q[threadIdx.x][3]);
    __syncthreads();
    const uint32_t* pk = chunk_ptr(packed, g, c);
    const int lane = threadIdx.x & 63;
    const int gi = lane & 15;                       // piece index within the block
    const int gbase = (threadIdx.x & ~15);          // first thread of the 16-lane group
    const int gsrc = lane & ~15;                    // first lane of the group in the wave
    const int group = threadIdx.x >> 4;             // 16 groups per workgroup
    for (int it = group; it < n; it += 16) {
        (void)gbase;
        int64_t k;
        if (irrseg) {
            int j = 0;
            while (j + 1 < nseg && sOffI[j + 1] <= it) ++j;
            k = irrlist[(c * nseg + j) * kThreads + (it - sOffI[j])];
        } else {
            k = irrlist[c * g.nsb + it];
        }
        const int64_t gid = c * g.nsb + k;
        const int j0 = g.jfirst(k), jend = g.jend(k);
        const longlong2 en = aent[c * (g.nsb + 1) + k];
        const double invS = ldexp(1.0, -vc.qshift);
        const double epsc = vc.eps + invS;
        const double hi = (double)mx(en.x, en.y) * invS + vc.eps;
        const int e = ilogb(-hi);
        const bool okA = binade_ok(vc, e), okB = binade_ok(vc, e + 1);
        const double S = ldexp(1.0, vc.qshift);
        // binade conditions as fixed-point thresholds (see K2b)
        const int64_t HA = (int64_t)floor((-ldexp(1.0, e) - epsc) * S);
        const int64_t LA = (int64_t)floor((-ldexp(1.0, e + 1) + epsc) * S);
        const int64_t HB = (int64_t)floor((-ldexp(1.0, e + 1) - epsc) * S);
        const int64_t LB = (int64_t)floor((-ldexp(1.0, e + 2) + epsc) * S);
        // locate: piece composite -> group scan -> entry of the piece
        CI pc = ci_id();
        walk_piece(pk, k, gi, j0, jend, [&](uint32_t d, int) {
            const int4 q = Q[d];
            pc = CI{cl(mx(pc.pp + q.x, pc.pm + q.y)), cl(mx(pc.pp + q.z, pc.pm + q.w)),
                    cl(mx(pc.mp + q.x, pc.mm + q.y)), cl(mx(pc.mp + q.z, pc.mm + q.w))};
        });
        CI sc = pc;
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
            const CI o = shfl_ci(sc, gsrc + ((gi - off) & 15));
            if (gi >= off) sc = ci_mul(o, sc);
        }
        const CI ex = shfl_ci(sc, gsrc + ((gi - 1) & 15));
        int64_t aP = en.x, aM = en.y;
        if (gi > 0) ci_apply(aP, aM, ex);
        int t1 = 1 << 20, lastbad = -1;
        walk_piece(pk, k, gi, j0, jend, [&](uint32_t d, int j) {
            const int4 q = Q[d];
            const int64_t c0 = aP + q.x, c1 = aM + q.y, c2 = aP + q.z, c3 = aM + q.w;
            const int64_t vmax = mx(aP, aM);
            const int64_t vmin = min(min(min(c0, c1), min(c2, c3)), min(aP, aM));
            const bool regA = okA && vmax <= HA && vmin > LA;
            const bool regB = okB && vmax <= HB && vmin > LB;
            if (!regA && j < t1) t1 = j;
            if (!regB) lastbad = j;
            aP = mx(c0, c1);
            aM = mx(c2, c3);
        });
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
            t1 = min(t1, __shfl_xor(t1, off));
            lastbad = max(lastbad, __shfl_xor(lastbad, off));
        }
        if (t1 > jend) t1 = jend;
        int t2 = max(lastbad + 1, j0);
        if (!okA) t1 = j0;
        if (!okB) t2 = jend;
        if (t2 < t1) t2 = t1;
        const bool split = !(t1 == j0 && t2 == jend);
        bool exact = split;
        C64 pre = c64_id(), post = c64_id();
        if (split) {
            const int ia = max(0, min(nb - 1, e - vc.emin)) * 16;
            const int ib = max(0, min(nb - 1, e + 1 - vc.emin)) * 16;
            // two walks, one per composite: a step choosing between `pre` and `post` at run
            // time makes the compiler address them through memory (scratch)
            walk_piece(pk, k, gi, j0, jend, [&](uint32_t d, int j) {
                if (j < t1) {
                    const double2 a = sA[ia + d], b = sB[ia + d];
                    c64_step(pre, a.x, a.y, b.x, b.y);
                }
            });
            walk_piece(pk, k, gi, j0, jend, [&](uint32_t d, int j) {
                if (j >= t2) {
                    const double2 a = sA[ib + d], b = sB[ib + d];
                    c64_step(post, a.x, a.y, b.x, b.y);
                }
            });
            // ordered products over the group (exact: same binade grid throughout)
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) {
                const C64 o1 = shfl_c64(pre, gsrc + ((gi - off) & 15));
                const C64 o2 = shfl_c64(post, gsrc + ((gi - off) & 15));
                if (gi >= off) {
                    pre = c64_mul(o1, pre);
                    post = c64_mul(o2, post);
                }
            }
            pre = shfl_c64(pre, gsrc + 15);
            post = shfl_c64(post, gsrc + 15);
            exact = c64_exact(pre, e, vc.spread) && c64_exact(post, e + 1, vc.spread);
        }
        if (gi == 0) {
            if (exact) {
                plan[gid] = VitPlan{PLAN_SPLIT, (int8_t)e, (int8_t)(e + 1), 0, (uint16_t)t1,
                                    (uint16_t)t2};
                comp3[gid] = make_double4(pre.pp, pre.pm, pre.mp, pre.mm);
                comp3[g.nchunks * g.nsb + gid] = make_double4(post.pp, post.pm, post.mp, post.mm);
            } else {
                plan[gid] = VitPlan{PLAN_SEQ, 0, 0, 0, 0, 0};
            }
        }
    }
}

// ---------------------------------------------------------------- K4: chain
__device__ __forceinline__ C64 ld_c64(const double4* p) {
    const double4 x = *p;
    return {x.x, x.y, x.z, x.w};
}
__device__ __forceinline__ void st_c64(double4* p, const C64& c) {
    *p = make_double4(c.pp, c.pm, c.mp, c.mm);
}

// The serial chain: wave 0 stages the constants of a window's steps in LDS (lanes in
// parallel), then lane 0 runs the reference recurrence over them; the LDS reads do not
// depend on the chain, so they issue ahead of it.
constexpr int kChainT = 1024;
constexpr int kMaxStagedBar = 64;     // barriers staged in LDS per chunk
constexpr int kStageSteps = 512;      // window steps staged in LDS per chunk (block 0
                                      // is walked by K2's head lanes, not here)
__device__ __forceinline__ double2 chain_window(const uint32_t* __restrict__ pk,
                                                const double4* sL, double4* stepL, int64_t k,
                                                int ja, int jb, double2 v, int lane) {
    const int n = jb - ja;
    if (n <= 0) return v;
    for (int j = lane; j < n; j += 64) {
        const int64_t pos = k * kSB + ja + j;
        const uint32_t d = base_at(pk, pos - 1) | (base_at(pk, pos) << 2);
        stepL[j] = sL[d];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    double P = v.x, M = v.y;
    if (lane == 0) {
#pragma unroll 8
        for (int j = 0; j < n; ++j) {
            const double4 l = stepL[j];
            const Step s = ref_step(P, M, l.x, l.y, l.z, l.w);
            P = s.P;
            M = s.M;
        }
    }
    __builtin_amdgcn_wave_barrier();
    return make_double2(__shfl(P, 0), __shfl(M, 0));
}

__global__ __launch_bounds__(kChainT) void k_vit_chain(
    VitConsts vc, const uint32_t* packed, Geo g, const VitPlan* __restrict__ plan,
    const double4* __restrict__ comp3, const uint8_t* __restrict__ degen,
    double2* __restrict__ entry, double4* __restrict__ gk, double4* __restrict__ gap,
    int32_t* __restrict__ barlist, double2* __restrict__ vout,
    const double2* __restrict__ vhead) {
    const int64_t c = blockIdx.x;
    const int t = threadIdx.x;
    const int64_t per = (g.nsb + kChainT - 1) / kChainT;
    const int64_t b0 = min((int64_t)t * per, g.nsb), b1 = min(b0 + per, g.nsb);
    double2* ent = entry + c * (g.nsb + 1);
    __shared__ double4 sL[16];
    __shared__ double4 stepL[kSB];
    __shared__ double4 stageL[kStageSteps];
    if (t < 16) sL[t] = make_double4(vc.L[t][0], vc.L[t][1], vc.L[t][2], vc.L[t][3]);
    if (degen[c]) {
        for (int64_t k = b0; k < b1; ++k) ent[k] = make_double2(-INFINITY, -INFINITY);
        if (t == kChainT - 1) ent[g.nsb] = make_double2(-INFINITY, -INFINITY);
        return;
    }
    const uint32_t* pk = chunk_ptr(packed, g, c);
    const VitPlan* pl = plan + c * g.nsb;
    const double4* cp = comp3 + c * g.nsb;                          // pre composites
    const double4* cq = comp3 + (g.nchunks + c) * g.nsb;            // post (SPLIT only)
    double4* gkc = gk + c * g.nsb;
    double4* gpc = gap + c * g.nsb;
    int32_t* blc = barlist + c * g.nsb;
    double2* voc = vout + c * g.nsb;

    // block 0's exit value (K2's head lanes), needed by the serial chain: read now, so that its
    // latency is not on the chain
    const double2 vhead0 = t == 0 ? vhead[c] : make_double2(0.0, 0.0);
    // phase 1: thread-local pieces.  A thread owns `per` (<= kPre for chunks up to 1 Mi)
    // consecutive blocks; their plans and composites are loaded up front, all in flight.
    constexpr int kPre = 4;
    const int cnt = (int)(b1 - b0);
    const bool pre = cnt > 0 && cnt <= kPre;   // cnt == 0: the generic loops do nothing
    // block b0 + i's plan and composites (i < cnt; callers unroll i)
// (the post composites are read for SPLIT blocks only: this one workgroup per chunk streams
// its chunk's block records at one CU's share of the memory system)
#define CPG_PREFETCH(P, A)                                     \
    VitPlan P[kPre];                                           \
    C64 A[kPre];                                               \
    _Pragma("unroll") for (int i = 0; i < kPre; ++i) {         \
        const int64_t kk = b0 + (i < cnt ? i : 0);             \
        P[i] = pl[kk];                                         \
        A[i] = ld_c64(cp + kk);                                \
    }
    C64 run = c64_id(), lead = c64_id();
    bool hasb = false;
    int nb = 0;
    auto piece = [&](int64_t k, const VitPlan& p, const C64& ca, const C64& cb) {
        if (p.type == PLAN_REGULAR) {
            run = c64_mul(run, ca);
        } else {
            if (p.type == PLAN_SPLIT) run = c64_mul(run, ca);
            if (!hasb) lead = run;
            else st_c64(gkc + k, run);
            hasb = true;
            ++nb;
            run = (p.type == PLAN_SPLIT) ? cb : c64_id();
        }
    };
    // phase 4 needs, per block, the composite applied after its entry (REGULAR: pre, SPLIT:
    // post) and the block's kind: kept in LDS and a register from phase 1 (chunks up to 1 Mi)
    // instead of reading the chunk's records from global memory a second time
    __shared__ double4 sApp[kPre * kChainT];
    uint32_t kinds = 0;   // 2 bits per block of the thread (1 REGULAR, 2 SPLIT, 3 SEQ)
    uint32_t wab[kPre] = {};   // barrier blocks' window [ja, jb) as ja | jb << 16
    // phase 3's staging metadata (first kMaxStagedBar barriers), written by phase 2's list
    // loop straight from registers when every thread's blocks were prefetched (chunks up to
    // 1 Mi): no global round trip through the barrier list and the plans before the chain
    __shared__ int sWoff[kMaxStagedBar + 1];
    __shared__ int sWa[kMaxStagedBar], sWb[kMaxStagedBar];
    __shared__ int64_t sWk[kMaxStagedBar];
    __shared__ C64 sGap[kMaxStagedBar];
    const bool pre_all = per <= kPre;   // uniform: every thread with blocks prefetched them
    if (pre) {
        CPG_PREFETCH(xp, xa)
#pragma unroll
        for (int i = 0; i < kPre; ++i)
            if (i < cnt) {
                const int64_t k = b0 + i;
                const bool reg = xp[i].type == PLAN_REGULAR, spl = xp[i].type == PLAN_SPLIT;
                // the post composite: SPLIT blocks only (rare; its load latency stays local)
                const C64 xb = spl ? ld_c64(cq + k) : c64_id();
                piece(k, xp[i], xa[i], xb);
                sApp[k] = spl ? make_double4(xb.pp, xb.pm, xb.mp, xb.mm)
                              : make_double4(xa[i].pp, xa[i].pm, xa[i].mp, xa[i].mm);
                const bool seq = xp[i].type == PLAN_SEQ;
                kinds |= (reg ? 1u : spl ? 2u : seq ? 3u : 0u) << (2 * i);
                const uint32_t ja = spl ? xp[i].t1 : g.jfirst(k), jb = spl ? xp[i].t2 : g.jend(k);
                wab[i] = k == 0 ? 0u : (ja | (jb << 16));   // block 0: walked by K2's head lanes
            }
    } else {
        for (int64_t k = b0; k < b1; ++k)
            piece(k, pl[k], ld_c64(cp + k), ld_c64(cq + k));
    }
    if (!hasb) lead = run;
    // phase 2: segmented scan of (hasb, trail) + barrier count scan: shuffle scans inside
    // each wave, then the 16 wave totals (exact max-plus products: any association)
    struct Seg {
        C64 m;
        int fl, n;
    };
    auto seg_comb = [](const Seg& a, const Seg& b) {   // a before b
        return Seg{b.fl ? b.m : c64_mul(a.m, b.m), a.fl | b.fl, a.n + b.n};
    };
    auto seg_shfl_up = [](const Seg& x, int d) {
        return Seg{{__shfl_up(x.m.pp, d), __shfl_up(x.m.pm, d), __shfl_up(x.m.mp, d),
                    __shfl_up(x.m.mm, d)},
                   __shfl_up(x.fl, d), __shfl_up(x.n, d)};
    };
    const int lane = t & 63, wv = t >> 6;
    Seg x{run, hasb ? 1 : 0, nb};
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const Seg y = seg_shfl_up(x, d);
        if (lane >= d) x = seg_comb(y, x);
    }
    __shared__ Seg sWave[kChainT / 64];
    if (lane == 63) sWave[wv] = x;
    __syncthreads();
    Seg before{c64_id(), 0, 0};   // everything before this wave
    for (int w = 0; w < wv; ++w) before = seg_comb(before, sWave[w]);
    const Seg prev = seg_shfl_up(x, 1);   // inclusive value of the lane before
    const Seg excl = lane > 0 ? seg_comb(before, prev) : before;
    const C64 incoming = excl.m;
    const int bidx0 = excl.n;
    int nbar = 0;
    for (int w = 0; w < kChainT / 64; ++w) nbar += sWave[w].n;
    if (pre) {   // the kinds from phase 1: no second read of the plans
        int idx = bidx0;
        bool first = true;
#pragma unroll
        for (int i = 0; i < kPre; ++i) {
            const int64_t k = b0 + i;
            if (i < cnt && ((kinds >> (2 * i)) & 3u) >= 2u) {
                const C64 gp = first ? c64_mul(incoming, lead) : ld_c64(gkc + k);
                blc[idx] = (int32_t)k;
                st_c64(gpc + idx, gp);
                if (idx < kMaxStagedBar) {
                    sWk[idx] = k;
                    sWa[idx] = (int)(wab[i] & 0xFFFFu);
                    sWb[idx] = (int)(wab[i] >> 16);
                    sGap[idx] = gp;
                }
                first = false;
                ++idx;
            }
        }
    } else {
        int idx = bidx0;
        bool first = true;
        for (int64_t k = b0; k < b1; ++k) {
            const VitPlan p = pl[k];
            if (p.type == PLAN_SPLIT || p.type == PLAN_SEQ) {
                blc[idx] = (int32_t)k;
                if (first) st_c64(gpc + idx, c64_mul(incoming, lead));
                else st_c64(gpc + idx, ld_c64(gkc + k));
                first = false;
                ++idx;
            }
        }
    }
    __syncthreads();
    // phase 3: the serial chain over barriers.  The whole workgroup first stages every
    // window's step constants and every gap composite in LDS, so lane 0's serial
    // recurrence never waits on global memory; windows beyond the staging capacity fall
    // back to per-window staging by wave 0.
    const uint32_t o0 = base_at(pk, 0);
    const double2 init = make_double2(vc.logpi[o0], vc.logpi[o0 + 4]);
    const int nst = min(nbar, kMaxStagedBar);
    if (!pre_all && t < nst) {
        const int64_t k = blc[t];
        const VitPlan p = pl[k];
        sWk[t] = k;
        sWa[t] = p.type == PLAN_SPLIT ? p.t1 : g.jfirst(k);
        sWb[t] = p.type == PLAN_SPLIT ? p.t2 : g.jend(k);
        if (k == 0) sWa[t] = sWb[t] = 0;   // block 0: walked by K2's head lanes
        sGap[t] = ld_c64(gpc + t);
    }
    __syncthreads();
    if (t == 0) {
        int o = 0;
        for (int i = 0; i < nst; ++i) {
            sWoff[i] = o;
            const int len = max(0, sWb[i] - sWa[i]);
            o = (o + len <= kStageSteps) ? o + len : kStageSteps + 1;   // overflow marker
        }
        sWoff[nst] = o;
    }
    __syncthreads();
    for (int i = t >> 6; i < nst; i += kChainT / 64) {   // one wave per window
        const int off = sWoff[i];
        const int len = max(0, sWb[i] - sWa[i]);
        if (off + len > kStageSteps) continue;
        for (int j = t & 63; j < len; j += 64) {
            const int64_t pos = sWk[i] * kSB + sWa[i] + j;
            const uint32_t d = base_at(pk, pos - 1) | (base_at(pk, pos) << 2);
            stageL[off + j] = sL[d];
        }
    }
    __syncthreads();
    const bool all_staged = nst == nbar && sWoff[nst] <= kStageSteps;
    if (all_staged) {
        // every window staged: lane 0 alone runs the chain (no per-window broadcasts); the
        // next window's offset, length and gap are read while this one's steps run
        if (t == 0) {
            double2 v = init;
            int i0 = 0;
            if (nbar > 0 && sWk[0] == 0) {   // block 0 (always the first barrier)
                v = vhead0;
                voc[0] = v;
                i0 = 1;
            }
            int offn = 0, lenn = 0;
            C64 gapn = c64_id();
            if (i0 < nbar) {
                offn = sWoff[i0];
                lenn = sWb[i0] - sWa[i0];
                gapn = sGap[i0];
            }
            for (int i = i0; i < nbar; ++i) {
                const int off = offn, len = lenn;
                const C64 gp = gapn;
                if (i + 1 < nbar) {
                    offn = sWoff[i + 1];
                    lenn = sWb[i + 1] - sWa[i + 1];
                    gapn = sGap[i + 1];
                }
                v = c64_apply(v, gp);
                double P = v.x, M = v.y;
                const double4* st = stageL + off;
#pragma unroll 8
                for (int j = 0; j < len; ++j) {
                    const double4 l = st[j];
                    const Step s = ref_step(P, M, l.x, l.y, l.z, l.w);
                    P = s.P;
                    M = s.M;
                }
                v = make_double2(P, M);
                voc[i] = v;
            }
        }
    } else if (t < 64) {
        double2 v = init;
        for (int i = 0; i < nbar; ++i) {
            if (i == 0 && nst > 0 && sWk[0] == 0) {   // block 0 (always the first barrier)
                v = vhead[c];
                if (t == 0) voc[0] = v;
            } else if (i < nst && sWoff[i] + max(0, sWb[i] - sWa[i]) <= kStageSteps) {
                const C64 gp = sGap[i];
                v = c64_apply(v, gp);
                if (t == 0) {
                    double P = v.x, M = v.y;
                    const double4* st = stageL + sWoff[i];
                    const int len = sWb[i] - sWa[i];
#pragma unroll 8
                    for (int j = 0; j < len; ++j) {
                        const double4 l = st[j];
                        const Step s = ref_step(P, M, l.x, l.y, l.z, l.w);
                        P = s.P;
                        M = s.M;
                    }
                    v = make_double2(P, M);
                    voc[i] = v;
                }
                v = make_double2(__shfl(v.x, 0), __shfl(v.y, 0));
            } else {
                const int64_t k = blc[i];
                const VitPlan p = pl[k];
                v = c64_apply(v, ld_c64(gpc + i));
                const int ja = p.type == PLAN_SPLIT ? p.t1 : g.jfirst(k);
                const int jb = p.type == PLAN_SPLIT ? p.t2 : g.jend(k);
                v = chain_window(pk, sL, stepL, k, ja, jb, v, t);
                if (t == 0) voc[i] = v;
            }
        }
    }
    __syncthreads();
    // phase 4: entries
    double2 v = (bidx0 > 0) ? voc[bidx0 - 1] : init;
    if (t > 0) v = c64_apply(v, incoming);
    int idx = bidx0;
    auto entries = [&](int64_t k, const VitPlan& p, const C64& ca, const C64& cb) {
        ent[k] = v;
        if (p.type == PLAN_REGULAR) {
            v = c64_apply(v, ca);
        } else {
            v = voc[idx++];
            if (p.type == PLAN_SPLIT) v = c64_apply(v, cb);
        }
    };
    if (pre) {
#pragma unroll
        for (int i = 0; i < kPre; ++i)
            if (i < cnt) {
                const int64_t k = b0 + i;
                ent[k] = v;
                const double4 a4 = sApp[k];
                const C64 ap{a4.x, a4.y, a4.z, a4.w};
                const uint32_t kd = (kinds >> (2 * i)) & 3u;
                if (kd == 1u) {
                    v = c64_apply(v, ap);
                } else {
                    v = voc[idx++];
                    if (kd == 2u) v = c64_apply(v, ap);
                }
            }
    } else {
        for (int64_t k = b0; k < b1; ++k)
            entries(k, pl[k], ld_c64(cp + k), ld_c64(cq + k));
    }
    if (b1 == g.nsb && b0 < b1) ent[g.nsb] = v;
}

// K4, segment path (one 256-lane workgroup per chunk of 16 segments): the barrier list from
// the segments' masks, each barrier's gap composite from the K3 summaries (the run before it
// inside its segment is its rx; a run across segments is the tail of the barrier's segment
// times the leads of the barrier-free segments between), the serial chain over the barriers
// (as k_vit_chain), then the anchor values (a barrier's exit, + its post composite for
// SPLIT) by block id and the entry value of every segment.  Block entries: K5.
constexpr int kSegT = 256;
__global__ __launch_bounds__(kSegT) void k_vit_chain_seg(
    VitConsts vc, const uint32_t* packed, Geo g, const VitPlan* __restrict__ plan,
    const double4* __restrict__ comp3, const uint8_t* __restrict__ degen,
    const double4* __restrict__ rx, const SegSum* __restrict__ seg, double2* __restrict__ entry,
    double2* __restrict__ went, double4* __restrict__ gap, int32_t* __restrict__ barlist,
    double2* __restrict__ vout, const double2* __restrict__ vhead) {
    const int64_t c = blockIdx.x;
    const int t = threadIdx.x;
    const int nseg = (int)(g.nsb / kThreads);
    const int64_t s0 = c * nseg;
    double2* ent = entry + c * (g.nsb + 1);
    if (degen[c]) {
        for (int w = t; w < nseg; w += kSegT) went[s0 + w] = make_double2(-INFINITY, -INFINITY);
        if (t == 0) ent[g.nsb] = make_double2(-INFINITY, -INFINITY);
        return;
    }
    const uint32_t* pk = chunk_ptr(packed, g, c);
    const VitPlan* pl = plan + c * g.nsb;
    const double4* cp = comp3 + c * g.nsb;                          // SPLIT pre composites
    const double4* cq = comp3 + (g.nchunks + c) * g.nsb;            // SPLIT post composites
    const double4* rxc = rx + c * g.nsb;
    double2* voc = vout + c * g.nsb;
    double4* gpc = gap + c * g.nsb;
    int32_t* blc = barlist + c * g.nsb;
    __shared__ double4 sL[16];
    __shared__ double4 stepL[kSB];
    __shared__ double4 stageL[kStageSteps];
    __shared__ C64 sLead[kMaxSeg], sTail[kMaxSeg];
    __shared__ int sOff[kMaxSeg * 4 + 1];
    __shared__ int32_t sBar[kMaxSeg * kThreads];
    __shared__ int sWoff[kMaxStagedBar + 1];
    __shared__ int sWa[kMaxStagedBar], sWb[kMaxStagedBar];
    __shared__ int64_t sWk[kMaxStagedBar];
    __shared__ C64 sGap[kMaxStagedBar];
    __shared__ double2 sVo[kMaxStagedBar];
    if (t < 16) sL[t] = make_double4(vc.L[t][0], vc.L[t][1], vc.L[t][2], vc.L[t][3]);
    const double2 vhead0 = t == 0 ? vhead[c] : make_double2(0.0, 0.0);
    // A. barrier list: popcounts of the chunk's mask words, one wave's scan, then every word's
    //    barriers at their rank
    const int nwords = nseg * 4;
    unsigned long long mw = 0;
    if (t < nwords) mw = seg[s0 + (t >> 2)].mask[t & 3];
    if (t < nseg) {
        sLead[t] = ld_c64(&seg[s0 + t].lead);
        sTail[t] = ld_c64(&seg[s0 + t].tail);
    }
    if (t < 64) {
        const int cnt = (int)__popcll(mw);
        int x = cnt;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int y = __shfl_up(x, d);
            if (t >= d) x += y;
        }
        if (t < nwords) sOff[t] = x - cnt;
        if (t == 63) sOff[nwords] = x;
    }
    __syncthreads();
    const int nbar = sOff[nwords];
    if (t < nwords) {
        int o = sOff[t];
        const int base = (t >> 2) * kThreads + (t & 3) * 64;
        while (mw) {
            sBar[o++] = base + (int)__builtin_ctzll(mw);
            mw &= mw - 1;
        }
    }
    __syncthreads();
    // B. gap composites and windows, one lane per barrier.  The first kMaxStagedBar barriers'
    //    plan, rx and SPLIT composites are loaded in ONE round (every load issued up front,
    //    the composites whatever the block's type) and kept in LDS for the gaps, the anchors
    //    and the segment entries: no further global round trip through the plans (each had
    //    cost one memory latency on this one-workgroup-per-chunk critical path)
    __shared__ C64 sPre[kMaxStagedBar], sPost[kMaxStagedBar];
    __shared__ int sPt[kMaxStagedBar];
    // the staged barriers' blocks: their 16 packed words and the word before, loaded in this
    // same round as the plans (the window codes of phase C come from here, not from a third
    // dependent round trip to memory)
    __shared__ uint32_t sWd[kMaxStagedBar * 17];
    C64* sRx = sGap;   // rx of barrier i, replaced by its gap composite
    {
        const int nstb = min(nbar, kMaxStagedBar);
        for (int w = t; w < nstb * 17; w += kSegT) {
            const int bi = w / 17, j = w - bi * 17;
            const int64_t wi = (int64_t)sBar[bi] * kSBWords - 1 + j;
            sWd[w] = wi >= 0 ? pk[wi] : 0u;
        }
    }
    for (int i = t; i < nbar; i += kSegT) {
        const int k = sBar[i];
        blc[i] = k;
        if (i < kMaxStagedBar) {
            const VitPlan p = pl[k];
            const C64 r = ld_c64(rxc + k), pre = ld_c64(cp + k), post = ld_c64(cq + k);
            int ja = p.type == PLAN_SPLIT ? p.t1 : g.jfirst(k);
            int jb = p.type == PLAN_SPLIT ? p.t2 : g.jend(k);
            if (k == 0) ja = jb = 0;   // block 0: walked by K2's head lanes
            sWk[i] = k;
            sWa[i] = ja;
            sWb[i] = jb;
            sPt[i] = p.type;
            sRx[i] = r;
            sPre[i] = pre;
            sPost[i] = post;
            continue;
        }
        const VitPlan p = pl[k];   // (past the staged barriers: from global memory)
        C64 R = c64_id();
        {
            const int kp = sBar[i - 1], sp = kp / kThreads, sk = k / kThreads;
            if (sp == sk) {
                R = ld_c64(rxc + k);
            } else {
                R = sTail[sp];
                for (int u = sp + 1; u < sk; ++u) R = c64_mul(R, sLead[u]);
                R = c64_mul(R, ld_c64(rxc + k));
            }
            if (pl[kp].type == PLAN_SPLIT) R = c64_mul(ld_c64(cq + kp), R);
            if (p.type == PLAN_SPLIT) R = c64_mul(R, ld_c64(cp + k));
        }
        st_c64(gpc + i, R);
    }
    __syncthreads();
    const int nst = min(nbar, kMaxStagedBar);
    C64 Rg = c64_id();   // the gap composite of staged barrier t
    if (t < nst && t > 0) {
        const int k = sWk[t], kp = sWk[t - 1], sp = kp / kThreads, sk = k / kThreads;
        if (sp == sk) {
            Rg = sRx[t];
        } else {
            Rg = sTail[sp];
            for (int u = sp + 1; u < sk; ++u) Rg = c64_mul(Rg, sLead[u]);
            Rg = c64_mul(Rg, sRx[t]);
        }
        if (sPt[t - 1] == PLAN_SPLIT) Rg = c64_mul(sPost[t - 1], Rg);
        if (sPt[t] == PLAN_SPLIT) Rg = c64_mul(Rg, sPre[t]);
    }
    // the staging offsets: an exclusive scan of the window lengths (one wave; nst <= 64),
    // overflow marked from the first window that does not fit
    const int wlen = t < nst ? max(0, sWb[t] - sWa[t]) : 0;
    __syncthreads();   // every lane has read its sRx before it becomes sGap
    if (t < nst) {
        sGap[t] = Rg;
        st_c64(gpc + t, Rg);
    }
    if (t < 64) {
        int x = wlen;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int y = __shfl_up(x, d);
            if (t >= d) x += y;
        }
        const int ex = x - wlen;
        if (t < nst) sWoff[t] = ex <= kStageSteps ? ex : kStageSteps + 1;
        if (nst > 0 ? t == nst - 1 : t == 0)
            sWoff[nst] = x <= kStageSteps ? x : kStageSteps + 1;
    }
    // C. the serial chain over the barriers (k_vit_chain's phase 3)
    const uint32_t o0 = base_at(pk, 0);
    const double2 init = make_double2(vc.logpi[o0], vc.logpi[o0 + 4]);
    __syncthreads();
    for (int i = t >> 6; i < nst; i += kSegT / 64) {   // one wave per window
        const int off = sWoff[i];
        const int len = max(0, sWb[i] - sWa[i]);
        if (off + len > kStageSteps) continue;
        const uint32_t* wd = sWd + i * 17 + 1;   // word q of block sWk[i] at wd[q], q >= -1
        for (int j = t & 63; j < len; j += 64) {
            const int q = sWa[i] + j;              // position within the block (q - 1 >= -1)
            const uint32_t b1 = (wd[q >> 4] >> ((q & 15) * 2)) & 3u;
            const uint32_t b0 = (wd[(q - 1) >> 4] >> (((q - 1) & 15) * 2)) & 3u;
            stageL[off + j] = sL[b0 | (b1 << 2)];
        }
    }
    __syncthreads();
    const bool all_staged = nst == nbar && sWoff[nst] <= kStageSteps;
    if (all_staged) {
        if (t == 0) {
            double2 v = init;
            int i0 = 0;
            if (nbar > 0 && sWk[0] == 0) {   // block 0 (always the first barrier)
                v = vhead0;
                voc[0] = v;
                sVo[0] = v;
                i0 = 1;
            }
            int offn = 0, lenn = 0;
            C64 gapn = c64_id();
            if (i0 < nbar) {
                offn = sWoff[i0];
                lenn = sWb[i0] - sWa[i0];
                gapn = sGap[i0];
            }
            for (int i = i0; i < nbar; ++i) {
                const int off = offn, len = lenn;
                const C64 gp = gapn;
                if (i + 1 < nbar) {
                    offn = sWoff[i + 1];
                    lenn = sWb[i + 1] - sWa[i + 1];
                    gapn = sGap[i + 1];
                }
                v = c64_apply(v, gp);
                double P = v.x, M = v.y;
                const double4* st = stageL + off;
#pragma unroll 8
                for (int j = 0; j < len; ++j) {
                    const double4 l = st[j];
                    const Step s = ref_step(P, M, l.x, l.y, l.z, l.w);
                    P = s.P;
                    M = s.M;
                }
                v = make_double2(P, M);
                voc[i] = v;
                sVo[i] = v;
            }
        }
    } else if (t < 64) {
        double2 v = init;
        for (int i = 0; i < nbar; ++i) {
            if (i == 0 && sBar[0] == 0) {   // block 0 (always the first barrier)
                v = vhead[c];
            } else if (i < nst && sWoff[i] + max(0, sWb[i] - sWa[i]) <= kStageSteps) {
                v = c64_apply(v, sGap[i]);
                if (t == 0) {
                    double P = v.x, M = v.y;
                    const double4* st = stageL + sWoff[i];
                    const int len = sWb[i] - sWa[i];
#pragma unroll 8
                    for (int j = 0; j < len; ++j) {
                        const double4 l = st[j];
                        const Step s = ref_step(P, M, l.x, l.y, l.z, l.w);
                        P = s.P;
                        M = s.M;
                    }
                    v = make_double2(P, M);
                }
                v = make_double2(__shfl(v.x, 0), __shfl(v.y, 0));
            } else {
                const int64_t k = blc[i];
                const VitPlan p = pl[k];
                v = c64_apply(v, ld_c64(gpc + i));
                const int ja = p.type == PLAN_SPLIT ? p.t1 : g.jfirst(k);
                const int jb = p.type == PLAN_SPLIT ? p.t2 : g.jend(k);
                v = chain_window(pk, sL, stepL, k, ja, jb, v, t);
            }
            if (t == 0) {
                voc[i] = v;
                if (i < kMaxStagedBar) sVo[i] = v;
            }
        }
    }
    __syncthreads();
    // D. anchor values by block id: the barrier's exit (SPLIT: + the post composite)
    auto anchor_val = [&](int i) {   // (staged barriers: plan and post composite from LDS)
        if (i < kMaxStagedBar) {
            double2 v = sVo[i];
            if (sPt[i] == PLAN_SPLIT) v = c64_apply(v, sPost[i]);
            return v;
        }
        const int k = sBar[i];
        double2 v = voc[i];
        if (pl[k].type == PLAN_SPLIT) v = c64_apply(v, ld_c64(cq + k));
        return v;
    };
    for (int i = t; i < nbar; i += kSegT) ent[sBar[i]] = anchor_val(i);
    // E. segment entries (segment 0: the initial value; block 0 is its first barrier) and the
    //    chunk's final value (K6)
    if (t <= nseg) {
        double2 E = init;
        if (t > 0) {
            const int il = sOff[4 * t] - 1;   // the last barrier before segment t (>= block 0)
            const int kl = sBar[il], sl = kl / kThreads;
            C64 R = sTail[sl];
            for (int u = sl + 1; u < t; ++u) R = c64_mul(R, sLead[u]);
            E = c64_apply(anchor_val(il), R);
        }
        if (t < nseg) went[s0 + t] = E;
        else ent[g.nsb] = E;
    }
}

// ---------------------------------------------------------------- K5: re-forward
__device__ __forceinline__ uint32_t map_apply(uint32_t m, uint32_t x) { return (m >> x) & 1u; }
__device__ __forceinline__ uint32_t map_compose(uint32_t f, uint32_t g) {   // f o g
    return map_apply(f, map_apply(g, 0)) | (map_apply(f, map_apply(g, 1)) << 1);
}
// w << 1 | c in one VALU op: the compare's lane mask is the carry-in of w + w (the compare
// writes the mask straight to an SGPR pair; the select + shift-or pair it replaces was two)
__device__ __forceinline__ uint32_t push_bit(uint32_t w, bool c) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(c);
    uint32_t r;
    uint64_t co;
    asm("v_addc_co_u32 %0, %1, %2, %2, %3" : "=v"(r), "=s"(co) : "v"(w), "s"(m));
    return r;
}

// nibble m (compile-time, 0..7) of w times 16 in one VALU op: SDWA byte selects — a low
// nibble shifted into a byte whose other bits are dropped, a high nibble masked in place
// (the shift + mask pair they replace was two ops per step of K5's walk)
__device__ __forceinline__ uint32_t nib16(uint32_t w, int m) {
#if !defined(__gfx950__)   // (SDWA is a gfx9-family encoding: other targets shift + mask)
    return ((w >> (4 * m)) & 15u) << 4;
#else
    uint32_t r;
    const uint32_t f0 = 0xF0u;
    switch (m) {
        case 0: asm("v_lshlrev_b32_sdwa %0, 4, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(r) : "v"(w)); break;
        case 1: r = w & 0xF0u; break;
        case 2: asm("v_lshlrev_b32_sdwa %0, 4, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(w)); break;
        case 3: asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(f0), "v"(w)); break;
        case 4: asm("v_lshlrev_b32_sdwa %0, 4, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(w)); break;
        case 5: asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(f0), "v"(w)); break;
        case 6: asm("v_lshlrev_b32_sdwa %0, 4, %1 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(w)); break;
        default: asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(f0), "v"(w)); break;
    }
    return r;
#endif
}

// origin map (bit x = origin sign of the state-x survivor, '+' = 1) of 64 steps from their
// backpointer bits (bit j of bP / bM: step j's '+' / '-' survivor came from '-'): step j maps
// its state to the previous one, b_j(1) = !bP_j, b_j(0) = !bM_j, and the quad's map is
// b_0 o b_1 o ... o b_63 — a 6-level tree of bit-parallel compositions, in the complemented
// encoding: (f o g).P = g.P ? f.M : f.P, (f o g).M = g.M ? f.M : f.P
__device__ __forceinline__ uint32_t quad_origin(uint64_t hP, uint64_t hM) {
#pragma unroll
    for (int sh = 1; sh < 64; sh <<= 1) {
        const uint64_t gP = hP >> sh, gM = hM >> sh;
        const uint64_t nP = (gP & hM) | (~gP & hP);
        const uint64_t nM = (gM & hM) | (~gM & hP);
        hP = nP;
        hM = nM;
    }
    return (uint32_t)((~hM & 1u) | ((~hP & 1u) << 1));
}

// one block's re-forward (lane = block gid): backpointers, the self-check; returns the
// block's origin map
// sgi: the segment (workgroup of the segment path) the block belongs to.
template <int kLook>
__device__ __forceinline__ uint32_t fwd_block(const VitConsts& vc, const uint32_t* packed,
                                              const Geo& g, const uint8_t* __restrict__ degen,
                                              const double2* __restrict__ entry,
                                              uint4* __restrict__ bp, uint32_t* status,
                                              const double4* __restrict__ rx,
                                              const SegSum* __restrict__ seg,
                                              const double2* __restrict__ went,
                                              const double2* LA, const double2* LB, int64_t gid,
                                              int64_t sgi) {
    const int64_t c = gid / g.nsb, k = gid - c * g.nsb;
    // backpointers quad-major: bp[q * nt + gid] = {bP bits 0-31, 32-63, bM bits 0-31, 32-63} of
    // the block's quad q (64 steps), so that each quad's store is one coalesced 16-B/lane row
    const int64_t nt = g.nchunks * g.nsb;
    uint4* bpo = bp + gid;
    auto put = [&](int q, uint4 w) { bpo[q * nt] = w; };
    if (degen[c]) {
        for (int i = 0; i < 4; ++i) put(i, make_uint4(0, 0, 0, 0));
        return 0x2u;   // identity
    }
    const uint32_t* pk = chunk_ptr(packed, g, c);
    const double2* ent = entry + c * (g.nsb + 1);
    // segment path (workgroup = segment): a block's entry = anchor value . rx, the anchor
    // being the last barrier before the block in the segment (K4's value by block id) or,
    // with none, the segment's entry.  The next block's entry (the self-check) is derived
    // after the walk, so that nothing of it stays live across the loop.
    auto entries = [&](bool next) -> double2 {
        if (!seg) return ent[k + (next ? 1 : 0)];
        const int l = threadIdx.x;
        const SegSum& sg = seg[sgi];
        const unsigned long long m[4] = {sg.mask[0], sg.mask[1], sg.mask[2], sg.mask[3]};
        const int q = l >> 6, r = l & 63;
        const unsigned long long mq = q == 0 ? m[0] : q == 1 ? m[1] : q == 2 ? m[2] : m[3];
        int a = -1;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
            if (qq < q && m[qq]) a = qq * 64 + 63 - (int)__builtin_clzll(m[qq]);
        const unsigned long long below = r ? (mq & ((1ull << r) - 1ull)) : 0ull;
        if (below) a = q * 64 + 63 - (int)__builtin_clzll(below);
        const int64_t sbase = k - l;
        const double2 E = went[sgi];
        if (!next) return c64_apply(a >= 0 ? ent[sbase + a] : E, ld_c64(rx + gid));
        if (l + 1 < kThreads) {
            const int a2 = ((mq >> r) & 1ull) ? l : a;
            return c64_apply(a2 >= 0 ? ent[sbase + a2] : E, ld_c64(rx + gid + 1));
        }
        return k + 1 == g.nsb ? ent[g.nsb] : went[sgi + 1];
    };
    const double2 v0 = entries(false);   // this block's entry
    // the next block's entry (the self-check below) is the next lane's own entry, the same
    // computation (entries(true) == its entries(false)): taken from it through LDS (same wave:
    // its LDS accesses complete in order; nothing held in registers across the walk), not
    // loaded again — except by the wave's last lane and a chunk's last block
    __shared__ double2 s_v0[kThreads];
    s_v0[threadIdx.x] = v0;
    const bool vn_here = (threadIdx.x & 63) != 63 && k + 1 < g.nsb;
    double P = v0.x, M = v0.y;
    uint32_t oP = 1u, oM = 0u;   // origin sign of the current '+' / '-' survivor
    uint32_t wP0 = 0, wP1 = 0, wM0 = 0, wM1 = 0;
    auto flush = [&](int q) {
        put(q, make_uint4(wP0, wP1, wM0, wM1));
        wP0 = wP1 = wM0 = wM1 = 0;
    };
    auto step2 = [&](double l0, double l1, double l2, double l3, int q, int jj) {
        const Step s = ref_step(P, M, l0, l1, l2, l3);
        P = s.P;
        M = s.M;
        const uint32_t noP = s.bP ? oM : oP;
        const uint32_t noM = s.bM ? oM : oP;
        oP = noP;
        oM = noM;
        if (jj < 32) { wP0 |= s.bP << jj; wM0 |= s.bM << jj; }
        else { wP1 |= s.bP << (jj - 32); wM1 |= s.bM << (jj - 32); }
        if (jj == 63) flush(q);
    };
    auto step = [&](uint32_t d, int q, int jj) {
        const double2 la = LA[d], lb = LB[d];
        step2(la.x, la.y, lb.x, lb.y, q, jj);
    };
    if (g.whole(k)) {
        // quads of 64 steps; the ring of kLook lookups in flight runs across quad borders
        static_assert(64 % kLook == 0, "the ring's slot of a step is its index mod kLook in every quad");
        const unsigned char* LAb = reinterpret_cast<const unsigned char*>(LA);
        const unsigned char* LBb = reinterpret_cast<const unsigned char*>(LB);
        auto fetch = [&](uint32_t a) {   // a = code * 16 (byte offset of the entry)
            const double2 x = *reinterpret_cast<const double2*>(LAb + a);
            const double2 y = *reinterpret_cast<const double2*>(LBb + a);
            return C64{x.x, x.y, y.x, y.y};
        };
        // step j's code (bases j-1, j) times 16, one VALU op per step: odd i = 2m + 1 is
        // nibble m of the word, even i = 2m nibble m of the word shifted in by one base
        // (one alignbit per word)
        auto code = [](const uint4 w, uint32_t prev, int j) {   // j compile-time, < 64
            const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
            const int r = j >> 4, i = j & 15;
            const uint32_t lo = r == 0 ? prev : ww[r - 1];
            return (i & 1) ? nib16(ww[r], i >> 1)
                           : nib16(__builtin_amdgcn_alignbit(ww[r], lo, 30), i >> 1);
        };
        const int64_t wbase = k * kSBWords;
        uint32_t prev = k > 0 ? pk[wbase - 1] : 0u;
        uint4 cur = *reinterpret_cast<const uint4*>(pk + wbase);
        C64 ring[kLook];
#pragma unroll
        for (int j = 0; j < kLook; ++j)
            ring[j] = fetch((j == 0 && k == 0) ? 16u * 16u : code(cur, prev, j));
        uint32_t omap = 0x2u;   // identity
#pragma unroll 1
        for (int q = 0; q < 4; ++q) {
            const uint4 nxt = *reinterpret_cast<const uint4*>(pk + wbase + 4 * (q < 3 ? q + 1 : q));
            // bits pushed in at the bottom: step jj ends at bit 31 - (jj mod 32), reversed below
            uint32_t aP0 = 0, aP1 = 0, aM0 = 0, aM1 = 0;
#pragma clang loop unroll(full)
            for (int jj = 0; jj < 64; ++jj) {
                const C64 l = ring[jj % kLook];
                const int j2 = jj + kLook;   // past the block's end (q == 3): harmless lookups
                ring[jj % kLook] = fetch(j2 < 64 ? code(cur, prev, j2) : code(nxt, cur.w, j2 - 64));
                const Step st = ref_step(P, M, l.pp, l.pm, l.mp, l.mm);
                P = st.P;
                M = st.M;
                if (jj < 32) {
                    aP0 = push_bit(aP0, st.bP);
                    aM0 = push_bit(aM0, st.bM);
                } else {
                    aP1 = push_bit(aP1, st.bP);
                    aM1 = push_bit(aM1, st.bM);
                }
            }
            const uint32_t p0 = __builtin_bitreverse32(aP0), p1 = __builtin_bitreverse32(aP1);
            const uint32_t m0 = __builtin_bitreverse32(aM0), m1 = __builtin_bitreverse32(aM1);
            put(q, make_uint4(p0, p1, m0, m1));
            omap = map_compose(omap, quad_origin(p0 | ((uint64_t)p1 << 32),
                                                 m0 | ((uint64_t)m1 << 32)));
            prev = cur.w;
            cur = nxt;
        }
        oP = (omap >> 1) & 1u;
        oM = omap & 1u;
    } else {
        // partial/first block: positions outside the chunk are skipped; flush every quad
        walk_block<false>(pk, k, g.C, [&](uint32_t d, int q, int jj) {
            step(d, q, jj);
        });
        // quads whose last position was skipped were not flushed: flush all remaining
        const int jend = g.jend(k);
        for (int q = 0; q < 4; ++q) {
            const int last = q * 64 + 63;
            if (last >= jend) {
                put(q, make_uint4(wP0, wP1, wM0, wM1));
                wP0 = wP1 = wM0 = wM1 = 0;
            }
        }
    }
    asm volatile("" ::: "memory");   // (the read stays after the walk and the write)
    const double2 nx = vn_here ? s_v0[threadIdx.x + 1] : entries(true);   // the self-check
    if (__double_as_longlong(nx.x) != __double_as_longlong(P) ||
        __double_as_longlong(nx.y) != __double_as_longlong(M))
        atomicOr(status, ST_VERIFY_ENTRY);
    return oM | (oP << 1);
}

// ---------------------------------------------------------------- K6: trace scan

// origin maps written by an earlier kernel (plain loads) or by other workgroups of this one
// (K5's chunk tail: agent-scope atomic words, see k_vit_forward)
template <bool kAgent>
__device__ __forceinline__ uint32_t ld_org4(const uint8_t* p) {   // 4 maps, p 4-B aligned
    if constexpr (kAgent)
        return __hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
    else
        return *reinterpret_cast<const uint32_t*>(p);
}
template <bool kAgent>
__device__ __forceinline__ uint32_t ld_org(const uint8_t* og, int64_t k) {
    if constexpr (kAgent) return (ld_org4<true>(og + (k & ~3ll)) >> (8 * (k & 3))) & 0xFFu;
    else return og[k];
}

// K6's work for chunk c (one workgroup of kThreads lanes): final argmax, suffix scan of the
// block origin maps, every block's end state
template <bool kAgent>
__device__ __forceinline__ void tscan_chunk(const Geo& g, const double2* __restrict__ entry,
                                            const uint8_t* __restrict__ origin,
                                            uint8_t* __restrict__ endst,
                                            double* __restrict__ score, int64_t c) {
    const int t = threadIdx.x;
    const int64_t per = (g.nsb + kThreads - 1) / kThreads;
    const int64_t b0 = t * per, b1 = min(b0 + per, g.nsb);
    const uint8_t* og = origin + c * g.nsb;
    const double2 fin = entry[c * (g.nsb + 1) + g.nsb];
    const uint32_t s_end = (fin.y > fin.x) ? 0u : 1u;   // '+' first: '-' only if strictly >
    if (t == 0 && score) score[c] = s_end ? fin.x : fin.y;
    // chunks of 1 Mi (nsb = 4096): a lane's 16 origin maps are one 16-B load and its 16 end
    // states one 16-B store (byte loops had issued 16 dependent loads and 16 byte stores)
    const bool vec = per == 16 && g.nsb % 16 == 0, have = b0 < b1;
    uint32_t ow[4] = {0, 0, 0, 0};
    if (vec && have) {
        if constexpr (kAgent) {
#pragma unroll
            for (int i = 0; i < 4; ++i) ow[i] = ld_org4<true>(og + b0 + 4 * i);
        } else {
            const uint4 w = *reinterpret_cast<const uint4*>(og + b0);
            ow[0] = w.x; ow[1] = w.y; ow[2] = w.z; ow[3] = w.w;
        }
    }
    uint32_t F = 0x2u;
    if (vec) {
        if (have) {
#pragma unroll
            for (int i = 0; i < 16; ++i) F = map_compose(F, (ow[i >> 2] >> (8 * (i & 3))) & 0xFFu);
        }
    } else {
        for (int64_t k = b0; k < b1; ++k) F = map_compose(F, ld_org<kAgent>(og, k));
    }
    // suffix composition over the lanes: wave shuffles (down), then the wave totals
    const int lane = t & 63, wv = t >> 6;
    uint32_t x = F;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_down(x, off);
        if (lane + off < 64) x = map_compose(x, y);
    }
    __shared__ uint32_t sW[kThreads / 64];
    if (lane == 0) sW[wv] = x;
    __syncthreads();
    uint32_t after = 0x2u;   // composition of the waves after this one
    for (int w = kThreads / 64 - 1; w > wv; --w) after = map_compose(sW[w], after);
    const uint32_t dn = __shfl_down(x, 1);
    const uint32_t G = lane < 63 ? map_compose(dn, after) : after;   // the lanes after t
    uint32_t e = map_apply(G, s_end);
    if (vec) {
        if (have) {
            uint32_t ew[4] = {0, 0, 0, 0};
#pragma unroll
            for (int i = 15; i >= 0; --i) {
                ew[i >> 2] |= e << (8 * (i & 3));
                e = map_apply((ow[i >> 2] >> (8 * (i & 3))) & 0xFFu, e);
            }
            *reinterpret_cast<uint4*>(endst + c * g.nsb + b0) = make_uint4(ew[0], ew[1], ew[2], ew[3]);
        }
    } else {
        for (int64_t k = b1 - 1; k >= b0; --k) {
            endst[c * g.nsb + k] = (uint8_t)e;
            e = map_apply(ld_org<kAgent>(og, k), e);
        }
    }
}

__global__ __launch_bounds__(kThreads) void k_vit_tscan(Geo g, const double2* __restrict__ entry,
                                                        const uint8_t* __restrict__ origin,
                                                        uint8_t* __restrict__ endst,
                                                        double* __restrict__ score) {
    tscan_chunk<false>(g, entry, origin, endst, score, blockIdx.x);
}

// K5.  kScan (chunks of whole workgroups, nsb % 256 == 0): the chunk's last workgroup to
// finish also runs K6's scan for it (done: per-chunk counters, zero between calls, reset by
// that workgroup); the origin maps then cross workgroups inside the kernel, 4 per
// agent-scope atomic word.
template <bool kScan>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(kScan ? kK5WavesPerEUFused : kK5WavesPerEU))) void k_vit_forward(VitConsts vc, const uint32_t* packed,
                                                          Geo g, const uint8_t* __restrict__ degen,
                                                          const double2* __restrict__ entry,
                                                          uint4* __restrict__ bp,
                                                          uint8_t* __restrict__ origin,
                                                          uint32_t* status,
                                                          const double4* __restrict__ rx,
                                                          const SegSum* __restrict__ seg,
                                                          const double2* __restrict__ went,
                                                          unsigned int* done,
                                                          uint8_t* __restrict__ endst,
                                                          double* __restrict__ score) {
    // conflict-free halves (16 x 16 B each); entry 16 is the identity step (0, -inf, -inf,
    // 0) standing for block 0's position 0: P + 0.0 = P and M + -inf = -inf exactly, so the
    // values, the tie bits that matter and the origins are unchanged by it
    __shared__ double2 LA[17], LB[17];
    if (threadIdx.x < 16) {
        LA[threadIdx.x] = make_double2(vc.L[threadIdx.x][0], vc.L[threadIdx.x][1]);
        LB[threadIdx.x] = make_double2(vc.L[threadIdx.x][2], vc.L[threadIdx.x][3]);
    } else if (threadIdx.x == 16) {
        LA[16] = make_double2(0.0, -INFINITY);
        LB[16] = make_double2(-INFINITY, 0.0);
    }
    __syncthreads();
    const int64_t gid = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (gid >= g.nchunks * g.nsb) return;   // (kScan: the grid is whole workgroups)
    const uint32_t org = fwd_block<kScan ? kK5LookFused : 2>(vc, packed, g, degen, entry, bp, status, rx, seg, went, LA,
                                   LB, gid, blockIdx.x);
    if constexpr (!kScan) {
        origin[gid] = (uint8_t)org;
    } else {
        const uint32_t o1 = __shfl_down(org, 1), o2 = __shfl_down(org, 2), o3 = __shfl_down(org, 3);
        if ((threadIdx.x & 3) == 0)
            __hip_atomic_store(reinterpret_cast<uint32_t*>(origin + gid),
                               org | (o1 << 8) | (o2 << 16) | (o3 << 24), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        __shared__ int s_last;
        __builtin_amdgcn_s_waitcnt(0);   // this wave's map stores have completed
        __syncthreads();
        const int64_t c = gid / g.nsb;
        if (threadIdx.x == 0) {
            const unsigned wpc = (unsigned)(g.nsb / kThreads);
            const unsigned old = __hip_atomic_fetch_add(done + c, 1u, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
            s_last = old == wpc - 1;
            if (s_last)   // zero again for the next call
                __hip_atomic_store(done + c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (s_last) tscan_chunk<true>(g, entry, origin, endst, score, c);
    }
}

// ---------------------------------------------------------------- K7: traceback

// Fused decode (cpg_decode_d): the workgroup is one island tile (its 256 blocks, inside one
// chunk).  From the block's 8 sign words just traced, its 16 packed words, the packed word
// and the state before the block, every lane counts its words (C, G, CpG, run starts and
// closes: isl_dev.h), one workgroup scan gives the tile-relative prefix at each word, and
// lanes holding a run boundary write its records — the island tile kernel's work without
// reading the sign words back.  Records and totals are agent-scope atomic stores: the
// chunk's last workgroup reads them (k_vit_trace).
// kAgent: the records are read by another workgroup of this launch (the chunk's resolve in
// its last workgroup); otherwise by the resolve kernels after it (plain stores).
template <bool kAgent>
__device__ __forceinline__ void trace_tile(const uint32_t (&out)[8], const uint32_t (&P)[16],
                                           uint32_t pprev, uint32_t sprev, int64_t k,
                                           const isl::IslWs& tl, int64_t tile) {
    using namespace isl;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    Cnt5 n{0, 0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 8; ++i)
        n = cadd(n, cnt_of(masks_reg(out[i], i ? out[i - 1] : sprev, P[2 * i], P[2 * i + 1],
                                     i ? P[2 * i - 1] : pprev)));
    // a wave's sums fit 16 bits (<= 64 x 256): two fields per word
    const uint32_t own0 = (uint32_t)n.c | ((uint32_t)n.g << 16),
                   own1 = (uint32_t)n.cg | ((uint32_t)n.st << 16), own2 = (uint32_t)n.cl;
    uint32_t x0 = own0, x1 = own1, x2 = own2;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y0 = __shfl_up(x0, off), y1 = __shfl_up(x1, off), y2 = __shfl_up(x2, off);
        if (lane >= off) {
            x0 += y0;
            x1 += y1;
            x2 += y2;
        }
    }
    __shared__ Cnt5 wt[kThreads / 64];
    if (lane == 63)
        wt[wv] = Cnt5{(int32_t)(x0 & 0xFFFFu), (int32_t)(x0 >> 16), (int32_t)(x1 & 0xFFFFu),
                      (int32_t)(x1 >> 16), (int32_t)x2};
    __syncthreads();
    Cnt5 e{0, 0, 0, 0, 0}, tot{0, 0, 0, 0, 0};
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) {
        const Cnt5 v = wt[w];
        if (w < wv) e = cadd(e, v);
        tot = cadd(tot, v);
    }
    const uint32_t ex0 = x0 - own0, ex1 = x1 - own1, ex2 = x2 - own2;
    e = cadd(e, Cnt5{(int32_t)(ex0 & 0xFFFFu), (int32_t)(ex0 >> 16), (int32_t)(ex1 & 0xFFFFu),
                     (int32_t)(ex1 >> 16), (int32_t)ex2});
    if (n.st | n.cl) {   // the lane's words hold a run boundary
        RunRec* st = tl.starts + tile * tl.cap_t;
        RunRec* cl = tl.closes + tile * tl.cap_t;
#pragma unroll
        for (int i = 0; i < 8; ++i)
            emit_word<kAgent>(masks_reg(out[i], i ? out[i - 1] : sprev, P[2 * i], P[2 * i + 1],
                                  i ? P[2 * i - 1] : pprev),
                        k * 8 + i, e, st, cl);
    }
    if (t == 0) st_cnt5<kAgent>(tl.ttot + tile, tot);
}

// kIsl: 0 = the traceback alone; 1 = + the island tile of its workgroup + the chunk's first
// resolve pass in the chunk's last workgroup (fused decode, <= 256 chunks; the records are
// placed by the write pass after it); 2 = + the island tile only, both resolve kernels run
// after it (fused decode past 256 chunks: no re-read of bases and signs)
template <int kIsl>
__global__ __launch_bounds__(kThreads) void k_vit_trace(Geo g, const uint4* __restrict__ bp,
                                                        const uint8_t* __restrict__ endst,
                                                        uint32_t* __restrict__ sign_out,
                                                        uint32_t* status, uint32_t* zero_at,
                                                        int64_t zero_n,
                                                        const uint32_t* __restrict__ packed,
                                                        IslFuse fz) {
    const int64_t gid = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    // the undecoded tail's sign words ('-'), in this launch rather than a memset of its own
    for (int64_t i = gid; i < zero_n; i += (int64_t)gridDim.x * kThreads) zero_at[i] = 0u;
    // kIsl: the grid is whole workgroups of whole blocks (no lane leaves before the barrier)
    if (gid >= g.nchunks * g.nsb) return;
    const int64_t c = gid / g.nsb, k = gid - c * g.nsb;
    uint32_t P[16], pprev = 0u;
    if constexpr (kIsl != 0) {   // the block's 256 bases: issued first, used after the traceback
        const uint32_t* pk = packed + c * (g.C >> 4) + k * 16;
        const uint4* p4 = reinterpret_cast<const uint4*>(pk);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint4 v = p4[i];
            P[4 * i] = v.x; P[4 * i + 1] = v.y; P[4 * i + 2] = v.z; P[4 * i + 3] = v.w;
        }
        if (k > 0) pprev = pk[-1];
    }
    uint32_t wP[8], wM[8];
    {
        const int64_t nt = g.nchunks * g.nsb;   // quad-major layout (k_vit_forward)
        const uint4* b = bp + gid;
        const uint4 x0 = b[0], x1 = b[nt], x2 = b[2 * nt], x3 = b[3 * nt];
        wP[0] = x0.x; wP[1] = x0.y; wM[0] = x0.z; wM[1] = x0.w;
        wP[2] = x1.x; wP[3] = x1.y; wM[2] = x1.z; wM[3] = x1.w;
        wP[4] = x2.x; wP[5] = x2.y; wM[4] = x2.z; wM[5] = x2.w;
        wP[6] = x3.x; wP[7] = x3.y; wM[6] = x3.z; wM[7] = x3.w;
    }
    // Word-parallel traceback.  Position j's backpointers are a map m_j: state at j ->
    // state at j-1 (m_j(+) = ~bP_j, m_j(-) = ~bM_j; identity past the block's end).  The
    // states of a word's 32 positions are H_j(s_31) with H_j = m_{j+1} o ... o m_31: a
    // 5-level suffix scan of map compositions on bit vectors (X = map(+), Y = map(-) per
    // bit; f o g = (bfi(Xg, Xf, Yf), bfi(Yg, Xf, Yf))), then m_0 steps into the next word.
    const int jend = g.jend(k);
    uint32_t s = endst[gid];   // state at the block's last position
    // the state before the block (the previous block's end state), loaded with it
    const uint32_t sb = k > 0 ? endst[gid - 1] : 0u;
    uint32_t out[8];
#pragma unroll
    for (int w = 7; w >= 0; --w) {
        const int n = jend - 32 * w;
        const uint32_t vm = n >= 32 ? 0xFFFFFFFFu : (n <= 0 ? 0u : (1u << n) - 1u);
        const uint32_t A = ~wP[w] | ~vm, B = ~wM[w] & vm;
        uint32_t X = (A >> 1) | 0x80000000u, Y = B >> 1;   // e_j = m_{j+1}, e_31 = id
#pragma unroll
        for (int d = 1; d < 32; d <<= 1) {
            const uint32_t Xg = __builtin_amdgcn_alignbit(0xFFFFFFFFu, X, d);   // id fill
            const uint32_t Yg = Y >> d;
            const uint32_t nX = (Xg & X) | (~Xg & Y), nY = (Yg & X) | (~Yg & Y);
            X = nX;
            Y = nY;
        }
        const uint32_t S = s ? X : Y;
        out[w] = S & vm;
        s = (S & 1u) ? (A & 1u) : (B & 1u);   // state at position 32w - 1
    }
    // block 0: bit 0 of out[0] is the state of position 0 itself; otherwise the state
    // reached before the block must be the previous block's end state
    if (k > 0 && s != sb) atomicOr(status, ST_VERIFY_CHAIN);
    // write the block's words (positions k*256 ... k*256+255 of the chunk)
    uint32_t* so = sign_out + c * (g.C >> 5) + k * 8;
    const int64_t nw = (g.C + 31) >> 5;
    if ((k + 1) * 8 <= nw) {
        uint4* s4 = reinterpret_cast<uint4*>(so);
        s4[0] = make_uint4(out[0], out[1], out[2], out[3]);
        s4[1] = make_uint4(out[4], out[5], out[6], out[7]);
    } else {
#pragma unroll
        for (int w = 0; w < 8; ++w)
            if (k * 8 + w < nw) so[w] = out[w];
    }
    if constexpr (kIsl == 2) trace_tile<false>(out, P, pprev, sb << 31, k, fz.ws, blockIdx.x);
    if constexpr (kIsl == 1) {
        trace_tile<true>(out, P, pprev, sb << 31, k, fz.ws, blockIdx.x);
        // the chunk's last workgroup to finish runs its first resolve pass (its run records are
        // complete; a done counter, nothing waits): the resolve kernel's work, overlapped with
        // the other chunks' tracebacks
        __shared__ int s_last;
        __builtin_amdgcn_s_waitcnt(0);   // this wave's record stores have completed
        __syncthreads();
        if (threadIdx.x == 0) {
            const unsigned wpc = (unsigned)(g.nsb / kThreads);
            const unsigned old = __hip_atomic_fetch_add(fz.done + c, 1u, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
            s_last = old == wpc - 1;
            if (s_last)   // zero again for the next call
                __hip_atomic_store(fz.done + c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (!s_last) return;
        __shared__ isl::ResolveLds L;
        __shared__ isl::Cnt5 s_to[kThreads / 16];
        isl::resolve_chunk<true, kThreads / 16>(packed, g.C, fz.ws, c, L, s_to);
    }
}

// ---------------------------------------------------------------- workspace layout
struct VitWs {
    int4* comp1;
    longlong2* aent;
    VitPlan* plan;
    double4* comp3;
    double2* entry;
    double4* gk;
    double4* gap;
    int32_t* barlist;
    double2* vout;
    double2* vhead;
    int32_t* splitlist;
    int32_t* splitcount;
    uint4* bp;
    uint8_t* origin;
    uint8_t* endst;
    uint8_t* degen;
    SegSum* seg;      // segment path: per 256-block segment
    double2* went;    // segment entries
    int32_t* irrseg;           // per segment: irregular blocks listed
    size_t bytes;
};

VitWs carve(void* base, int64_t nchunks, int64_t nsb) {
    const int64_t nt = nchunks * nsb;
    char* p = static_cast<char*>(base);
    size_t off = 0;
    auto take = [&](size_t bytes) {
        off = (off + 255) & ~size_t(255);
        char* r = p ? p + off : nullptr;
        off += bytes;
        return r;
    };
    VitWs w;
    w.comp1 = (int4*)take(nt * sizeof(int4));
    w.aent = (longlong2*)take(nchunks * (nsb + 1) * sizeof(longlong2));
    w.plan = (VitPlan*)take(nt * sizeof(VitPlan));
    w.comp3 = (double4*)take(nt * 2 * sizeof(double4));
    w.entry = (double2*)take(nchunks * (nsb + 1) * sizeof(double2));
    w.gk = (double4*)take(nt * sizeof(double4));
    w.gap = (double4*)take(nt * sizeof(double4));
    w.barlist = (int32_t*)take(nt * sizeof(int32_t));
    w.vout = (double2*)take(nt * sizeof(double2));
    w.vhead = (double2*)take(nchunks * sizeof(double2));
    w.splitlist = (int32_t*)take(nt * sizeof(int32_t));
    w.splitcount = (int32_t*)take(nchunks * sizeof(int32_t));
    w.bp = (uint4*)take(nt * 4 * sizeof(uint4));
    w.origin = (uint8_t*)take(nt);
    w.endst = (uint8_t*)take(nt);
    w.degen = (uint8_t*)take(nchunks);
    w.seg = (SegSum*)take((nt / kThreads + 1) * sizeof(SegSum));
    w.went = (double2*)take((nt / kThreads + 1) * sizeof(double2));
    w.irrseg = (int32_t*)take((nt / kThreads + 1) * sizeof(int32_t));
    w.bytes = off + 256;
    return w;
}

}  // namespace

int64_t vit_nsb(int64_t chunk_len) { return chunk_len <= 1 ? 1 : (chunk_len + kSB - 1) / kSB; }

// [segment][8] K1's segment products
size_t viterbi_agg_bytes(int64_t nchunks, int64_t chunk_len) {
    return (size_t)(nchunks * vit_nsb(chunk_len) / kThreads + 1) * 8 * sizeof(unsigned long long);
}

size_t viterbi_ws_bytes(int64_t nchunks, int64_t chunk_len) {
    return carve(nullptr, nchunks, vit_nsb(chunk_len)).bytes;
}

hipError_t launch_viterbi(const VitConsts& vc, const VitTables* d_vt, const uint32_t* packed,
                          int64_t nchunks, int64_t chunk_len, void* ws, size_t ws_bytes,
                          uint32_t* sign_out, double* score, uint8_t* degen_out,
                          uint32_t* status, hipStream_t s, unsigned long long* agg,
                          uint32_t* zero_at, int64_t zero_n, const IslFuse* fuse,
                          unsigned int* done5) {
    const int64_t nsb = vit_nsb(chunk_len);
    VitWs w = carve(ws, nchunks, nsb);
    if (w.bytes > ws_bytes) return hipErrorInvalidValue;
    Geo g{nchunks, chunk_len, nsb};
    const int64_t nt = nchunks * nsb;
    const unsigned grid = (unsigned)((nt + kThreads - 1) / kThreads);
    // block 0 of every chunk is walked by extra workgroups of K2's launch (one lane per chunk):
    // a 256-step dependent chain (~13 us) that set K1's duration; K2 takes as long without it
    // (as K3's extra workgroups it cost K3 0.9 us more: measured, not kept)
    const unsigned head = (unsigned)((nchunks + kScanT - 1) / kScanT);
    // the segment path for chunks of whole 256-block segments, at most kMaxSeg of them (the
    // reference's 1 Mi decode chunk: 16): K1 also forms each segment's product, K2 runs per
    // segment (k_vit_segplan), block 0's walk in K3's launch, K4 over barriers and segment
    // summaries only; rx in the gk slot
    const bool segp = nsb % kThreads == 0 && nsb / kThreads <= kMaxSeg && chunk_len == nsb * kSB;
    SegSum* sg = segp ? w.seg : nullptr;
    ApproxSeg as{nullptr, w.aent, w.degen, w.plan, w.splitlist, w.irrseg};
    if (segp) {   // the segment products (WS_VAGG)
        if (!agg) return hipErrorInvalidValue;
        as.segprod = reinterpret_cast<CI*>(agg);
    }
    hipLaunchKernelGGL(k_vit_approx, dim3(grid), dim3(kThreads), 0, s, vc, packed, g, d_vt,
                       w.comp1, as);
    if (segp)
        hipLaunchKernelGGL(k_vit_segplan, dim3(grid), dim3(kThreads), 0, s, vc, packed, g, w.comp1,
                           as);
    else
        hipLaunchKernelGGL(k_vit_scan, dim3((unsigned)nchunks + head), dim3(kScanT), 0, s, vc,
                           packed, g, w.comp1, w.aent, w.degen, w.plan, w.splitlist, w.splitcount,
                           w.vhead);
    const size_t nbz = (size_t)(vc.emax - vc.emin + 1);
    const size_t lds3x = segp ? std::max((size_t)kW4 * 2, nbz * 16 * 2) * sizeof(double2)
                              : (nbz * 16 * 2 + std::max(nbz * 64 * 2, (size_t)kW4 * 2)) * sizeof(double2);
    // K3 + K3b in one launch: the chunks' irregular blocks run as extra workgroups (segment
    // path: and block 0's walks, one lane per chunk)
    const unsigned heads3 = segp ? (unsigned)((nchunks + kThreads - 1) / kThreads) : 0u;
    hipLaunchKernelGGL(k_vit_exact, dim3(grid + (unsigned)nchunks + heads3), dim3(kThreads), lds3x,
                       s, vc, d_vt, packed, g, w.plan, w.comp3, status, grid, w.aent, w.splitlist,
                       w.splitcount, w.gk, sg, segp ? w.irrseg : nullptr, w.vhead);
    if (segp)
        hipLaunchKernelGGL(k_vit_chain_seg, dim3((unsigned)nchunks), dim3(kSegT), 0, s, vc, packed,
                           g, w.plan, w.comp3, w.degen, w.gk, sg, w.entry, w.went, w.gap,
                           w.barlist, w.vout, w.vhead);
    else
        hipLaunchKernelGGL(k_vit_chain, dim3((unsigned)nchunks), dim3(kChainT), 0, s, vc, packed,
                           g, w.plan, w.comp3, w.degen, w.entry, w.gk, w.gap, w.barlist, w.vout,
                           w.vhead);
    // chunks of whole K5 workgroups: the trace scan runs in each chunk's last K5 workgroup —
    // while the chunks are few (tail_fusion_pays); past that, as its own launch
    if (done5 && nsb % kThreads == 0 && tail_fusion_pays(nchunks)) {
        hipLaunchKernelGGL(k_vit_forward<true>, dim3(grid), dim3(kThreads), 0, s, vc, packed, g,
                           w.degen, w.entry, w.bp, w.origin, status, w.gk, sg, w.went, done5,
                           w.endst, score);
    } else {
        hipLaunchKernelGGL(k_vit_forward<false>, dim3(grid), dim3(kThreads), 0, s, vc, packed, g,
                           w.degen, w.entry, w.bp, w.origin, status, w.gk, sg, w.went, nullptr,
                           nullptr, nullptr);
        hipLaunchKernelGGL(k_vit_tscan, dim3((unsigned)nchunks), dim3(kThreads), 0, s, g, w.entry,
                           w.origin, w.endst, score);
    }
    if (fuse) {   // fused decode: the workgroups are whole island tiles inside one chunk
        if (nsb % kThreads || chunk_len != nsb * kSB || fuse->ws.ntile != nsb / kThreads)
            return hipErrorInvalidValue;
        if (fuse->done)   // the chunk's resolve in its last workgroup
            hipLaunchKernelGGL(k_vit_trace<1>, dim3(grid), dim3(kThreads), 0, s, g, w.bp, w.endst,
                               sign_out, status, zero_at, zero_n, packed, *fuse);
        else              // the tiles only (islands_resolve after it)
            hipLaunchKernelGGL(k_vit_trace<2>, dim3(grid), dim3(kThreads), 0, s, g, w.bp, w.endst,
                               sign_out, status, zero_at, zero_n, packed, *fuse);
    } else {
        hipLaunchKernelGGL(k_vit_trace<0>, dim3(grid), dim3(kThreads), 0, s, g, w.bp, w.endst,
                           sign_out, status, zero_at, zero_n, nullptr, IslFuse{});
    }
    if (degen_out) {
        hipError_t e = hipMemcpyAsync(degen_out, w.degen, nchunks, hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) return e;
    }
    return hipGetLastError();
}

size_t vit_derived_bytes() { return sizeof(VitDerived); }

hipError_t launch_vit_tables(const VitConsts& vc, VitTables* d_vt, hipStream_t s) {
    hipLaunchKernelGGL(k_vit_tables, dim3(128), dim3(kThreads), 0, s, vc, d_vt);
    return hipGetLastError();
}

}  // namespace cpg
