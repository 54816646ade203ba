// k_estep.hip — Baum-Welch E-step (the MAHOUT-627 "rescaling" mapper behind
// BaumWelchDriver.runBaumWelchMR, CpGIslandFinder.java:200; unvendored — the textbook
// Rabiner rescaled forward-backward of SURVEY.md A.3 is the restated convention) on gfx950.
//
// Every 65,536-base chunk is an independent observation sequence (:130-141).  With the
// deterministic emission matrix only two states are live per position, so the chain is a
// product of 2x2 positive matrices M_p (rows: previous state +/-, cols: current state).
// One workgroup (1024 lanes) owns one chunk (16 KiB of packed bases, staged in LDS):
//   1. each lane forms the product of its 64 matrices (power-of-two exponent tracking);
//   2. workgroup prefix / suffix scans give the forward vector entering and the backward
//      vector leaving every lane's 64 positions;
//   3. each lane walks its positions in 16-position mini-blocks, last to first: forward
//      alphas recomputed into registers from 3 checkpoints, then the backward chain with the
//      posterior pair marginals xi_p(i,j) = alpha_{p-1}(i) M_p(i,j) beta_p(j) / Z, beta
//      pre-scaled by 2^47 / Z so that each xi is one fma onto the integer grid (unsigned fixed
//      point 2^-47, round to nearest), accumulated into LDS bins with integer LDS atomics:
//      exact, order-independent sums (measured: fp64 LDS atomics were 2x the integer ones).
// Posteriors are normalised per position, so the scaling scheme (exact powers of two here,
// reciprocal of the sum in the reference) changes results only at rounding level: parity
// with the oracle is by tolerance (tests: 1e-9 relative).  Emission counts follow exactly
// from sum_i xi(i,j) = gamma(j): emit[j] = init[j] + column sum j of trans.
// Per-chunk results are added to 128-bit fixed-point accumulators (64-bit integer atomics
// with carry into a high word: exact, order-independent, so deterministic); the last
// workgroup to finish converts them to the cpg_counts_f64 stripes (one launch per call).

#include <algorithm>
#include <cmath>

#include "count_dev.h"

// The E-step is a tolerance-bound fp64 computation (unlike the bit-exact Viterbi): products
// and sums may be contracted to FMAs here (the fixed-point conversion of a posterior becomes
// one fma(x, rz, 1.5*2^52): a single rounding onto the integer grid).
#pragma clang fp contract(fast)

namespace cpg {
namespace {

constexpr int kET = 1024;               // max lanes per chunk
constexpr int kLanePos = 64;            // positions per lane
// accumulator slab: class bins trans[64] (by dinucleotide x 4) | init[8] | loglik, then the
// two-position blocks' key bins [64 keys][4] (see 3b)
constexpr int kSlabCls = 73;
constexpr int kKeys = 80;               // 64 trinucleotides + 16 one-step keys (lane 0's first block)
constexpr int kKeyRows = 64 * 4;        // LDS bin rows / key accumulators (one-step keys: direct)
constexpr int kSlab = kSlabCls + kKeyRows;
// workgroups add into kAccRep replicated accumulator sets (chosen by chunk index) so that
// ~700 workgroups do not serialise on 73 device-scope atomic addresses; the finalize sums
// the replicas in 128-bit integer arithmetic (exact, order-independent)
constexpr int kAccRep = 16;
// bins: ONE set of 256 rows (row = key * 4 + pair) x 16 columns (u64), lane column = lane % 16.  An LDS 64-bit access serves 16 lanes per cycle with bank = (address /
// 4) mod 32: the 16 lanes of a pass always hit 16 different columns = 32 different banks,
// whatever their classes — no bank conflicts and no same-address collisions inside a pass
// (per-wave replicated sets, measured earlier, collide whenever two lanes of a pass share a
// class).
// LDS: TA/TB (512 B) | T2A/T2B (2.5 KB) | union { 4-step tables, scan buffer, bins } |
// epilogue scratch | alpha checkpoints
constexpr size_t kUnionOff = (32 + 2 * kKeys) * 16;
constexpr size_t kUnionBytes = 2048 * 16;
static_assert(kKeyRows * 16 * 8 <= kUnionBytes, "bins fit the union");

struct Mat {
    double a, b, c, d;   // [[a b] [c d]]
    int e;               // value = 2^e * matrix
};

// floor(log2 mx) for finite mx > 0 (denormals included: v_frexp_exp), 0 for mx == 0 — a
// select, not a branch, so independent normalisations (prefix / suffix scans, forward /
// backward chains) interleave
__device__ __forceinline__ int exp2_floor(double mx) {
    const int k = __builtin_amdgcn_frexp_exp(mx) - 1;
    return mx > 0.0 ? k : 0;
}
__device__ __forceinline__ void mnorm(Mat& m) {
    const double mx = fmax(fmax(m.a, m.b), fmax(m.c, m.d));
    const int k = exp2_floor(mx);
    m.a = ldexp(m.a, -k); m.b = ldexp(m.b, -k); m.c = ldexp(m.c, -k); m.d = ldexp(m.d, -k);
    m.e += k;
}
__device__ __forceinline__ Mat mmul(const Mat& x, const Mat& y) {
    Mat r{x.a * y.a + x.b * y.c, x.a * y.b + x.b * y.d, x.c * y.a + x.d * y.c,
          x.c * y.b + x.d * y.d, x.e + y.e};
    mnorm(r);
    return r;
}
// product without the renormalisation: inside a scan of normalised positive products the
// entries of two or three unnormalised levels stay far inside fp64's range, so the scans
// renormalise only at their last level (a normalisation is ~11 VALU of the ~20 of a product)
__device__ __forceinline__ Mat mmul_nn(const Mat& x, const Mat& y) {
    return {x.a * y.a + x.b * y.c, x.a * y.b + x.b * y.d, x.c * y.a + x.d * y.c,
            x.c * y.b + x.d * y.d, x.e + y.e};
}
__device__ __forceinline__ Mat mid() { return {1.0, 0.0, 0.0, 1.0, 0}; }
__device__ __forceinline__ Mat msel(bool c, const Mat& x, const Mat& y) {   // field selects
    return {c ? x.a : y.a, c ? x.b : y.b, c ? x.c : y.c, c ? x.d : y.d, c ? x.e : y.e};
}
// product of two 2x2 matrices given as rows (x = row 0, y = row 1), not normalised
__device__ __forceinline__ Mat mmul_raw(double2 xa, double2 xb, double2 ya, double2 yb) {
    return {xa.x * ya.x + xa.y * yb.x, xa.x * ya.y + xa.y * yb.y, xb.x * ya.x + xb.y * yb.x,
            xb.x * ya.y + xb.y * yb.y, 0};
}
// DPP moves (VALU, no LDS crossbar): CTRL 0x110+n = row_shr:n, 0x100+n = row_shl:n (inside
// 16-lane rows), 0x138 = wave_shr:1, 0x130 = wave_shl:1.  Lanes without a source take `old`.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v, double old) {
    const long long vi = __double_as_longlong(v), oi = __double_as_longlong(old);
    const int lo = __builtin_amdgcn_update_dpp((int)oi, (int)vi, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(oi >> 32), (int)(vi >> 32), CTRL, 0xF, 0xF,
                                               false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
template <int CTRL>
__device__ __forceinline__ Mat dpp_mat(const Mat& x, const Mat& old) {
    return {dpp_f64<CTRL>(x.a, old.a), dpp_f64<CTRL>(x.b, old.b), dpp_f64<CTRL>(x.c, old.c),
            dpp_f64<CTRL>(x.d, old.d),
            __builtin_amdgcn_update_dpp(old.e, x.e, CTRL, 0xF, 0xF, false)};
}
// x from the lane `off` below (up) / above (down) inside its 16-lane row, identity where
// there is none (off compile-time, < 16): mmul with the identity returns x exactly
__device__ __forceinline__ Mat row_up(const Mat& x, int off) {
    const Mat I = {1.0, 0.0, 0.0, 1.0, 0};
    switch (off) {
        case 1: return dpp_mat<0x111>(x, I);
        case 2: return dpp_mat<0x112>(x, I);
        case 4: return dpp_mat<0x114>(x, I);
        default: return dpp_mat<0x118>(x, I);
    }
}
__device__ __forceinline__ Mat row_down(const Mat& x, int off) {
    const Mat I = {1.0, 0.0, 0.0, 1.0, 0};
    switch (off) {
        case 1: return dpp_mat<0x101>(x, I);
        case 2: return dpp_mat<0x102>(x, I);
        case 4: return dpp_mat<0x104>(x, I);
        default: return dpp_mat<0x108>(x, I);
    }
}
__device__ __forceinline__ Mat shfl_mat(const Mat& x, int src) {
    return {__shfl(x.a, src), __shfl(x.b, src), __shfl(x.c, src), __shfl(x.d, src),
            __shfl(x.e, src)};
}
__device__ __forceinline__ Mat shfl_up_mat(const Mat& x, int d) {
    return {__shfl_up(x.a, d), __shfl_up(x.b, d), __shfl_up(x.c, d), __shfl_up(x.d, d),
            __shfl_up(x.e, d)};
}
__device__ __forceinline__ Mat shfl_down_mat(const Mat& x, int d) {
    return {__shfl_down(x.a, d), __shfl_down(x.b, d), __shfl_down(x.c, d), __shfl_down(x.d, d),
            __shfl_down(x.e, d)};
}

__device__ __forceinline__ int vnorm(double& x, double& y) {   // returns the shift applied
    const int k = exp2_floor(fmax(x, y));
    x = ldexp(x, -k);
    y = ldexp(y, -k);
    return k;
}

// 1/z to full fp64 precision: hardware reciprocal + two Newton steps (explicit fma)
__device__ __forceinline__ double rcp_nr(double z) {
    double r = __builtin_amdgcn_rcp(z);
    double e = fma(-z, r, 1.0);
    r = fma(r, e, r);
    e = fma(-z, r, 1.0);
    return fma(r, e, r);
}

// posterior in [0,1] -> unsigned fixed point 2^-47, rounded to nearest: adding 1.5*2^52
// puts round(y) in the low mantissa bits (exact for 0 <= y < 2^51); subtracting the
// constant's bit pattern leaves the integer.  A chunk's 65,536 positions sum below 2^63,
// so integer LDS atomics are exact and order-independent.
constexpr double kFix = 140737488355328.0;        // 2^47
constexpr double kMagic = 6755399441055744.0;     // 1.5 * 2^52
__device__ __forceinline__ unsigned long long to_fixed_scaled(double y) {   // y = x * 2^47
    return (unsigned long long)__double_as_longlong(y + kMagic) -
           (unsigned long long)__double_as_longlong(kMagic);
}
// K + round(a * b) for a * b in [0, 2^51), K = the bit pattern of 1.5*2^52: one fma onto the
// integer grid, its bits taken as they are.  The xi bins sum these raw patterns; K is removed
// per bin once per chunk (class_count below), not per value.
constexpr unsigned long long kMagicBits = 0x4338000000000000ull;
__device__ __forceinline__ unsigned long long raw_fma(double a, double b) {
    return (unsigned long long)__double_as_longlong(fma(a, b, kMagic));
}
// Every position of class d adds one raw value to each of its 4 bins (k = pair), so all 4 hold
// n_d * K + sum_k y (mod 2^64), and the 4 pairs' y sum to 2^47 per position up to rounding
// (|e| <= 3 per position): S = sum of the 4 = n_d * (4K + 2^47) + e (mod 2^64), where
// 4K + 2^47 = 0x0CE08 << 44 (mod 2^64) and |e| < 2^43.  Bits 44..63 of S (rounded) give
// n_d * 0x0CE08 mod 2^20 = 8 * (n_d * 0x19C1 mod 2^17), and 0x19C1 is odd: n_d (< 2^17) is
// that times its inverse mod 2^17 (0xF641).
__device__ __forceinline__ unsigned long long class_count(unsigned long long S) {
    const unsigned long long q = ((S + (1ull << 43)) >> 44) & 0xFFFFFull;
    return ((q >> 3) * 0xF641ull) & 0x1FFFFull;
}
constexpr int kLogFix = 24;   // log-likelihood fixed point: 2^-24 (|chunk loglik| < 2^30)
// init posteriors (one gamma_0 per chunk and state): fixed point 2^-62, so that a state whose
// gamma_0 is small keeps full relative precision (on the xi bins' 2^-47 grid a chunk's
// gamma_0 of 1e-3 carried a relative error of up to 3.6e-12, summed over the chunks)
constexpr double kFixInit = 4611686018427387904.0;   // 2^62
__device__ __forceinline__ unsigned long long to_fixed_init(double y47) {   // y47 = gamma_0 * 2^47
    return __double2ull_rn(ldexp(y47, 15));
}

// a 64-bit addend (sign-extended when negative) into a split 128-bit accumulator
// (acc_split_add, cpg_internal.h)
__device__ __forceinline__ void acc128_add(unsigned long long* lohi, unsigned long long v,
                                           bool negative) {
    acc_split_add(lohi, v, negative ? ~0ull : 0ull);
}

// the lane's 64 dinucleotide codes (prev | cur << 2), 8 per word, read once from HBM
struct Codes {
    uint32_t w[8];
    uint32_t raw[4], prev;   // the lane's packed words and the word before them
    // 10-bit index of the 5-base window ending at position 4g+3 (4 matrices 4g..4g+3)
    __device__ __forceinline__ uint32_t win(int g) const {   // g compile-time
        const int r = g >> 2, s = g & 3;
        const uint32_t lo = r == 0 ? prev : raw[r - 1];
        return s == 0 ? (__builtin_amdgcn_alignbit(raw[r], lo, 30) & 0x3FFu)
                      : ((raw[r] >> (8 * s - 2)) & 0x3FFu);
    }
    // the 16 codes of mini-block m (m compile-time)
    __device__ __forceinline__ uint64_t mb(int m) const {
        return ((uint64_t)w[2 * m + 1] << 32) | w[2 * m];
    }
};
// 16 2-bit fields -> 16 4-bit fields (in their low 2 bits)
__device__ __forceinline__ uint64_t spread2(uint32_t v) {
    uint64_t x = v;
    x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
    x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
    x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x << 2)) & 0x3333333333333333ull;
    return x;
}
// the 16 dinucleotide codes (prev | cur << 2) of the packed word x; pb = the base before it
__device__ __forceinline__ uint64_t codes16(uint32_t x, uint32_t pb) {
    return spread2((x << 2) | pb) | (spread2(x) << 2);
}
__device__ __forceinline__ uint32_t code_at(uint64_t mb, int i) {   // i compile-time
    return (uint32_t)(mb >> (4 * i)) & 15u;
}
__device__ __forceinline__ Codes lane_codes(const uint32_t* __restrict__ pk, int t) {
    const uint4 v = *reinterpret_cast<const uint4*>(pk + 4 * t);
    const uint32_t ww[4] = {v.x, v.y, v.z, v.w};
    uint32_t prev = t > 0 ? pk[4 * t - 1] : 0u;
    Codes c;
    c.raw[0] = v.x; c.raw[1] = v.y; c.raw[2] = v.z; c.raw[3] = v.w;
    c.prev = prev;
#pragma unroll
    for (int k = 0; k < 8; ++k) c.w[k] = 0u;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int j = r * 16 + i;
            const uint32_t d = (i == 0) ? (__builtin_amdgcn_alignbit(ww[r], prev, 30) & 15u)
                                        : ((ww[r] >> (2 * i - 2)) & 15u);
            c.w[j >> 3] |= d << ((j & 7) * 4);
        }
        prev = ww[r];
    }
    return c;
}

// __shfl_xor(v, m) with the lane address taken from an opaque thread index te (the builtin
// derives it from the lane id, which the compiler then shares with the prologue's shuffles
// and keeps live across the main loop)
__device__ __forceinline__ unsigned long long xor_te(unsigned long long v, int te, int m) {
    const int a = ((te & 63) ^ m) << 2;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)(v >> 32));
    return ((unsigned long long)hi << 32) | lo;
}

template <bool kAgent>
__device__ void finalize(const cpg_model& model, unsigned long long* acc, double* vsum,
                         double* out);
__device__ void final_estep(const double* v, int t, double* __restrict__ out);

// waves per SIMD: the workgroup's 16 waves take 4 per SIMD; with <= 96 VGPRs (5 per SIMD) a
// fifth wave slot and 128 VGPRs per SIMD stay free for the decode stream's kernels, whose
// latency-bound waves then fill this kernel's idle issue slots (overlapped bench +3-4 %,
// tools/ab_libs.sh; a few spills, none of them in the main loop's steady state).  At 4 per
// SIMD (122 VGPRs, no spills) the kernel alone is as fast; 6 per SIMD spills 38.
constexpr int kWavesPerEU = 5;
// kRep (147.5 KB of LDS: one workgroup per CU, nothing co-resides): 4 waves per SIMD, so the
// whole 128-VGPR share of a wave is this kernel's
constexpr int kWavesPerEURep = 4;
// table rows issued this many two-position blocks ahead of their use (forward / backward)
constexpr int kFwdAheadRep = 1, kBwdAheadRep = 1;
// blocks (two positions each) between the alpha renormalisations of the main loop (2: every
// 4 positions)
constexpr int kRenormBlocks = 2;
// kCnt: the fused training pass — each lane also counts its 64 bases' labelled transitions
// (count_dev.h; sign = the label bits), added into the count accumulators cacc, and the last
// workgroup finalizes both (cout: cpg_counts_i64).  Needs >= 256 lanes (chunks >= 16 Ki).
// kRep: the two-step rows (forward and backward) read from a lane-private LDS copy — key k's
// halves at [k][lane & 15], so every ds_read_b128 lane group reads 16 distinct bank quads
// (40 KB more LDS: 147.5 KB per workgroup); otherwise forward rows from the shared LDS rows
// (bank conflicts) and backward rows from L1.  See launch_estep for when.
template <bool kCnt, bool kRep>
__device__ __forceinline__ void estep_chunk(const cpg_model& model, const uint32_t* __restrict__ packed,
                                            int64_t C, unsigned long long* __restrict__ acc,
                                            const double2* __restrict__ gtab, unsigned int* done,
                                            double* __restrict__ out,
                                            const uint32_t* __restrict__ sign,
                                            unsigned long long* __restrict__ cacc,
                                            int64_t* __restrict__ cout, int64_t c, bool fresh) {
    // c: the chunk; fresh: the model's tables are not in LDS yet (a persistent workgroup's
    // first chunk, or every chunk of a one-chunk workgroup)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nl = blockDim.x;             // lanes = C / 64
    const int nw = nl / 64;                // waves
    // conflict-free constant tables: 16 x 16 B each = one 256-B bank row
    double2* TA = reinterpret_cast<double2*>(smem);          // (M(+,+), M(+,-))
    double2* TB = TA + 16;                                    // (M(-,+), M(-,-))
    // one union region after TA/TB, used in turn by: the 4-step tables (phase 1), the scan
    // buffer (phase 2), the xi bins (phase 3) — each phase ends with a barrier
    double2* T2A = TB + 16;                                   // 2-step (P(+,+), P(+,-))
    double2* T2B = T2A + kKeys;                               // 2-step (P(-,+), P(-,-))
    auto* part = reinterpret_cast<unsigned long long*>(
        smem + kUnionOff + kUnionBytes);
    // alpha checkpoints [NMB][nl] (kRep: mini-blocks 1.. only, [NMB - 1][nl]; mini-block 0's
    // stays in registers)
    double2* fck = reinterpret_cast<double2*>(part + 16 * 64);
    constexpr int kCkLds = kRep ? kLanePos / 16 - 1 : kLanePos / 16;
    // kRep: the lane-private row copy of the 64 trinucleotide keys (the one-step keys of lane
    // 0's first block are read from T2A / T2B), then the 4-step tables — all built once per
    // persistent workgroup; otherwise the 4-step tables live in the union, rebuilt per chunk
    double2* RA = fck + (size_t)kCkLds * nl;
    double2* RB = RA + 64 * 16;
    double2* TA4 = kRep ? RB + 64 * 16 : reinterpret_cast<double2*>(smem + kUnionOff);
    unsigned char* uni = smem + kUnionOff;   // scan buffer (phase 2), xi bins (phase 3)
    double2* TB4 = TA4 + 1024;                                // 4-step products, rows 0 / 1
    auto* bins = reinterpret_cast<unsigned long long*>(uni);  // [64 rows][16 columns]
    // the thread index from an opaque copy made per chunk: in the persistent form the compiler
    // would otherwise keep every lane-derived address live across the whole loop (spills)
    int t = threadIdx.x;
    if (kRep) asm volatile("" : "+v"(t));
    const int lane = t & 63;
    const uint32_t* pk = packed + c * (C / 16);
    // the one- and two-step rows from the model's cached table (est_tables: L2-resident, 3 KB)
    // rather than per-lane reads of the kernel-argument model
    if (fresh)
        for (int i = t; i < 32 + 2 * kKeys; i += nl) TA[i] = gtab[i];   // TB, T2A, T2B follow TA
    // (kRep: the lane-private row copy is made by waves 1.. while wave 0 walks the rows, 2c)
    const double2* __restrict__ rA = RA + (t & 15);   // this lane's column of the copy
    const double2* __restrict__ rB = RB + (t & 15);
    const Codes cd0 = lane_codes(pk, t);   // (in flight across the barrier)
    // fused counts: the workgroup's 72 count sums (LDS atomics) and the finalize's raw sums
    // in the epilogue scratch `part` (free until the epilogue's first 76 words)
    uint32_t* scnt = reinterpret_cast<uint32_t*>(part + 128);
    uint2 sg = make_uint2(0u, 0u);
    uint32_t sgp = 0u;
    if (kCnt) {
        if (t < cnt::kRaw) scnt[t] = 0u;
        if (t < 64) {   // wave 0's label words (the other waves load theirs in 2c)
            const uint32_t* sk = sign + c * (C / 32);
            sg = *reinterpret_cast<const uint2*>(sk + 2 * t);
            sgp = sk[t > 0 ? 2 * t - 1 : 0];   // (unconditional; its sign bit taken at use)
        }
    }
    __syncthreads();
    // the lane's 64 bases = one count block (its first is the chunk's first).  Wave 0 counts
    // here; the other waves count while wave 0 walks the rows (2c), where they would wait
    if (kCnt && t < 64) {
        __builtin_amdgcn_sched_barrier(0);   // kept apart from phase 1: registers
        if (t == 0) atomicAdd(&scnt[64 + cnt::init_state(cd0.raw[0], sg.x)], 1u);
        cnt::Lane lc;
        lc.template block<false>(make_uint4(cd0.raw[0], cd0.raw[1], cd0.raw[2], cd0.raw[3]), sg, cd0.prev,
                 sgp >> 31, t == 0, scnt);
        lc.flush(scnt);
        __builtin_amdgcn_sched_barrier(0);
    }
    // 4-step products: window (b0..b4) -> M(b0,b1) M(b1,b2) M(b2,b3) M(b3,b4), from the rows
    // (computing them here measured faster than copying a per-model table: 32 KB of L2 reads
    // per workgroup)
    if (!kRep || fresh)
    for (int i = t; i < 1024; i += nl) {
        double x00 = 1.0, x01 = 0.0, x10 = 0.0, x11 = 1.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int d = (i >> (2 * k)) & 15;   // bases k, k+1 of the window
            const double2 ma = TA[d], mb = TB[d];
            const double n00 = x00 * ma.x + x01 * mb.x, n01 = x00 * ma.y + x01 * mb.y;
            const double n10 = x10 * ma.x + x11 * mb.x, n11 = x10 * ma.y + x11 * mb.y;
            x00 = n00; x01 = n01; x10 = n10; x11 = n11;
        }
        TA4[i] = make_double2(x00, x01);
        TB4[i] = make_double2(x10, x11);
    }
    __syncthreads();
    constexpr int L = kLanePos;            // 64 positions per lane
    constexpr int kMB = 16, NMB = L / kMB;
    const int p0 = t * L;
    // 1. lane product of M_p over its positions: per mini-block, its four 4-step matrices
    //    multiplied as a tree (W0 W1)(W2 W3), then into the running product (position 0
    //    carries no matrix: lane 0's first window is M_1 M_2 M_3).  The running products
    //    after mini-blocks 0 .. NMB-2 (the alpha checkpoints' factors) stay in registers
    //    through the scans (the exponent is dropped: alpha's scale per position is free) —
    //    in LDS they took 96 KB, which kept the decode kernels' workgroups (K3: ~37 KB) off
    //    the training CUs.
    Mat P = mid();
    double4 Pk[NMB - 1];
#pragma unroll
    for (int g = 0; g < NMB; ++g) {
        double2 ra[4], rb[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int gq = 4 * g + j;
            if (gq == 0 && t == 0) {
                double x00 = 1.0, x01 = 0.0, x10 = 0.0, x11 = 1.0;
                const uint64_t cm = cd0.mb(0);
#pragma unroll
                for (int i = 1; i < 4; ++i) {
                    const uint32_t d = code_at(cm, i);
                    const double2 ma = TA[d], mb = TB[d];
                    const double n00 = x00 * ma.x + x01 * mb.x, n01 = x00 * ma.y + x01 * mb.y;
                    const double n10 = x10 * ma.x + x11 * mb.x, n11 = x10 * ma.y + x11 * mb.y;
                    x00 = n00; x01 = n01; x10 = n10; x11 = n11;
                }
                ra[j] = make_double2(x00, x01);
                rb[j] = make_double2(x10, x11);
            } else {
                const uint32_t wi = cd0.win(gq);
                ra[j] = TA4[wi];
                rb[j] = TB4[wi];
            }
        }
        const Mat w01 = mmul_raw(ra[0], rb[0], ra[1], rb[1]);
        const Mat w23 = mmul_raw(ra[2], rb[2], ra[3], rb[3]);
        const Mat G{w01.a * w23.a + w01.b * w23.c, w01.a * w23.b + w01.b * w23.d,
                    w01.c * w23.a + w01.d * w23.c, w01.c * w23.b + w01.d * w23.d, 0};
        P = mmul(P, G);   // normalised
        if (g < NMB - 1) Pk[g] = make_double4(P.a, P.b, P.c, P.d);
    }
    // 2. alpha entering and beta leaving every lane.  (a) prefix and suffix products of the
    //    lane products inside each 16-lane row (DPP, identity at the row edges); (b) the 64
    //    row totals to LDS; (c) one wave: 16 lanes form the totals of 4 rows each, scan them
    //    (DPP) and walk their 4 rows with VECTORS — alpha entering / beta leaving every row
    //    (one mat-vec per row, exponents tracked for the log-likelihood) — to LDS; (d) every
    //    lane: alpha = its row's entering alpha x the row prefix before it, beta likewise.
    //    Two barriers; no cross-row matrix shuffles.
    Mat xp = P, xs = P;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {   // inside rows: DPP (identity at row edges)
        const Mat yp = row_up(xp, off), ys = row_down(xs, off);
        xp = off < 8 ? mmul_nn(yp, xp) : mmul(yp, xp);
        xs = off < 8 ? mmul_nn(xs, ys) : mmul(xs, ys);
    }
    const Mat up1 = row_up(xp, 1), dn1 = row_down(xs, 1);   // exclusive, inside the row
    // (the scan buffer lies outside the union: no barrier for the 4-step table reads here)
    const int nr = nl >> 4, row = t >> 4;                      // rows of 16 lanes
    // (the epilogue scratch after the count sums; 4.6 KB)
    Mat* sRP = reinterpret_cast<Mat*>(part + 192);             // [64] row totals
    double2* sAR = reinterpret_cast<double2*>(sRP + 64);       // [64] alpha entering row r
    double2* sBR = sAR + 64;                                   // [64] beta leaving row r
    double* sLL = reinterpret_cast<double*>(sBR + 64);         // the chunk log-likelihood
    if ((t & 15) == 15) sRP[row] = xp;   // (the same product as the suffix scan's lane 0)
    const uint32_t o0 = pk[0] & 3u;
    const double fa = model.pi[o0], fb = model.pi[o0 + 4];   // alpha_0 (b = 1 when live)
    __syncthreads();
    if (t < 64) {
        // lane r: row r (rows past nr: identity).  Inclusive prefix and suffix products of the
        // 64 row totals — DPP inside 16-lane rows, then two cross-row levels by shuffles —
        // give alpha entering and beta leaving every row as ONE mat-vec each (round 5: the
        // walk of 4 rows per lane by 16 lanes had been a chain of 4 + 4 dependent steps)
        const int r = t;
        const Mat x = r < nr ? sRP[r] : mid();
        Mat xp = x, xs = x;
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
            const Mat yp = row_up(xp, off), ys = row_down(xs, off);
            xp = off < 8 ? mmul_nn(yp, xp) : mmul(yp, xp);
            xs = off < 8 ? mmul_nn(xs, ys) : mmul(xs, ys);
        }
#pragma unroll
        for (int off = 16; off < 64; off <<= 1) {   // across the 16-lane rows
            Mat yp = shfl_up_mat(xp, off), ys = shfl_down_mat(xs, off);
            if (r < off) yp = mid();
            if (r + off >= 64) ys = mid();
            xp = mmul(yp, xp);
            xs = mmul(xs, ys);
        }
        Mat ep = shfl_up_mat(xp, 1), es = shfl_down_mat(xs, 1);   // rows before / after r
        if (r == 0) ep = mid();
        if (r == 63) es = mid();
        // alpha entering row r: alpha_0 x the rows before; beta leaving it: the rows after x 1
        double vP = fa * ep.a + fb * ep.c, vM = fa * ep.b + fb * ep.d;
        vnorm(vP, vM);
        double uP = es.a + es.b, uM = es.c + es.d;
        vnorm(uP, uM);
        if (r < nr) {
            sAR[r] = make_double2(vP, vM);
            sBR[r] = make_double2(uP, uM);
        }
        if (r == 63) {   // the chunk log-likelihood: alpha_0 x all rows (lane 63's inclusive)
            double aP = fa * xp.a + fb * xp.c, aM = fa * xp.b + fb * xp.d;
            const int k = vnorm(aP, aM);
            *sLL = log(aP + aM) + (double)(xp.e + k) * 0.69314718055994530942;
        }
    } else {
        // waves 1..: work that would otherwise sit in the prologue's critical path —
        // the lane-private row copy (kRep) and the labelled counts of their blocks (kCnt,
        // the words reloaded: nothing kept live across the scans)
        // every lane is past its 4-step table reads (phase 1, before the barrier above): the
        // union becomes the bins
        for (int i = t - 64; i < kKeyRows * 16; i += nl - 64) bins[i] = 0ull;
        if (kRep && fresh)
            for (int i = t - 64; i < 64 * 16; i += nl - 64) {
                RA[i] = gtab[32 + (i >> 4)];
                RB[i] = gtab[32 + kKeys + (i >> 4)];
            }
        if (kCnt) {
            const uint4 w = *reinterpret_cast<const uint4*>(pk + 4 * t);
            const uint32_t wp = pk[4 * t - 1];
            const uint32_t* sk = sign + c * (C / 32);
            const uint2 sw = *reinterpret_cast<const uint2*>(sk + 2 * t);
            const uint32_t swp = sk[2 * t - 1];
            cnt::Lane lc;
            lc.template block<false>(w, sw, wp, swp >> 31, false, scnt);
            lc.flush(scnt);
        }
    }
    __syncthreads();
    // the union has become the bins: zeroed by waves 1.. during the walk (2c), or here by the
    // only wave (its own LDS accesses stay in order: no barrier before the main loop either)
    if (nl == 64) {
        for (int i = t; i < kKeyRows * 16; i += nl) bins[i] = 0ull;
        if (kRep && fresh)   // (the one wave makes the row copy too: chunks of 4,096 bases)
            for (int i = t; i < 64 * 16; i += nl) {
                RA[i] = gtab[32 + (i >> 4)];
                RB[i] = gtab[32 + kKeys + (i >> 4)];
            }
    }
    unsigned long long* racc = acc + 2 * kSlab * (c % kAccRep);
    if (t == nl - 1) {   // the chunk log-likelihood, in signed 2^-24 units (added now: nothing
                         // stays live across the main loop)
        const long long L = llrint(ldexp(*sLL, kLogFix));
        acc128_add(racc + 2 * 72, (unsigned long long)L, L < 0);
    }
    double aP = fa, aM = fb;   // alpha at position p0-1 (t > 0); alpha_0 for t == 0
    if (t > 0) {
        const double2 ar = sAR[row];
        aP = ar.x * up1.a + ar.y * up1.c;
        aM = ar.x * up1.b + ar.y * up1.d;
    }
    vnorm(aP, aM);
    double bP, bM;   // beta at the lane's last position
    {
        const double2 br = sBR[row];
        bP = dn1.a * br.x + dn1.b * br.y;
        bM = dn1.c * br.x + dn1.d * br.y;
    }
    vnorm(bP, bM);
    // the alpha checkpoints (see 3a) of every mini-block in LDS ([m][lane], 16 B: a wave's
    // row is conflict-free per 8-lane pass); mini-block 0's is (aP, aM) itself (no register
    // stays live across the main loop for it)
#pragma unroll
    for (int m = 1; m < NMB; ++m) {
        const double4 A = Pk[m - 1];
        double xP = aP * A.x + aM * A.z, xM = aP * A.y + aM * A.w;
        vnorm(xP, xM);
        fck[(m - (kRep ? 1 : 0)) * nl + t] = make_double2(xP, xM);
    }
    if (!kRep) fck[t] = make_double2(aP, aM);
    const double2 ck0 = make_double2(aP, aM);   // (kRep: mini-block 0's checkpoint, see 3b)
    // (no barrier: a lane reads only its own checkpoints; the bins were zeroed before the
    // walk's barrier)

    // 3a. (bins zeroed above) alpha entering mini-block m = alpha entering the lane times
    //     phase 1's product of the first m mini-blocks (any per-position scale cancels in the
    //     normalised posteriors)
    // 3b. mini-blocks, last to first, in TWO-POSITION BLOCKS: block j of a mini-block is its
    //     positions (2j, 2j+1), keyed by the trinucleotide tau = (x_{2j-1}, x_{2j}, x_{2j+1})
    //     and stepped by the 2-step matrix P_tau = M_{2j} M_{2j+1} (T2A/T2B).  Forward: the
    //     alphas A_j = alpha_{2j-1} of the 8 blocks in registers (the whole mini-block: no
    //     second forward pass).  Backward: beta pre-scaled by 2^47 / Z as in one-step form —
    //     A_j . (P_tau y_{2j+1}) = 2^47 at every block — so the joint posterior of the states
    //     at 2j-1 and 2j+1,  Zeta(a,c) * 2^47 = A_j(a) * (P_tau(a,c) y(c)),  is one fma onto
    //     the fixed-point grid; both positions' pair posteriors are exact linear images of it
    //     (xi_{2j}(a,b) = sum_c f(a,b,c) Zeta(a,c), xi_{2j+1}(b,c) = sum_a f(a,b,c) Zeta(a,c),
    //     f(a,b,c) = M(a,b) M(b,c) / P(a,c): the share of the paths a -> c through b), applied
    //     once to the exact integer sums in the finalize.  4 LDS atomics per TWO positions,
    //     one table row pair per two positions each way, ~half the fp64 of one-step form.
    //     Lane 0's first block holds position 1 alone (position 0 carries no transition): its
    //     key 64 + class(x0, x1) selects the one-step matrix, its Zeta IS xi_1 (added to the
    //     class accumulators directly) and it ends with gamma_0 (the init posteriors).
    unsigned long long* wb = bins + (lane & 15);
    constexpr int kBS = 16;   // row stride
    const double2* __restrict__ g2a = gtab + 32;          // backward rows (global, L1-resident)
    const double2* __restrict__ g2b = gtab + 32 + kKeys;
    double yP = bP, yM = bM;   // beta at the last position of the mini-block
    // kRep rows: the 64 trinucleotide keys from this lane's column of the copy, the one-step
    // keys (64 ..: lane 0's first block only) from T2A / T2B — one load from a selected address
    auto repA = [&](uint32_t kk) { return *(kk < 64u ? rA + kk * 16 : T2A + kk); };
    auto repB = [&](uint32_t kk) { return *(kk < 64u ? rB + kk * 16 : T2B + kk); };
#pragma unroll 1
    for (int m = NMB - 1; m >= 0; --m) {
        // the mini-block's bases from its packed word and the last base of the word before:
        // base q at bits 2q+2 of cm, base -1 at bits 0-1; block j's key = bits 4j .. 4j+5
        const uint32_t xw = pk[4 * t + m];
        const uint32_t pw = (t > 0 || m > 0) ? pk[4 * t + m - 1] : 0u;
        const uint64_t cm = ((uint64_t)xw << 2) | (pw >> 30);
        const bool sp = t == 0 && m == 0;
        auto key = [&](int j) -> uint32_t {   // j compile-time
            const uint32_t k = (uint32_t)(cm >> (4 * j)) & 63u;
            return (j == 0 && sp) ? 64u + (k >> 2) : k;
        };
        // alpha at the position before the mini-block.  kRep: mini-block m >= 1's from slot
        // m - 1; the last mini-block's slot, read first, then takes mini-block 0's (its
        // register dies here)
        const int ci = kRep ? (m == 0 ? NMB - 2 : m - 1) : m;
        const double2 f = fck[ci * nl + t];
        if (kRep && m == NMB - 1) fck[(NMB - 2) * nl + t] = ck0;
        constexpr int kB = kMB / 2;          // blocks per mini-block
        double alP[kB], alM[kB];
        // alpha renormalised after every kRNB blocks (2: positions 3, 7, 11, 15, i.e. A_2, A_4,
        // A_6, A_8); kf = the power-of-two shifts applied there
        constexpr int kRNB = kRenormBlocks;
        int kf[kB / kRNB];
        double xP = f.x, xM = f.y;
        // the rows are issued kFPD steps ahead (the scheduling barrier keeps them there: the
        // compiler had waited for each step's reads right before using them, one LDS round
        // trip on every step of the chain)
        constexpr int kFPD = kRep ? kFwdAheadRep : 1;   // (2: one spill at 96 VGPRs and no faster)
        double2 fa[kFPD + 1], fb[kFPD + 1];
#pragma unroll
        for (int j = 0; j < kFPD; ++j) {
            fa[j] = kRep ? repA(key(j)) : T2A[key(j)];
            fb[j] = kRep ? repB(key(j)) : T2B[key(j)];
        }
#pragma unroll
        for (int j = 0; j < kB; ++j) {
            alP[j] = xP;
            alM[j] = xM;
            if (j + kFPD < kB) {
                fa[(j + kFPD) % (kFPD + 1)] = kRep ? repA(key(j + kFPD)) : T2A[key(j + kFPD)];
                fb[(j + kFPD) % (kFPD + 1)] = kRep ? repB(key(j + kFPD)) : T2B[key(j + kFPD)];
            }
            __builtin_amdgcn_sched_barrier(0);
            const double2 ma = fa[j % (kFPD + 1)], mb = fb[j % (kFPD + 1)];
            const double nP = xP * ma.x + xM * mb.x, nM = xP * ma.y + xM * mb.y;
            xP = nP;
            xM = nM;
            if ((j + 1) % kRNB == 0) kf[(j + 1) / kRNB - 1] = vnorm(xP, xM);
        }
        // y_15 = beta_15 * 2^{47 - s_15} / (A_8 . beta_15)  (A_8 = alpha_15 after its shift)
        vnorm(yP, yM);
        {
            const double r = ldexp(rcp_nr(xP * yP + xM * yM), 47 - kf[kB / kRNB - 1]);
            yP *= r;
            yM *= r;
        }
        constexpr int kPFD = kRep ? kBwdAheadRep : 1;   // backward rows this many blocks ahead
        double2 qa[kPFD + 1], qb[kPFD + 1];
#pragma unroll
        for (int j = 0; j < kPFD; ++j) {
            const uint32_t k = key(kB - 1 - j);
            qa[j] = kRep ? repA(k) : g2a[k];
            qb[j] = kRep ? repB(k) : g2b[k];
        }
#pragma unroll
        for (int j = kB - 1; j >= 0; --j) {
            // rows issued kPFD blocks ahead; the scheduling barrier keeps the compiler from
            // sinking them to their use (one L1/L2 round trip on every block's chain)
            if (j - kPFD >= 0) {
                const uint32_t k = key(j - kPFD);
                qa[(kB - 1 - j + kPFD) % (kPFD + 1)] = kRep ? repA(k) : g2a[k];
                qb[(kB - 1 - j + kPFD) % (kPFD + 1)] = kRep ? repB(k) : g2b[k];
            }
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t k = key(j);
            const double2 ma = qa[(kB - 1 - j) % (kPFD + 1)], mb = qb[(kB - 1 - j) % (kPFD + 1)];
            // P y products, shared by the joint posteriors and the beta update
            const double t00 = ma.x * yP, t01 = ma.y * yM, t10 = mb.x * yP, t11 = mb.y * yM;
            if (j == 0 && sp) {   // xi_1 and gamma_0, added at once to the class and init
                                  // accumulators (nothing stays live across the main loop)
                const uint32_t d = k - 64u;
                acc128_add(racc + 2 * (d * 4 + 0), to_fixed_scaled(alP[0] * t00), false);
                acc128_add(racc + 2 * (d * 4 + 1), to_fixed_scaled(alP[0] * t01), false);
                acc128_add(racc + 2 * (d * 4 + 2), to_fixed_scaled(alM[0] * t10), false);
                acc128_add(racc + 2 * (d * 4 + 3), to_fixed_scaled(alM[0] * t11), false);
                const uint32_t b0 = xw & 3u;
                acc128_add(racc + 2 * (64 + b0), to_fixed_init(alP[0] * (t00 + t01)), false);
                acc128_add(racc + 2 * (64 + b0 + 4), to_fixed_init(alM[0] * (t10 + t11)), false);
            } else {
                unsigned long long* row = wb + (int)k * (4 * kBS);
                atomicAdd(row + 0 * kBS, raw_fma(alP[j], t00));
                atomicAdd(row + 1 * kBS, raw_fma(alP[j], t01));
                atomicAdd(row + 2 * kBS, raw_fma(alM[j], t10));
                atomicAdd(row + 3 * kBS, raw_fma(alM[j], t11));
            }
            yP = t00 + t01;
            yM = t10 + t11;
            if (j > 0 && j % kRNB == 0) {   // crossing A_j's renormalisation point
                yP = ldexp(yP, -kf[j / kRNB - 1]);
                yM = ldexp(yM, -kf[j / kRNB - 1]);
            }
        }
    }
    __syncthreads();
    // the epilogue's indices from an opaque copy of the thread index: the compiler would
    // otherwise keep the prologue's (shuffle) indices live across the main loop, in scratch
    int te = threadIdx.x;
    asm volatile("" : "+v"(te));
    // chunk totals: row te = key * 4 + (2a + c), the sum of its 16 columns (integer: exact in
    // any order); the key's 4 raw sums (lanes 4 key .. 4 key + 3 of one wave) -> its block
    // count -> K removed -> the key accumulators (slots kSlabCls + row)
    if (nl == 4 * kKeyRows) {   // the reference's chunk: 4 lanes per row, 4 columns each
        const int r = te >> 2, q = te & 3;
        const unsigned long long* row = bins + r * 16 + 4 * q;
        unsigned long long s = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) s += row[(i + r) & 3];   // rotated: 16 lanes, 16 columns
        s += xor_te(s, te, 1);   // the row's sum (lane addresses from te, see above)
        s += xor_te(s, te, 2);
        unsigned long long S = s;
        S += xor_te(S, te, 4);   // the key's 4 rows
        S += xor_te(S, te, 8);
        s -= class_count(S) * kMagicBits;
        if (q == 0 && s) acc128_add(racc + 2 * (kSlabCls + r), s, false);
    } else {
        for (int r = te; r < kKeyRows; r += nl) {   // (nl: a multiple of 64)
            const unsigned long long* row = bins + r * 16;
            unsigned long long s = 0;
#pragma unroll
            for (int col = 0; col < 16; ++col) s += row[(col + r) & 15];   // rotated: no conflicts
            unsigned long long S = s;
            S += xor_te(S, te, 1);   // (lane addresses from te, see above)
            S += xor_te(S, te, 2);
            s -= class_count(S) * kMagicBits;
            if (s) acc128_add(racc + 2 * (kSlabCls + r), s, false);
        }
    }
    if (kCnt && te < cnt::kRaw) {   // the count sums (kCnt: >= 256 lanes)
        const uint32_t v = cnt::raw_of(scnt, te);
        if (v) atomicAdd(cacc + (c % cnt::kRep) * cnt::kRaw + te, (unsigned long long)v);
    }
    // done != nullptr: the last workgroup to finish converts the sums (one launch per call)
    if (done && last_workgroup(done, reinterpret_cast<int*>(part))) {
        // the count replicas are read by waves 2-3 beside the E-step's (finalize's barrier)
        uint64_t* craw = reinterpret_cast<uint64_t*>(part + 192);
        if (kCnt && te >= 128 && te < 128 + cnt::kRaw) cnt::fin_load<true>(cacc, craw, te - 128);
        finalize<true>(model, acc, reinterpret_cast<double*>(part + 512), out);
        if (kCnt) cnt::fin_store(cacc, craw, cout, te, nl);
        reset_done(done);
    }
}

template <bool kCnt>
__global__ __launch_bounds__(kET) __attribute__((amdgpu_waves_per_eu(kWavesPerEU)))
void k_estep_chunk(const cpg_model model, const uint32_t* __restrict__ packed, int64_t C,
                   unsigned long long* __restrict__ acc, const double2* __restrict__ gtab,
                   unsigned int* done, double* __restrict__ out,
                   const uint32_t* __restrict__ sign, unsigned long long* __restrict__ cacc,
                   int64_t* __restrict__ cout) {
    estep_chunk<kCnt, false>(model, packed, C, acc, gtab, done, out, sign, cacc, cout, blockIdx.x,
                             true);
}
// the long launches' form (kRep): lane-private row copies, the registers of 4 waves per SIMD,
// and kRepRun consecutive chunks per workgroup — the model's tables, the lane-private row copy
// and the 4-step tables made once per workgroup instead of once per chunk, kRepRun - 1
// workgroup launches fewer.  (Persistent workgroups, one per CU taking chunks from a work
// counter, were faster alone but never gave a compute unit back: beside the decode stream
// they starved its kernels for milliseconds; a run of a few chunks returns each CU every
// ~0.1 ms.)
constexpr int kRepRun = 4;
template <bool kCnt>
__global__ __launch_bounds__(kET) __attribute__((amdgpu_waves_per_eu(kWavesPerEURep)))
void k_estep_chunk_rep(const cpg_model model, const uint32_t* __restrict__ packed, int64_t C,
                       unsigned long long* __restrict__ acc, const double2* __restrict__ gtab,
                       double* __restrict__ out, const uint32_t* __restrict__ sign,
                       unsigned long long* __restrict__ cacc, int64_t* __restrict__ cout,
                       int64_t nchunks) {
    // chunks blockIdx.x + i * gridDim.x: the workgroups running at one time hold consecutive
    // chunks, so their accumulator replicas (c % kAccRep) are all in use (runs of consecutive
    // chunks per workgroup put every resident workgroup on a quarter of them)
    for (int64_t c = blockIdx.x, i = 0; i < kRepRun && c < nchunks; ++i, c += gridDim.x) {
        estep_chunk<kCnt, true>(model, packed, C, acc, gtab, nullptr, out, sign, cacc, cout, c,
                                i == 0);
        __syncthreads();   // (the chunk's LDS reads are done before the next chunk's writes)
    }
}


// The accumulators (replicas summed in 128-bit integer arithmetic) -> doubles, re-zeroed
// for the next call; the key bins of the two-position blocks mapped onto the class bins
// (k_estep_chunk 3b: xi_{2j}(a,b) = sum_c f Zeta(a,c), xi_{2j+1}(b,c) = sum_a f Zeta(a,c)
// with f(a,b,c) = M1(a,b) M2(b,c) / sum_b' M1(a,b') M2(b',c), M1 / M2 the one-step matrices
// of the key's two classes); then the cpg_counts_f64 assembly.  kAgent: written by
// workgroups of the same launch (device-scope loads).
template <bool kAgent>
__device__ void finalize(const cpg_model& model, unsigned long long* acc, double* vsum,
                         double* out) {
    const int t = threadIdx.x;
    for (int i = t; i < kSlab; i += blockDim.x) {
        unsigned long long s0 = 0ull, s1 = 0ull;   // the replicas' split sums
        for (int r = 0; r < kAccRep; ++r) {
            const unsigned long long* a = acc + 2 * (r * kSlab + i);
            s0 += kAgent ? load_agent(a) : a[0];
            s1 += kAgent ? load_agent(a + 1) : a[1];
        }
        unsigned long long lo, hi;   // 128-bit value
        acc_sum128(s0, s1, lo, hi);
        const bool neg = (long long)hi < 0;   // only the log-likelihood row can be negative
        if (neg) {                             // magnitude first: no cancellation
            lo = ~lo + 1ull;
            hi = ~hi + (lo == 0ull ? 1ull : 0ull);
        }
        const double mag = (double)hi * 18446744073709551616.0 + (double)lo;
        vsum[i] = i < 64 ? mag * (1.0 / kFix)
                : i < 72 ? mag * (1.0 / kFixInit)
                : i == 72 ? ldexp(neg ? -mag : mag, -kLogFix) : mag * (1.0 / kFix);
    }
    __syncthreads();
    for (int i = t; i < 2 * kSlab * kAccRep; i += blockDim.x) acc[i] = 0ull;
    double xs = 0.0;
    if (t < 64) {   // class bin t = d * 4 + 2a + b
        const int d = t >> 2, a = (t >> 1) & 1, b = t & 1;
        // M_e(s, s') = a[p + 4s][q + 4s'], e = p | q << 2 (p the previous base, q the current)
        auto M = [&](int e, int s, int s2) { return model.a[(e & 3) + 4 * s][(e >> 2) + 4 * s2]; };
        auto share = [&](int d1, int d2, int x, int y, int z) {   // f(x, y, z)
            const double w0 = M(d1, x, 0) * M(d2, 0, z), w1 = M(d1, x, 1) * M(d2, 1, z);
            const double w = w0 + w1;
            return w > 0.0 ? (y ? w1 : w0) / w : 0.0;
        };
        const double* zk = vsum + kSlabCls;
        for (int r = 0; r < 4; ++r) {   // keys whose first position has class d: (a, b) first
            const int key = d | (r << 4), d2 = key >> 2;
            for (int cc = 0; cc < 2; ++cc)
                xs += share(d, d2, a, b, cc) * zk[key * 4 + 2 * a + cc];
        }
        for (int p = 0; p < 4; ++p) {   // keys whose second position has class d: (a, b) second
            const int key = p | (d << 2), d1 = key & 15;
            for (int aa = 0; aa < 2; ++aa)
                xs += share(d1, d, aa, a, b) * zk[key * 4 + 2 * aa + b];
        }
    }
    __syncthreads();
    if (t < 64) vsum[t] += xs;
    __syncthreads();
    for (int i = t; i < 105; i += blockDim.x) final_estep(vsum, i, out);
}

// One workgroup: finalize of accumulators filled by earlier launches (streamed genome,
// contig batches).
__global__ __launch_bounds__(256) void k_estep_final(const cpg_model model,
                                                     unsigned long long* __restrict__ acc,
                                                     double* __restrict__ out) {
    __shared__ double vsum[kSlab];
    finalize<false>(model, acc, vsum, out);
}

// The long launches' finalize as its own one-workgroup launch (both outputs of a training
// pass): the chunk kernel then skips the last-workgroup protocol — the wait for every one of
// its atomics, two barriers and a returning device-scope atomic per workgroup (0.7 us of a
// workgroup's ~27, stamped) — for one launch per call.
__global__ __launch_bounds__(256) void k_train_final(const cpg_model model,
                                                     unsigned long long* __restrict__ acc,
                                                     double* __restrict__ out,
                                                     unsigned long long* __restrict__ cacc,
                                                     int64_t* __restrict__ cout) {
    __shared__ double vsum[kSlab];
    __shared__ uint64_t craw[cnt::kRaw];
    if (cacc && threadIdx.x < cnt::kRaw) cnt::fin_load<false>(cacc, craw, threadIdx.x);
    finalize<false>(model, acc, vsum, out);   // (its barriers order craw too)
    if (cacc) cnt::fin_store(cacc, craw, cout, threadIdx.x, blockDim.x);
}

// cpg_counts_f64 from the 73 sums: init[8] trans[8][8] emit[8][4] loglik; thread t < 105
__device__ void final_estep(const double* v, int t, double* __restrict__ out) {
    double r = 0.0;
    if (t < 8) {
        r = v[64 + t];
    } else if (t < 72) {
        const int i = (t - 8) >> 3, j = (t - 8) & 7;
        const int d = (i & 3) | ((j & 3) << 2);
        r = v[d * 4 + (i >> 2) * 2 + (j >> 2)];
    } else if (t < 104) {
        const int jj = (t - 72) >> 2, k = (t - 72) & 3;
        if (k == (jj & 3)) {                       // emit[j] = init[j] + sum_i trans[i][j]
            r = v[64 + jj];
            for (int i = 0; i < 8; ++i) {
                const int d = (i & 3) | ((jj & 3) << 2);
                r += v[d * 4 + (i >> 2) * 2 + (jj >> 2)];
            }
        }
    } else {
        r = v[72];
    }
    out[t] = r;
}

}  // namespace

// accumulators | done counter (in the 1 KiB tail)
size_t estep_ws_bytes(int64_t, int64_t) { return (size_t)2 * kSlab * 8 * kAccRep + 1024; }

namespace {
size_t estep_lds(int lanes, bool rep) {   // the union is sized for 16 waves; fewer lanes use a prefix
    // (kRep: checkpoints of mini-blocks 1.., the 64-key row copy, the 4-step tables)
    const size_t ck = (size_t)(kLanePos / 16 - (rep ? 1 : 0)) * lanes * sizeof(double2);
    return kUnionOff + kUnionBytes + 16 * 64 * sizeof(unsigned long long) + ck +
           (rep ? ((size_t)64 * 16 * 2 + 2 * 1024) * sizeof(double2) : 0);
}
// The lane-private row copy (kRep) makes the pass itself 7-10 % faster (46 Mbp: 0.0959 ->
// 0.0887 ms; 3.1 Gbp: 4.89 -> 4.38 ms) but takes 40 KB of LDS from the decode kernels that
// share the training CUs: the overlapped C2 step (702 chunks) lost 2.5 %, the C3 genome on one
// GPU (47,303 chunks) gained 7 % (365-372 -> 395-397 Gbase/s; profiles/r04_rep/).  Used from
// 2,048 chunks (128 Mbp) on: the multi-GPU C3 shards (5,900 chunks at 8 GPUs) and up.
constexpr int64_t kEstRepMinChunks = 2048;
// from this many chunks the finalize runs as its own launch (k_train_final): a launch costs
// ~2-4 us, the last-workgroup protocol ~0.7 us per round of workgroups
constexpr int64_t kEstSepFinMinChunks = 2048;
unsigned est_rep_grid(int64_t nchunks) { return (unsigned)((nchunks + kRepRun - 1) / kRepRun); }
}  // namespace

hipError_t launch_estep(const cpg_model& model, const uint32_t* packed, int64_t nchunks,
                        int64_t C, unsigned long long* acc, double* out, hipStream_t s,
                        int parts, const double2* gtab) {
    if (C % 4096 || C > (int64_t)kET * kLanePos) return hipErrorInvalidValue;
    if (nchunks == 0 && parts == PART_ALL)
        return hipMemsetAsync(out, 0, 105 * sizeof(double), s);
    if ((parts & PART_ACC) && nchunks > 0) {
        const int lanes = (int)(C / kLanePos);
        if (!gtab) return hipErrorInvalidValue;   // est_tables
        const bool sepfin = parts == PART_ALL && nchunks >= kEstSepFinMinChunks;
        unsigned int* done = parts == PART_ALL && !sepfin
                                 ? reinterpret_cast<unsigned int*>(acc + 2 * kSlab * kAccRep) : nullptr;
        if (nchunks >= kEstRepMinChunks && !done)
            hipLaunchKernelGGL((k_estep_chunk_rep<false>), dim3(est_rep_grid(nchunks)),
                               dim3(lanes), estep_lds(lanes, true), s, model, packed, C, acc, gtab,
                               out, nullptr, nullptr, nullptr, nchunks);
        else
            hipLaunchKernelGGL((k_estep_chunk<false>), dim3((unsigned)nchunks), dim3(lanes),
                               estep_lds(lanes, false), s, model, packed, C, acc, gtab, done, out,
                               nullptr, nullptr, nullptr);
        if (sepfin) {
            hipLaunchKernelGGL(k_train_final, dim3(1), dim3(256), 0, s, model, acc, out, nullptr,
                               nullptr);
            return hipGetLastError();
        }
        if (done) return hipGetLastError();
    }
    if (parts & PART_FINAL)
        hipLaunchKernelGGL(k_estep_final, dim3(1), dim3(256), 0, s, model, acc, out);
    return hipGetLastError();
}

bool train_fusable(int64_t C) { return C % 4096 == 0 && C >= 16384 && C <= (int64_t)kET * kLanePos; }

hipError_t launch_train(const cpg_model& model, const uint32_t* packed, const uint32_t* sign,
                        int64_t nchunks, int64_t C, unsigned long long* acc, double* out,
                        unsigned long long* cacc, int64_t* cout, hipStream_t s,
                        const double2* gtab) {
    if (!train_fusable(C) || !gtab) return hipErrorInvalidValue;
    if (nchunks == 0) {
        hipError_t e = hipMemsetAsync(out, 0, 105 * sizeof(double), s);
        return e != hipSuccess ? e : hipMemsetAsync(cout, 0, 124 * sizeof(int64_t), s);
    }
    const int lanes = (int)(C / kLanePos);
    const bool sepfin = nchunks >= kEstSepFinMinChunks;
    unsigned int* done =
        sepfin ? nullptr : reinterpret_cast<unsigned int*>(acc + 2 * kSlab * kAccRep);
    if (nchunks >= kEstRepMinChunks && !done)
        hipLaunchKernelGGL((k_estep_chunk_rep<true>), dim3(est_rep_grid(nchunks)), dim3(lanes),
                           estep_lds(lanes, true), s, model, packed, C, acc, gtab, out, sign, cacc,
                           cout, nchunks);
    else
        hipLaunchKernelGGL((k_estep_chunk<true>), dim3((unsigned)nchunks), dim3(lanes),
                           estep_lds(lanes, false), s, model, packed, C, acc, gtab, done, out, sign,
                           cacc, cout);
    if (sepfin)
        hipLaunchKernelGGL(k_train_final, dim3(1), dim3(256), 0, s, model, acc, out, cacc, cout);
    return hipGetLastError();
}

}  // namespace cpg
