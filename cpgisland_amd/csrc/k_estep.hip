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
//   3. each lane walks its positions in 16-position mini-blocks: forward alphas kept in
//      registers, backward betas from 3 checkpoints, posterior pair marginals xi_p(i,j)
//      = alpha_{p-1}(i) M_p(i,j) beta_p(j) / Z_p accumulated into per-wave LDS bins in
//      unsigned fixed point (2^-47, round to nearest) with integer LDS atomics: exact,
//      order-independent sums (measured: fp64 LDS atomics were 2x the integer ones).
// Posteriors are normalised per position, so the scaling scheme (exact powers of two here,
// reciprocal of the sum in the reference) changes results only at rounding level: parity
// with the oracle is by tolerance (tests: 1e-9 relative).  Emission counts follow exactly
// from sum_i xi(i,j) = gamma(j): emit[j] = init[j] + column sum j of trans.
// Per-chunk results are added to 128-bit fixed-point accumulators (64-bit integer atomics
// with carry into a high word: exact, order-independent, so deterministic); a
// one-workgroup finalize converts them to the cpg_counts_f64 stripes.

#include <algorithm>
#include <cmath>

#include "cpg_internal.h"

namespace cpg {
namespace {

constexpr int kET = 1024;               // max lanes per chunk
constexpr int kLanePos = 64;            // positions per lane
constexpr int kSlab = 73;               // trans[64] (by dinucleotide x 4) | init[8] | loglik
// xi bins of one 16-lane replica: [k = from,to pair][d] (64 x u64) padded to 80 so that the
// two replicas an LDS pass serves sit in opposite bank halves (80 * 8 B = 640 B = 160 banks)
#ifndef EST_REP
#define EST_REP 80
#endif
#ifndef EST_KD
#define EST_KD 1
#endif
constexpr int kRep = EST_REP;
#ifndef EST_NREP
#define EST_NREP 8
#endif
constexpr int kNRep = EST_NREP;   // bin replicas per wave (64 / kNRep lanes share one)
// LDS: TA/TB (512 B) | union { 4-step tables, scan buffer, bins } | per-wave partials
constexpr size_t kUnionOff = 32 * 16;
constexpr size_t kUnionBytes =
    (size_t)16 * kNRep * kRep * 8 > 2048 * 16 ? (size_t)16 * kNRep * kRep * 8 : 2048 * 16;
__device__ __forceinline__ int bin_of(int d, int k) { return EST_KD ? k * 16 + d : d * 4 + k; }

struct Mat {
    double a, b, c, d;   // [[a b] [c d]]
    int e;               // value = 2^e * matrix
};

__device__ __forceinline__ void mnorm(Mat& m) {
    const double mx = fmax(fmax(m.a, m.b), fmax(m.c, m.d));
    if (mx > 0.0) {
        const int k = ilogb(mx);
        m.a = ldexp(m.a, -k); m.b = ldexp(m.b, -k); m.c = ldexp(m.c, -k); m.d = ldexp(m.d, -k);
        m.e += k;
    }
}
__device__ __forceinline__ Mat mmul(const Mat& x, const Mat& y) {
    Mat r{x.a * y.a + x.b * y.c, x.a * y.b + x.b * y.d, x.c * y.a + x.d * y.c,
          x.c * y.b + x.d * y.d, x.e + y.e};
    mnorm(r);
    return r;
}
__device__ __forceinline__ Mat mid() { return {1.0, 0.0, 0.0, 1.0, 0}; }

__device__ __forceinline__ void vnorm(double& x, double& y) {
    const double mx = fmax(x, y);
    if (mx > 0.0) {
        const int k = ilogb(mx);
        x = ldexp(x, -k);
        y = ldexp(y, -k);
    }
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
constexpr int kLogFix = 24;   // log-likelihood fixed point: 2^-24 (|chunk loglik| < 2^30)

// 128-bit two's-complement accumulation with 64-bit atomics: the adder that wraps the low
// word carries into the high word (plus the sign extension of a negative addend)
__device__ __forceinline__ void acc128_add(unsigned long long* lohi, unsigned long long v,
                                           bool negative) {
    const unsigned long long old = atomicAdd(lohi, v);
    const unsigned long long hi = (negative ? ~0ull : 0ull) + (old + v < old ? 1ull : 0ull);
    if (hi) atomicAdd(lohi + 1, hi);
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
    // the 16 codes of mini-block m (runtime m: a select chain, no register indexing)
    __device__ __forceinline__ uint64_t mb(int m) const {
        const uint32_t lo = m == 0 ? w[0] : m == 1 ? w[2] : m == 2 ? w[4] : w[6];
        const uint32_t hi = m == 0 ? w[1] : m == 1 ? w[3] : m == 2 ? w[5] : w[7];
        return ((uint64_t)hi << 32) | lo;
    }
};
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

__global__ __launch_bounds__(kET) void k_estep_chunk(const cpg_model model,
                                                     const uint32_t* __restrict__ packed,
                                                     int64_t C,
                                                     unsigned long long* __restrict__ acc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nl = blockDim.x;             // lanes = C / 64
    const int nw = nl / 64;                // waves
    // conflict-free constant tables: 16 x 16 B each = one 256-B bank row
    double2* TA = reinterpret_cast<double2*>(smem);          // (M(+,+), M(+,-))
    double2* TB = TA + 16;                                    // (M(-,+), M(-,-))
    // one union region after TA/TB, used in turn by: the 4-step tables (phase 1), the scan
    // buffer (phase 2), the xi bins (phase 3) — each phase ends with a barrier
    double2* TA4 = TB + 16;                                   // 4-step products, row 0
    double2* TB4 = TA4 + 1024;                                //                  row 1
    Mat* sm = reinterpret_cast<Mat*>(TA4);                    // [nl]
    auto* bins = reinterpret_cast<unsigned long long*>(TA4);  // [wave][kNRep][kRep]
    auto* part = reinterpret_cast<unsigned long long*>(
        smem + kUnionOff + (kUnionBytes > nl * sizeof(Mat) ? kUnionBytes : nl * sizeof(Mat)));
    const int t = threadIdx.x;
    const int lane = t & 63;
    const int64_t c = blockIdx.x;
    const uint32_t* pk = packed + c * (C / 16);
    if (t < 16) {
        const int p = t & 3, b = t >> 2;
        TA[t] = make_double2(model.a[p][b], model.a[p][b + 4]);
        TB[t] = make_double2(model.a[p + 4][b], model.a[p + 4][b + 4]);
    }
    // 4-step products: window (b0..b4) -> M(b0,b1) M(b1,b2) M(b2,b3) M(b3,b4)
    for (int i = t; i < 1024; i += nl) {
        int b[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) b[k] = (i >> (2 * k)) & 3;
        double x00 = 1.0, x01 = 0.0, x10 = 0.0, x11 = 1.0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int p = b[k], q = b[k + 1];
            const double m00 = model.a[p][q], m01 = model.a[p][q + 4],
                         m10 = model.a[p + 4][q], m11 = model.a[p + 4][q + 4];
            const double n00 = x00 * m00 + x01 * m10, n01 = x00 * m01 + x01 * m11;
            const double n10 = x10 * m00 + x11 * m10, n11 = x10 * m01 + x11 * m11;
            x00 = n00; x01 = n01; x10 = n10; x11 = n11;
        }
        TA4[i] = make_double2(x00, x01);
        TB4[i] = make_double2(x10, x11);
    }
    const Codes cd = lane_codes(pk, t);
    __syncthreads();

    constexpr int L = kLanePos;            // 64 positions per lane
    constexpr int kMB = 16, NMB = L / kMB;
    const int p0 = t * L;
    // 1. lane product of M_p over its positions, four matrices per lookup (position 0
    //    carries no matrix: lane 0's first group is M_1 M_2 M_3)
    Mat P = mid();
    Mat Pm[NMB - 1];   // products after mini-blocks 0 .. NMB-2: the alpha checkpoints
#pragma unroll
    for (int gq = 0; gq < L / 4; ++gq) {
        double2 ra, rb;
        if (t == 0 && gq == 0) {
            double x00 = 1.0, x01 = 0.0, x10 = 0.0, x11 = 1.0;
            const uint64_t cm = cd.mb(0);
#pragma unroll
            for (int i = 1; i < 4; ++i) {
                const uint32_t d = code_at(cm, i);
                const double2 ma = TA[d], mb = TB[d];
                const double n00 = x00 * ma.x + x01 * mb.x, n01 = x00 * ma.y + x01 * mb.y;
                const double n10 = x10 * ma.x + x11 * mb.x, n11 = x10 * ma.y + x11 * mb.y;
                x00 = n00; x01 = n01; x10 = n10; x11 = n11;
            }
            ra = make_double2(x00, x01);
            rb = make_double2(x10, x11);
        } else {
            const uint32_t wi = cd.win(gq);
            ra = TA4[wi];
            rb = TB4[wi];
        }
        Mat r{P.a * ra.x + P.b * rb.x, P.a * ra.y + P.b * rb.y, P.c * ra.x + P.d * rb.x,
              P.c * ra.y + P.d * rb.y, P.e};
        P = r;
        if ((gq & 1) == 1) mnorm(P);
        if ((gq & 3) == 3 && gq / 4 < NMB - 1) Pm[gq / 4] = P;
    }
    __syncthreads();   // the 4-step tables are dead from here: the scan buffer reuses them
    // 2a. inclusive prefix (Hillis-Steele)
    sm[t] = P;
    __syncthreads();
    for (int off = 1; off < nl; off <<= 1) {
        Mat x = sm[t];
        if (t >= off) x = mmul(sm[t - off], x);
        __syncthreads();
        sm[t] = x;
        __syncthreads();
    }
    const uint32_t o0 = pk[0] & 3u;
    const double fa = model.pi[o0], fb = model.pi[o0 + 4];   // alpha_0 (b = 1 when live)
    double loglik = 0.0;
    if (t == nl - 1) {
        const Mat A = sm[nl - 1];
        loglik = log(fa * (A.a + A.b) + fb * (A.c + A.d)) + (double)A.e * 0.69314718055994530942;
    }
    double aP, aM;   // alpha at position p0-1 (t > 0); alpha_0 for t == 0
    if (t > 0) {
        const Mat A = sm[t - 1];
        aP = fa * A.a + fb * A.c;
        aM = fa * A.b + fb * A.d;
    } else {
        aP = fa;
        aM = fb;
    }
    vnorm(aP, aM);
    double fcP[NMB], fcM[NMB];   // the alpha checkpoints (see 3a)
    fcP[0] = aP;
    fcM[0] = aM;
#pragma unroll
    for (int m = 1; m < NMB; ++m) {
        const Mat& A = Pm[m - 1];
        fcP[m] = aP * A.a + aM * A.c;
        fcM[m] = aP * A.b + aM * A.d;
        vnorm(fcP[m], fcM[m]);
    }
    __syncthreads();
    // 2b. inclusive suffix
    sm[t] = P;
    __syncthreads();
    for (int off = 1; off < nl; off <<= 1) {
        Mat x = sm[t];
        if (t + off < nl) x = mmul(x, sm[t + off]);
        __syncthreads();
        sm[t] = x;
        __syncthreads();
    }
    double bP = 1.0, bM = 1.0;   // beta at the lane's last position
    if (t + 1 < nl) {
        const Mat B = sm[t + 1];
        bP = B.a + B.b;
        bM = B.c + B.d;
    }
    vnorm(bP, bM);
    __syncthreads();

    // 3a. bins (aliasing the scan buffer, read above) zeroed; alpha entering mini-block m
    //     = alpha entering the lane times phase 1's product of the first m mini-blocks
    //     (any per-position scale cancels in the normalised xi)
    for (int i = t; i < nw * kNRep * kRep; i += nl) bins[i] = 0ull;
    __syncthreads();
    // 3b. mini-blocks, last to first: forward alphas in registers from the checkpoint, then
    //     backward with xi accumulation; beta flows on from one mini-block to the previous
    unsigned long long* wb = bins + ((t >> 6) * kNRep + lane / (64 / kNRep)) * kRep;
    double g0P = 0.0, g0M = 0.0;
    double yP = bP, yM = bM;   // beta at the last position of the mini-block
#pragma unroll 1
    for (int m = NMB - 1; m >= 0; --m) {
        const uint64_t cm = cd.mb(m);
        // alpha at the position before the mini-block (select chain: no register indexing)
        double bfP = fcP[0], bfM = fcM[0];
#pragma unroll
        for (int k = 1; k < NMB; ++k) {
            bfP = m == k ? fcP[k] : bfP;
            bfM = m == k ? fcM[k] : bfM;
        }
        double alP[kMB], alM[kMB];
        double xP = bfP, xM = bfM;
#pragma unroll
        for (int i = 0; i < kMB; ++i) {
            if (t == 0 && m == 0 && i == 0) {   // alpha_0 itself
                alP[i] = xP;
                alM[i] = xM;
                continue;
            }
            const uint32_t d = code_at(cm, i);
            const double2 ma = TA[d], mb = TB[d];
            const double nP = xP * ma.x + xM * mb.x, nM = xP * ma.y + xM * mb.y;
            xP = nP;
            xM = nM;
            if ((i & 3) == 3) vnorm(xP, xM);
            alP[i] = xP;
            alM[i] = xM;
        }
#pragma unroll
        for (int i = kMB - 1; i >= 0; --i) {
            if (t == 0 && m == 0 && i == 0) {   // gamma_0 -> init counts
                const double gp = alP[0] * yP, gm = alM[0] * yM, z = gp + gm;
                g0P = gp / z;
                g0M = gm / z;
                continue;
            }
            const double uP = i > 0 ? alP[i - 1] : bfP;
            const double uM = i > 0 ? alM[i - 1] : bfM;
            const uint32_t d = code_at(cm, i);
            const double2 ma = TA[d], mb = TB[d];
            const double x00 = uP * ma.x * yP, x01 = uP * ma.y * yM, x10 = uM * mb.x * yP,
                         x11 = uM * mb.y * yM;
            const double rz = rcp_nr((x00 + x01) + (x10 + x11)) * kFix;   // exact scaling
            atomicAdd(wb + bin_of(d, 0), to_fixed_scaled(x00 * rz));
            atomicAdd(wb + bin_of(d, 1), to_fixed_scaled(x01 * rz));
            atomicAdd(wb + bin_of(d, 2), to_fixed_scaled(x10 * rz));
            atomicAdd(wb + bin_of(d, 3), to_fixed_scaled(x11 * rz));
            const double nP = ma.x * yP + ma.y * yM, nM = mb.x * yP + mb.y * yM;
            yP = nP;
            yM = nM;
            if ((i & 3) == 0) vnorm(yP, yM);
        }
    }
    __syncthreads();
    // chunk totals of the nw * kNRep replicas: wave q sums replicas q, q + nw, ... of every
    // bin (integer sums: exact in any order), then 64 lanes add the nw partials
    {
        const int q = t >> 6, b = bin_of(lane >> 2, lane & 3);   // lane = slab row d*4+k
        unsigned long long s = 0;
        for (int r = q; r < nw * kNRep; r += nw) s += bins[r * kRep + b];
        part[q * 64 + lane] = s;
    }
    __syncthreads();
    // chunk results -> the global 128-bit accumulators: xi bins and the init posteriors in
    // 2^-47 units, the log-likelihood in signed 2^-24 units
    if (t < 64) {   // row t = d * 4 + k
        unsigned long long s = 0;
        for (int q = 0; q < nw; ++q) s += part[q * 64 + t];
        acc128_add(acc + 2 * t, s, false);
    }
    if (t == 0) {
        acc128_add(acc + 2 * (64 + o0), to_fixed_scaled(g0P * kFix), false);
        acc128_add(acc + 2 * (64 + o0 + 4), to_fixed_scaled(g0M * kFix), false);
    }
    if (t == nl - 1) {
        const long long L = llrint(ldexp(loglik, kLogFix));
        acc128_add(acc + 2 * 72, (unsigned long long)L, L < 0);
    }
}

__device__ void final_estep(const double* v, int t, double* __restrict__ out);

// One workgroup: the 73 accumulators -> doubles (re-zeroed for the next call), then the
// cpg_counts_f64 assembly.
__global__ __launch_bounds__(256) void k_estep_final(unsigned long long* __restrict__ acc,
                                                     double* __restrict__ out) {
    __shared__ double vsum[kSlab];
    const int t = threadIdx.x;
    if (t < kSlab) {
        unsigned long long lo = acc[2 * t], hi = acc[2 * t + 1];
        const bool neg = (long long)hi < 0;   // only the log-likelihood row can be negative
        if (neg) {                             // magnitude first: no cancellation
            lo = ~lo + 1ull;
            hi = ~hi + (lo == 0ull ? 1ull : 0ull);
        }
        const double mag = (double)hi * 18446744073709551616.0 + (double)lo;
        vsum[t] = t < 72 ? mag * (1.0 / kFix) : ldexp(neg ? -mag : mag, -kLogFix);
    }
    __syncthreads();
    if (t < 2 * kSlab) acc[t] = 0ull;
    if (t < 105) final_estep(vsum, t, out);
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

size_t estep_ws_bytes(int64_t, int64_t) { return (size_t)2 * kSlab * 8; }

hipError_t launch_estep(const cpg_model& model, const uint32_t* packed, int64_t nchunks,
                        int64_t C, unsigned long long* acc, double* out, hipStream_t s) {
    if (C % 4096 || C > (int64_t)kET * kLanePos) return hipErrorInvalidValue;
    if (nchunks == 0) return hipMemsetAsync(out, 0, 105 * sizeof(double), s);
    const int lanes = (int)(C / kLanePos);
    // the union is sized for 16 waves; a smaller chunk (fewer lanes) uses a prefix of it
    const size_t uni = std::max(kUnionBytes, (size_t)lanes * sizeof(Mat));
    const size_t lds = kUnionOff + uni + 16 * 64 * sizeof(unsigned long long);
    hipLaunchKernelGGL(k_estep_chunk, dim3((unsigned)nchunks), dim3(lanes), lds, s, model,
                       packed, C, acc);
    hipLaunchKernelGGL(k_estep_final, dim3(1), dim3(256), 0, s, acc, out);
    return hipGetLastError();
}

}  // namespace cpg
