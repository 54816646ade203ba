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
//      = alpha_{p-1}(i) M_p(i,j) beta_p(j) / Z_p accumulated into per-wave LDS bins.
// Posteriors are normalised per position, so the scaling scheme (exact powers of two here,
// reciprocal of the sum in the reference) changes results only at rounding level: parity
// with the oracle is by tolerance (tests: 1e-9 relative).  Emission counts follow exactly
// from sum_i xi(i,j) = gamma(j): emit[j] = init[j] + column sum j of trans.
// Per-chunk results go to a slab summed in chunk order: deterministic.

#include <algorithm>
#include <cmath>

#include "cpg_internal.h"

namespace cpg {
namespace {

constexpr int kET = 1024;               // max lanes per chunk
constexpr int kLanePos = 64;            // positions per lane
constexpr int kSlab = 73;               // trans[64] (by dinucleotide x 4) | init[8] | loglik

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

__device__ __forceinline__ uint32_t dinuc_lds(const uint32_t* sw, int p) {   // p >= 1
    const uint32_t b = (sw[p >> 4] >> ((p & 15) * 2)) & 3u;
    const int q = p - 1;
    const uint32_t a = (sw[q >> 4] >> ((q & 15) * 2)) & 3u;
    return a | (b << 2);
}

__global__ __launch_bounds__(kET) void k_estep_chunk(const cpg_model model,
                                                     const uint32_t* __restrict__ packed,
                                                     int64_t C, double* __restrict__ slab) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nl = blockDim.x;             // lanes = C / 64
    const int nwords = (int)(C / 16);
    uint32_t* sw = reinterpret_cast<uint32_t*>(smem);                          // C/16 words
    double4* T = reinterpret_cast<double4*>(smem + ((nwords * 4 + 15) & ~15));  // 16
    double* bins = reinterpret_cast<double*>(T + 16);                            // [waves][64]
    Mat* sm = reinterpret_cast<Mat*>(bins + (kET / 64) * 64);                    // [nl]
    const int t = threadIdx.x;
    const int64_t c = blockIdx.x;
    const uint32_t* pk = packed + c * (C / 16);
    for (int i = t; i < nwords; i += nl) sw[i] = pk[i];
    if (t < 16) {
        const int p = t & 3, b = t >> 2;
        T[t] = make_double4(model.a[p][b], model.a[p][b + 4], model.a[p + 4][b],
                            model.a[p + 4][b + 4]);
    }
    for (int i = t; i < (kET / 64) * 64; i += nl) bins[i] = 0.0;
    __syncthreads();

    constexpr int L = kLanePos;            // 64 positions per lane
    constexpr int kMB = 16, NMB = L / kMB;
    const int p0 = t * L;
    // 1. lane product of M_p over its positions (position 0 carries no matrix)
    Mat P = mid();
    for (int p = (t == 0 ? 1 : p0); p < p0 + L; ++p) {
        const double4 m = T[dinuc_lds(sw, p)];
        Mat r{P.a * m.x + P.b * m.z, P.a * m.y + P.b * m.w, P.c * m.x + P.d * m.z,
              P.c * m.y + P.d * m.w, P.e};
        P = r;
        if ((p & 7) == 7) mnorm(P);
    }
    mnorm(P);
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
    const uint32_t o0 = sw[0] & 3u;
    const double fa = model.pi[o0], fb = model.pi[o0 + 4];   // alpha_0 (b = 1 on the live states)
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

    // 3a. backward checkpoints: beta at the last position of each mini-block, kept in LDS
    //     ([m][lane] double2, aliasing the scan buffer: conflict-free 16-B rows)
    __syncthreads();
    double2* ck = reinterpret_cast<double2*>(sm);
    {
        double xP = bP, xM = bM;
        for (int m = NMB - 1; m >= 0; --m) {
            ck[m * nl + t] = make_double2(xP, xM);
            if (m == 0) break;
            for (int p = p0 + m * kMB + kMB - 1; p >= p0 + m * kMB; --p) {
                const double4 mm = T[dinuc_lds(sw, p)];
                const double nP = mm.x * xP + mm.y * xM, nM = mm.z * xP + mm.w * xM;
                xP = nP;
                xM = nM;
                vnorm(xP, xM);
            }
        }
    }
    // 3b. mini-blocks: forward alphas in registers, then backward with xi accumulation
    double* wb = bins + (t >> 6) * 64;
    double g0P = 0.0, g0M = 0.0;
    double bfP = aP, bfM = aM;   // alpha at the position before the mini-block
#pragma unroll
    for (int m = 0; m < NMB; ++m) {
        const int q0 = p0 + m * kMB;
        double alP[kMB], alM[kMB];
        double xP = bfP, xM = bfM;
#pragma unroll
        for (int i = 0; i < kMB; ++i) {
            const int p = q0 + i;
            if (p == 0) {   // alpha_0 itself (lane 0, mini-block 0)
                alP[i] = xP;
                alM[i] = xM;
                continue;
            }
            const double4 mm = T[dinuc_lds(sw, p)];
            const double nP = xP * mm.x + xM * mm.z, nM = xP * mm.y + xM * mm.w;
            xP = nP;
            xM = nM;
            vnorm(xP, xM);
            alP[i] = xP;
            alM[i] = xM;
        }
        const double2 cz = ck[m * nl + t];
        double yP = cz.x, yM = cz.y;
#pragma unroll
        for (int i = kMB - 1; i >= 0; --i) {
            const int p = q0 + i;
            if (p == 0) {   // gamma_0 -> init counts
                const double gp = alP[0] * yP, gm = alM[0] * yM, z = gp + gm;
                g0P = gp / z;
                g0M = gm / z;
                continue;
            }
            const double uP = i > 0 ? alP[i - 1] : bfP;
            const double uM = i > 0 ? alM[i - 1] : bfM;
            const uint32_t d = dinuc_lds(sw, p);
            const double4 mm = T[d];
            const double x00 = uP * mm.x * yP, x01 = uP * mm.y * yM, x10 = uM * mm.z * yP,
                         x11 = uM * mm.w * yM;
            const double rz = 1.0 / ((x00 + x01) + (x10 + x11));
            double* bq = wb + d * 4;
            atomicAdd(bq + 0, x00 * rz);
            atomicAdd(bq + 1, x01 * rz);
            atomicAdd(bq + 2, x10 * rz);
            atomicAdd(bq + 3, x11 * rz);
            const double nP = mm.x * yP + mm.y * yM, nM = mm.z * yP + mm.w * yM;
            yP = nP;
            yM = nM;
            vnorm(yP, yM);
        }
        bfP = alP[kMB - 1];
        bfM = alM[kMB - 1];
    }
    __syncthreads();
    double* sl = slab + c * kSlab;
    if (t < 64) {
        double s = 0.0;
        for (int w = 0; w < nl / 64; ++w) s += bins[w * 64 + t];
        sl[t] = s;
    }
    if (t == 0) {
        for (int i = 0; i < 8; ++i) sl[64 + i] = 0.0;
        sl[64 + o0] = g0P;
        sl[64 + o0 + 4] = g0M;
    }
    if (t == nl - 1) sl[72] = loglik;
}

__global__ __launch_bounds__(128) void k_estep_final(const double* __restrict__ slab,
                                                     int64_t nchunks, double* __restrict__ out) {
    __shared__ double v[kSlab];
    const int t = threadIdx.x;
    if (t < kSlab) {
        double s = 0.0;
        for (int64_t c = 0; c < nchunks; ++c) s += slab[c * kSlab + t];
        v[t] = s;
    }
    __syncthreads();
    if (t != 0) return;
    // cpg_counts_f64: init[8] trans[8][8] emit[8][4] loglik
    double* init = out;
    double* trans = out + 8;
    double* emit = out + 72;
    for (int i = 0; i < 105; ++i) out[i] = 0.0;
    for (int s = 0; s < 8; ++s) init[s] = v[64 + s];
    for (int d = 0; d < 16; ++d) {
        const int p = d & 3, b = d >> 2;
        trans[p * 8 + b] = v[d * 4 + 0];
        trans[p * 8 + b + 4] = v[d * 4 + 1];
        trans[(p + 4) * 8 + b] = v[d * 4 + 2];
        trans[(p + 4) * 8 + b + 4] = v[d * 4 + 3];
    }
    for (int j = 0; j < 8; ++j) {
        double col = init[j];
        for (int i = 0; i < 8; ++i) col += trans[i * 8 + j];
        emit[j * 4 + (j & 3)] = col;
    }
    out[104] = v[72];
}

}  // namespace

size_t estep_ws_bytes(int64_t nchunks, int64_t) { return (size_t)(nchunks + 1) * kSlab * 8 + 1024; }

hipError_t launch_estep(const cpg_model& model, const uint32_t* packed, int64_t nchunks,
                        int64_t C, void* ws, size_t ws_bytes, double* out, hipStream_t s) {
    if (estep_ws_bytes(nchunks, C) > ws_bytes) return hipErrorInvalidValue;
    if (C % 4096 || C > (int64_t)kET * kLanePos) return hipErrorInvalidValue;
    const int lanes = (int)(C / kLanePos);
    double* slab = static_cast<double*>(ws);
    const size_t lds = (size_t)((C / 16 * 4 + 15) & ~15) + 16 * sizeof(double4) +
                       (kET / 64) * 64 * sizeof(double) +
                       std::max(lanes * sizeof(Mat), (size_t)lanes * (kLanePos / 16) * 16);
    if (nchunks > 0)
        hipLaunchKernelGGL(k_estep_chunk, dim3((unsigned)nchunks), dim3(lanes), lds, s, model,
                           packed, C, slab);
    hipLaunchKernelGGL(k_estep_final, dim3(1), dim3(128), 0, s, slab, nchunks, out);
    return hipGetLastError();
}

}  // namespace cpg
