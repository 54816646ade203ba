// Development microbenchmark: the K4 serial walk (reference step, constants staged in LDS and
// read kAhead steps ahead) in lane 0 of a 256-lane workgroup, against the same chain with
// the constants in registers.  Ticks of clock64 (2.4 GHz) per step.
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr int kN = 512;
struct Step { double P, M; };
__device__ __forceinline__ Step ref_step(double P, double M, double l0, double l1, double l2, double l3) {
    return {fmax(P + l0, M + l1), fmax(P + l2, M + l3)};
}
template <int kMode>   // 0: LDS + write per step, 1: LDS no write, 2: registers, 3: LDS, no sched barrier
__global__ __launch_bounds__(256) void walk(const double4* L, int n, long long* ticks, double* out) {
    __shared__ double4 st[kN + 8];
    __shared__ double2 vs[kN + 8];
    for (int i = threadIdx.x; i < kN + 8; i += 256) st[i] = L[i & 15];
    __syncthreads();
    if (threadIdx.x == 0) {
        double P = -1.0, M = -2.0;
        const long long t0 = clock64();
        if (kMode == 2) {
            double4 r[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) r[j] = L[j];
            for (int s0 = 0; s0 < n; s0 += 16) {
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const Step s = ref_step(P, M, r[j].x, r[j].y, r[j].z, r[j].w);
                    P = s.P; M = s.M;
                }
            }
        } else {
            double4 X[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) X[j] = st[j];
            for (int s0 = 0; s0 < n; s0 += 4) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const Step s = ref_step(P, M, X[j].x, X[j].y, X[j].z, X[j].w);
                    P = s.P; M = s.M;
                    X[j] = st[s0 + 4 + j];
                    if (kMode == 0) vs[s0 + j] = make_double2(P, M);
                    if (kMode != 3) __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
        const long long t1 = clock64();
        ticks[kMode] = t1 - t0;
        out[kMode] = P + M + (kMode == 0 ? vs[n / 2].x : 0.0);
    }
}
int main() {
    double4 h[16];
    for (int i = 0; i < 16; ++i) h[i] = make_double4(-0.5 - 0.1 * i, -7.3 - 0.01 * i, -4.6, -1.2 - 0.05 * i);
    double4* L; long long* t; double* o;
    (void)hipMalloc(&L, sizeof h); (void)hipMalloc(&t, 64); (void)hipMalloc(&o, 64);
    (void)hipMemcpy(L, h, sizeof h, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 3; ++rep) {
        walk<0><<<1, 256>>>(L, kN, t, o);
        walk<1><<<1, 256>>>(L, kN, t, o);
        walk<2><<<1, 256>>>(L, kN, t, o);
        walk<3><<<1, 256>>>(L, kN, t, o);
        long long ht[4];
        (void)hipMemcpy(ht, t, sizeof ht, hipMemcpyDeviceToHost);
        printf("{\"lds_write\": %.1f, \"lds\": %.1f, \"regs\": %.1f, \"lds_nosb\": %.1f}\n",
               ht[0] / (double)kN, ht[1] / (double)kN, ht[2] / (double)kN, ht[3] / (double)kN);
    }
    return 0;
}
