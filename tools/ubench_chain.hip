// Development microbenchmark: latency of the K4 serial step (two fp64 adds into a max, per
// state) in one lane, and the tick rates of clock64 (s_memtime) and wall_clock64.
#include <hip/hip_runtime.h>
#include <cstdio>
struct Out { long long t0, t1, w0, w1; double P, M; };
template <int kMode>
__global__ void chain(const double* L, int n, Out* o) {
    if (threadIdx.x != 0) return;
    double l[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) l[i] = L[i];
    double P = -1.0, M = -2.0;
    const long long w0 = wall_clock64(), t0 = clock64();
    for (int s = 0; s < n; s += 4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (kMode == 0) {   // the reference step: adds into max
                const double a = P + l[4 * j], b = M + l[4 * j + 1], c = P + l[4 * j + 2], d = M + l[4 * j + 3];
                P = fmax(a, b);
                M = fmax(c, d);
            } else if (kMode == 1) {   // add chain only
                P = P + l[4 * j];
                M = M + l[4 * j + 3];
            } else {   // max chain only
                P = fmax(P, l[4 * j]);
                M = fmax(M, l[4 * j + 3]);
            }
        }
    }
    const long long t1 = clock64(), w1 = wall_clock64();
    o->t0 = t0; o->t1 = t1; o->w0 = w0; o->w1 = w1; o->P = P; o->M = M;
}
int main() {
    double h[16];
    for (int i = 0; i < 16; ++i) h[i] = -0.5 - 0.37 * i;
    double* L; Out* o; hipMalloc(&L, sizeof h); hipMalloc(&o, sizeof(Out));
    hipMemcpy(L, h, sizeof h, hipMemcpyHostToDevice);
    int rate = 0; hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0);
    for (int mode = 0; mode < 3; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
            const int n = 1 << 16;
            if (mode == 0) chain<0><<<1, 64>>>(L, n, o);
            if (mode == 1) chain<1><<<1, 64>>>(L, n, o);
            if (mode == 2) chain<2><<<1, 64>>>(L, n, o);
            Out r; hipMemcpy(&r, o, sizeof r, hipMemcpyDeviceToHost);
            const double ns = (r.w1 - r.w0) * 1e6 / rate;
            printf("{\"mode\": %d, \"steps\": %d, \"clock64_per_step\": %.2f, \"ns_per_step\": %.3f, \"clock64_GHz\": %.3f, \"wall_kHz\": %d}\n",
                   mode, n, double(r.t1 - r.t0) / n, ns / n, (r.t1 - r.t0) / ns, rate);
        }
    }
    return 0;
}
