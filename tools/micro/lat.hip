// Dependent-chain latency of fp64 / fp32 / int VALU ops on gfx950, and throughput with
// several independent chains (dev microbenchmark: s_memtime around N dependent ops, one wave
// per SIMD or W waves per CU).  Build: hipcc --offload-arch=gfx950 -O3 lat.hip -o lat
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CH>
__global__ void k_f64(double* out, long long* cyc, int n, double a, double b) {
    double x[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = threadIdx.x * 1e-3 + c;
    const long long t0 = clock64();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int c = 0; c < CH; ++c) x[c] = fma(x[c], a, b);
    }
    const long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
template <int CH>
__global__ void k_f32(float* out, long long* cyc, int n, float a, float b) {
    float x[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) x[c] = threadIdx.x * 1e-3f + c;
    const long long t0 = clock64();
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int c = 0; c < CH; ++c) x[c] = fmaf(x[c], a, b);
    }
    const long long t1 = clock64();
    float s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class F>
void run(const char* name, F launch, int blocks, int threads, int n, int ops_per_iter) {
    long long* cyc;
    (void)hipMalloc(&cyc, blocks * sizeof(long long));
    launch(cyc, blocks, threads, n);   // warm
    (void)hipDeviceSynchronize();
    launch(cyc, blocks, threads, n);
    (void)hipDeviceSynchronize();
    long long h[1024];
    (void)hipMemcpy(h, cyc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < blocks; ++i) avg += h[i];
    avg /= blocks;
    printf("%-34s blocks %4d threads %4d: %.2f cycles per dependent step, %.2f per op (per wave)\n",
           name, blocks, threads, avg / n, avg / n / ops_per_iter);
    (void)hipFree(cyc);
}

int main() {
    double* od;
    float* of;
    (void)hipMalloc(&od, 1 << 24);
    (void)hipMalloc(&of, 1 << 24);
    const int n = 4096;
    for (int threads : {64, 256, 1024}) {
        run("f64 fma, 1 chain", [&](long long* c, int b, int t, int n) {
            hipLaunchKernelGGL(k_f64<1>, dim3(b), dim3(t), 0, 0, od, c, n, 0.999999, 1e-9); }, 256, threads, n, 1);
        run("f64 fma, 2 chains", [&](long long* c, int b, int t, int n) {
            hipLaunchKernelGGL(k_f64<2>, dim3(b), dim3(t), 0, 0, od, c, n, 0.999999, 1e-9); }, 256, threads, n, 2);
        run("f64 fma, 4 chains", [&](long long* c, int b, int t, int n) {
            hipLaunchKernelGGL(k_f64<4>, dim3(b), dim3(t), 0, 0, od, c, n, 0.999999, 1e-9); }, 256, threads, n, 4);
        run("f64 fma, 8 chains", [&](long long* c, int b, int t, int n) {
            hipLaunchKernelGGL(k_f64<8>, dim3(b), dim3(t), 0, 0, od, c, n, 0.999999, 1e-9); }, 256, threads, n, 8);
        run("f32 fma, 1 chain", [&](long long* c, int b, int t, int n) {
            hipLaunchKernelGGL(k_f32<1>, dim3(b), dim3(t), 0, 0, of, c, n, 0.999999f, 1e-9f); }, 256, threads, n, 1);
        run("f32 fma, 4 chains", [&](long long* c, int b, int t, int n) {
            hipLaunchKernelGGL(k_f32<4>, dim3(b), dim3(t), 0, 0, of, c, n, 0.999999f, 1e-9f); }, 256, threads, n, 4);
    }
    return 0;
}
