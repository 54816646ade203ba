// ubench_fp64.hip — gfx950 issue cost and dependent latency of the E-step's instruction mix
// (fp64 fma/mul/ldexp, integer LDS atomics, ds_read_b128), measured with s_memtime inside one
// workgroup.  Dev tool: the E-step design numbers in DESIGN.md §4.4 come from it.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int kIter = 256;

// NC independent fma chains per lane, kIter steps each
template <int NC>
__global__ void k_fma(double* out, long long* cyc, double a, double b) {
    double x[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) x[c] = threadIdx.x * 1e-3 + c;
    __syncthreads();
    const long long t0 = clock64();
    for (int i = 0; i < kIter; ++i) {
#pragma unroll
        for (int c = 0; c < NC; ++c) x[c] = fma(x[c], a, b);
    }
    __syncthreads();
    const long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NC>
__global__ void k_mul(double* out, long long* cyc, double a, double b) {
    double x[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) x[c] = threadIdx.x * 1e-3 + c;
    __syncthreads();
    const long long t0 = clock64();
    for (int i = 0; i < kIter; ++i) {
#pragma unroll
        for (int c = 0; c < NC; ++c) x[c] = x[c] * a;
    }
    __syncthreads();
    const long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + b;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// integer add chains (v_add_u32)
template <int NC>
__global__ void k_iadd(double* out, long long* cyc, double a, double b) {
    unsigned x[NC];
    const unsigned k = (unsigned)a;
#pragma unroll
    for (int c = 0; c < NC; ++c) x[c] = threadIdx.x + c;
    __syncthreads();
    const long long t0 = clock64();
    for (int i = 0; i < kIter; ++i) {
#pragma unroll
        for (int c = 0; c < NC; ++c) { x[c] = (x[c] ^ k) + (x[c] >> 3); }
    }
    __syncthreads();
    const long long t1 = clock64();
    unsigned s = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) s += x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + b;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// LDS u64 atomics, no return: 16 columns per row (the E-step bin layout), NA per iteration
template <int NA>
__global__ void k_atom(double* out, long long* cyc, double a, double b) {
    __shared__ unsigned long long bins[64 * 16];
    for (int i = threadIdx.x; i < 64 * 16; i += blockDim.x) bins[i] = 0;
    __syncthreads();
    unsigned long long* wb = bins + (threadIdx.x & 15);
    unsigned d = threadIdx.x * 2654435761u;
    const long long t0 = clock64();
    for (int i = 0; i < kIter; ++i) {
        d = d * 1664525u + 1013904223u;
        const unsigned r = (d >> 28) & 15u;
#pragma unroll
        for (int c = 0; c < NA; ++c) atomicAdd(wb + (c * 16 + r) * 16, (unsigned long long)(i + c));
    }
    __syncthreads();
    const long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = (double)bins[threadIdx.x & 1023] + a + b;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// dependent ds_read_b128 chain (address from the loaded value): latency
__global__ void k_ldsdep(double* out, long long* cyc, double a, double b) {
    __shared__ double2 tab[1024];
    for (int i = threadIdx.x; i < 1024; i += blockDim.x)
        tab[i] = make_double2((double)((i * 37 + 11) & 1023), 1.0);
    __syncthreads();
    int idx = threadIdx.x & 1023;
    const long long t0 = clock64();
    for (int i = 0; i < kIter; ++i) {
        const double2 v = tab[idx];
        idx = (int)v.x;
    }
    __syncthreads();
    const long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = idx + a + b;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// ldexp + frexp chain (the vnorm pattern)
__global__ void k_vnorm(double* out, long long* cyc, double a, double b) {
    double x = 1.0 + threadIdx.x * 1e-3, y = 0.5;
    __syncthreads();
    const long long t0 = clock64();
    for (int i = 0; i < kIter; ++i) {
        x = x * a; y = y * b;
        const double mx = fmax(x, y);
        const int k = __builtin_amdgcn_frexp_exp(mx) - 1;
        const int kk = mx > 0.0 ? k : 0;
        x = ldexp(x, -kk);
        y = ldexp(y, -kk);
    }
    __syncthreads();
    const long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x + y;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

typedef void (*KF)(double*, long long*, double, double);

static void run(const char* name, KF k, int threads, int ops_per_iter_per_lane) {
    double* d_out; long long* d_cyc;
    const int blocks = 256;
    CHECK(hipMalloc(&d_out, sizeof(double) * blocks * threads));
    CHECK(hipMalloc(&d_cyc, sizeof(long long) * blocks));
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, d_out, d_cyc, 1.0000001, 0.999);
    CHECK(hipDeviceSynchronize());
    std::vector<long long> c(blocks);
    CHECK(hipMemcpy(c.data(), d_cyc, sizeof(long long) * blocks, hipMemcpyDeviceToHost));
    std::vector<long long> s(c);
    std::sort(s.begin(), s.end());
    const double med = (double)s[blocks / 2];
    const int waves = threads / 64;
    const double per_wave_instr = (double)kIter * ops_per_iter_per_lane;
    // cycles per instruction per wave, and per SIMD (waves spread over 4 SIMDs)
    printf("%-18s threads=%5d waves/SIMD=%5.2f  cyc=%9.0f  cyc/instr(wave)=%7.2f  cyc/instr(SIMD)=%6.2f\n",
           name, threads, waves / 4.0, med, med / per_wave_instr,
           med / (per_wave_instr * (waves < 4 ? 1 : waves / 4.0)));
    CHECK(hipFree(d_out)); CHECK(hipFree(d_cyc));
}

int main() {
    int thr[] = {64, 256, 512, 1024};
    for (int t : thr) {
        run("fma dep x1", k_fma<1>, t, 1);
        run("fma x4", k_fma<4>, t, 4);
        run("fma x8", k_fma<8>, t, 8);
        run("mul x8", k_mul<8>, t, 8);
        run("int(xor+shr+add) x8", k_iadd<8>, t, 8 * 3);
        run("lds atom u64 x4", k_atom<4>, t, 4);
        run("lds read dep", k_ldsdep, t, 1);
        run("vnorm chain", k_vnorm, t, 1);
    }
    return 0;
}
