// ubench_bits.hip — gfx950 issue cost of the labelled-count kernel's integer instruction mix
// (v_bcnt_u32_b32, v_bitop3_b32, v_add_u32, v_alignbit_b32, v_mov_b32_dpp wave_shr), measured
// with clock64 inside one workgroup: NC independent chains per lane, W waves per SIMD.
// Dev tool: the count-kernel design numbers in DESIGN.md §4.1 come from it.
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_bits.hip -o build/ubench_bits
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int kIter = 512;
constexpr int NC = 8;

template <int OP>
__global__ void k_op(unsigned* out, long long* cyc, unsigned a, unsigned b) {
    unsigned x[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) x[c] = threadIdx.x * 2654435761u + c;
    __syncthreads();
    const long long t0 = clock64();
    for (int i = 0; i < kIter; ++i) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const unsigned y = x[(c + 1) % NC], z = x[(c + 2) % NC];
            if (OP == 0) x[c] = x[c] + y;                                   // v_add_u32
            if (OP == 1) x[c] = __popc(x[c]) + x[c];                        // v_bcnt_u32_b32
            if (OP == 2) asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x80" : "=v"(x[c]) : "v"(x[c]), "v"(y), "v"(z));
            if (OP == 3) x[c] = __builtin_amdgcn_alignbit(x[c], y, 30);
            if (OP == 4) x[c] = (unsigned)__builtin_amdgcn_update_dpp((int)x[c], (int)x[c], 0x138, 0xF, 0xF, false) + a;
            if (OP == 5) x[c] = __popc(x[c] & y) + x[c];                    // and + bcnt
            if (OP == 6) x[c] = x[c] & y;                                   // v_and_b32
            if (OP == 7) asm volatile("v_bfi_b32 %0, %1, %2, %3" : "=v"(x[c]) : "v"(x[c]), "v"(y), "v"(z));
            if (OP == 8) x[c] = (x[c] << 1) | y;                            // v_lshl_or_b32
            if (OP >= 9) {   // 64-bit ops on (x[c], y) pairs: the K5 step's candidates
                const unsigned long long a = ((unsigned long long)y << 32) | x[c];
                const unsigned long long b = ((unsigned long long)z << 32) | x[(c + 3) % NC];
                unsigned long long r;
                if (OP == 9) r = a + b;                                          // v_lshl_add_u64
                if (OP == 10) r = (long long)a > (long long)b ? a : b;            // cmp_i64 + 2 cndmask
                if (OP == 11) {                                                   // v_add_f64
                    const double d = __longlong_as_double((long long)a) + __longlong_as_double((long long)b);
                    r = (unsigned long long)__double_as_longlong(d);
                }
                if (OP == 12) {                                                   // v_max_f64
                    const double d = fmax(__longlong_as_double((long long)a), __longlong_as_double((long long)b));
                    r = (unsigned long long)__double_as_longlong(d);
                }
                if (OP == 13) r = a + (__longlong_as_double((long long)a) > __longlong_as_double((long long)b) ? 1 : 0);   // v_cmp_gt_f64 (+ addc)
                x[c] = (unsigned)r ^ (unsigned)(r >> 32);
            }
        }
    }
    __syncthreads();
    const long long t1 = clock64();
    unsigned s = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) s ^= x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int OP>
void run(const char* name, int threads) {
    unsigned* out;
    long long* cyc;
    CHECK(hipMalloc(&out, 4 * 1024 * sizeof(unsigned)));
    CHECK(hipMalloc(&cyc, 4 * sizeof(long long)));
    long long best = 1ll << 60;
    for (int rep = 0; rep < 5; ++rep) {
        hipLaunchKernelGGL(k_op<OP>, dim3(1), dim3(threads), 0, 0, out, cyc, 12345u, 678u);
        CHECK(hipDeviceSynchronize());
        long long c;
        CHECK(hipMemcpy(&c, cyc, sizeof c, hipMemcpyDeviceToHost));
        best = std::min(best, c);
    }
    const int waves_per_simd = threads / 256 > 0 ? threads / 256 : 1;
    // cycles per wave-instruction issued on one SIMD (all its waves' chains together)
    const double per = (double)best / ((double)kIter * NC * waves_per_simd);
    printf("%-8s waves/SIMD %d: %.2f cycles per wave-instruction per SIMD (%.2f per wave)\n", name,
           waves_per_simd, per, (double)best / ((double)kIter * NC));
    CHECK(hipFree(out));
    CHECK(hipFree(cyc));
}

int main() {
    for (int th : {256, 1024}) {
        run<0>("add", th);
        run<1>("bcnt", th);
        run<2>("bitop3", th);
        run<3>("alignbit", th);
        run<4>("dpp+add", th);
        run<5>("and+bcnt", th);
        run<6>("and", th);
        run<7>("bfi", th);
        run<8>("lshl_or", th);
        run<9>("add_u64", th);
        run<10>("max_i64", th);
        run<11>("add_f64", th);
        run<12>("max_f64", th);
        run<13>("cmp_f64", th);
    }
    return 0;
}
