// loadshape.hip — measurement tool (not product): the read rate of candidate LOAD SHAPES for the
// labelled-count kernel (k_count.hip) over its two streams — the packed bases (16 B per 64-base
// block) and the label bits (8 B per block) — with the counting replaced by an XOR, so that the
// shape's own ceiling is known before the counting is built on it.
//   shape 0  one block per lane per round: 16-B packed + 8-B label load (k_count.hip today),
//            grid-stride rounds of 64 blocks per wave
//   shape 1  two blocks per lane per round: packed of blocks g+l and g+64+l (two coalesced
//            1-KiB loads per wave), labels of blocks g+2l, g+2l+1 (one coalesced 16-B load),
//            grid-stride rounds of 128 blocks per wave
//   shape 2  shape 1's loads, each wave streaming one contiguous range of rounds
// kDepth rounds of loads are issued before any is consumed.  Occupancy is set by the dynamic
// LDS a workgroup asks for (0: as many as the registers allow).
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/loadshape.hip -o tools/libloadshape.so
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int kShape, int kDepth>
__global__ __launch_bounds__(256) void k_loadshape(const uint4* __restrict__ packed4,
                                                   const uint2* __restrict__ sign2,
                                                   const uint4* __restrict__ sign4, int64_t nblk,
                                                   uint32_t* __restrict__ out) {
    extern __shared__ uint32_t pad[];
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    uint32_t acc = 0;
    if (kShape == 0) {
        const int64_t stride = nwaves * 64;
        for (int64_t g = wave * 64; g < nblk; g += kDepth * stride) {
            uint4 w[kDepth];
            uint2 s[kDepth];
#pragma unroll
            for (int r = 0; r < kDepth; ++r) {
                const int64_t b = g + r * stride + lane;
                const int64_t bb = b < nblk ? b : nblk - 1;
                w[r] = packed4[bb];
                s[r] = sign2[bb];
            }
#pragma unroll
            for (int r = 0; r < kDepth; ++r) acc ^= w[r].x ^ w[r].y ^ w[r].z ^ w[r].w ^ s[r].x ^ s[r].y;
        }
    } else {
        const int64_t nround = nblk / 128;   // whole 128-block rounds (the tool sizes nblk so)
        int64_t r0, r1, rstep;
        if (kShape == 1) {
            r0 = wave; r1 = nround; rstep = nwaves;
        } else {
            const int64_t per = (nround + nwaves - 1) / nwaves;
            r0 = wave * per; r1 = r0 + per < nround ? r0 + per : nround; rstep = 1;
        }
        for (int64_t r = r0; r < r1; r += kDepth * rstep) {
            uint4 a[kDepth], b[kDepth], s[kDepth];
#pragma unroll
            for (int d = 0; d < kDepth; ++d) {
                int64_t rr = r + d * rstep;
                rr = rr < r1 ? rr : r1 - 1;
                a[d] = packed4[rr * 128 + lane];
                b[d] = packed4[rr * 128 + 64 + lane];
                s[d] = sign4[rr * 64 + lane];
            }
#pragma unroll
            for (int d = 0; d < kDepth; ++d)
                acc ^= a[d].x ^ a[d].y ^ a[d].z ^ a[d].w ^ b[d].x ^ b[d].y ^ b[d].z ^ b[d].w ^
                       s[d].x ^ s[d].y ^ s[d].z ^ s[d].w;
        }
    }
    if (acc == 0x9E3779B9u) out[0] = acc + pad[0];   // keeps the loads; practically never stores
}

template <int kShape>
static void launch_shape(int depth, dim3 grid, size_t lds, hipStream_t s, const uint4* p,
                         const uint2* s2, const uint4* s4, int64_t nblk, uint32_t* out) {
    switch (depth) {
    case 1: hipLaunchKernelGGL((k_loadshape<kShape, 1>), grid, dim3(256), lds, s, p, s2, s4, nblk, out); break;
    case 2: hipLaunchKernelGGL((k_loadshape<kShape, 2>), grid, dim3(256), lds, s, p, s2, s4, nblk, out); break;
    case 4: hipLaunchKernelGGL((k_loadshape<kShape, 4>), grid, dim3(256), lds, s, p, s2, s4, nblk, out); break;
    default: hipLaunchKernelGGL((k_loadshape<kShape, 8>), grid, dim3(256), lds, s, p, s2, s4, nblk, out); break;
    }
}

extern "C" int loadshape(const void* packed, const void* sign, int64_t nblk, void* out, int shape,
                         int depth, int grid, int lds_bytes, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    const uint4* p = (const uint4*)packed;
    const uint2* s2 = (const uint2*)sign;
    const uint4* s4 = (const uint4*)sign;
    uint32_t* o = (uint32_t*)out;
    if (shape == 0) launch_shape<0>(depth, dim3(grid), lds_bytes, s, p, s2, s4, nblk, o);
    else if (shape == 1) launch_shape<1>(depth, dim3(grid), lds_bytes, s, p, s2, s4, nblk, o);
    else launch_shape<2>(depth, dim3(grid), lds_bytes, s, p, s2, s4, nblk, o);
    return (int)hipGetLastError();
}
