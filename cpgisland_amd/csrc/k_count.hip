// k_count.hip — labelled int64 counts on gfx950.
//
// Training-side counterpart of the BW mapper stripes (init / transition / emission rows,
// CpGIslandFinder.java:200) computed from hard labels: state s_t = base_t + (sign_t?0:4).
// Streams 2-bit packed bases (16 B per lane = 64 bases) and sign bits (8 B per lane) in
// grid-stride batches, the next batch's loads in flight while a batch is counted, and counts
// with v_bcnt over the bases' bit-planes (count_dev.h; shared with the fused training pass in
// k_estep.hip).
//
// Per-workgroup partial counts (and the init states of the chunks starting in the
// workgroup) are added to 72 global 64-bit accumulators (integer atomics: exact and
// order-independent, one per counter per workgroup); the last workgroup to finish derives the
// emission/dinucleotide/mono counts from the transition + init counts (exact integer
// identities) and re-zeroes the accumulators.  One launch per call (a separate one-workgroup
// finalize launch for the streamed genome, which accumulates every window first).

#include <type_traits>

#include "count_dev.h"

namespace cpg {
namespace {

using cnt::kRaw;
constexpr int kCountThreads = 256;
constexpr int kCntRep = cnt::kRep;
// blocks per lane per batch, and the grid cap: 4 waves per SIMD (<= 128 VGPRs) hold 1,024
// workgroups of 4 waves at once; every lane has two batches in flight (the one being counted
// and the next one's loads)
constexpr int kBatch = 1;
constexpr int kCntGrid = 2048;
constexpr int kCntWavesPerEU = 4;

// the value of `v` in the lane below (wave_shr:1 DPP); lane 0 takes `old`
__device__ __forceinline__ uint32_t from_lane_below(uint32_t v, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}

// One batch of a wave: block g + lane + r * stride of each lane, r < kBatch (the wave's 64
// lanes read 64 consecutive blocks: coalesced 16-B and 8-B loads off a wave-uniform base with
// 32-bit lane offsets), plus the packed word and sign word before the wave's first block of
// each round (wave-uniform addresses); the other lanes' words before their block are the lane
// below's last words (DPP, no load).  Offsets clamped to the last block: no branch around a
// load.
struct Batch {
    uint4 w[kBatch];
    uint2 s[kBatch];
    uint32_t wp0[kBatch], sp0[kBatch];
};
__device__ __forceinline__ void load_batch(Batch& b, const uint4* __restrict__ packed4,
                                           const uint2* __restrict__ sign2,
                                           const uint32_t* __restrict__ packed,
                                           const uint32_t* __restrict__ sign, int64_t g,
                                           int lane, uint32_t stride, int64_t nblk, uint32_t zv) {
    const int64_t lim64 = nblk - 1 - g;   // wave-uniform; >= 0 for the rounds that count
    const uint32_t lim = lim64 < 0 ? 0u : lim64 > 0x7FFFFFFF ? 0x7FFFFFFFu : (uint32_t)lim64;
    const uint4* pb = packed4 + min(g, nblk - 1);
    const uint2* sb = sign2 + min(g, nblk - 1);
    const uint32_t base_ok = g < nblk ? 1u : 0u;   // (past the end: every offset 0)
#pragma unroll
    for (int r = 0; r < kBatch; ++r) {
        const uint32_t o = min((uint32_t)lane + (uint32_t)r * stride, lim) * base_ok;
        b.w[r] = pb[o];
        b.s[r] = sb[o];
        // (zv: an opaque zero in a VGPR, so that these wave-uniform loads stay VECTOR loads,
        // counted in order with the batch's other loads: as scalar loads they made every
        // batch wait lgkmcnt(0) — for the NEXT batch's scalar loads too, which SMEM returns
        // out of order)
        const int64_t ip = min(max(g + (int64_t)r * stride - 1, (int64_t)0), nblk - 1);
        b.wp0[r] = packed[4 * ip + 3 + zv];
        b.sp0[r] = sign[2 * ip + 1 + zv];
    }
}

// done != nullptr: the last workgroup to finish also finalizes (one launch per call).
// kPow2: chunk_len / 64 is a power of two (the reference's 0x10000: chunk starts by a mask).
template <bool kPow2>
__global__ __launch_bounds__(kCountThreads) __attribute__((amdgpu_waves_per_eu(kCntWavesPerEU)))
void k_count_main(const uint4* __restrict__ packed4, const uint2* __restrict__ sign2,
                  const uint32_t* __restrict__ packed, const uint32_t* __restrict__ sign,
                  int64_t nblk, int64_t blk_per_chunk, unsigned long long* __restrict__ gacc,
                  unsigned int* done, int64_t* __restrict__ out) {
    __shared__ uint32_t scnt[kRaw];   // the workgroup's counters (LDS atomics)
    __shared__ uint32_t spp[16 * 16];  // '+'->'+' moments, lane-spread replicas (Lane)
    __shared__ uint64_t raw[kRaw];
    __shared__ int s_last;
    const int t = threadIdx.x, lane = t & 63;
    if (t < kRaw) scnt[t] = 0u;
    spp[t] = 0u;   // (kCountThreads == 256 == 16 x 16)
    __syncthreads();
    cnt::Lane lc(spp);
    const uint32_t stride = gridDim.x * blockDim.x;
    const int64_t step = (int64_t)kBatch * stride;
    // the wave's first block (wave-uniform): every lane of a wave runs every batch, so the
    // flush's shuffles see the whole wave
    int64_t g = (int64_t)blockIdx.x * blockDim.x + __builtin_amdgcn_readfirstlane(t & ~63);
    // kTail: the last round, some of whose blocks lie past the end (their lanes count
    // nothing; the full rounds carry no validity test)
    auto count = [&](const Batch& b, int64_t gb, auto tail) {
        constexpr bool kTail = decltype(tail)::value;
#pragma unroll
        for (int r = 0; r < kBatch; ++r) {
            const uint32_t o = (uint32_t)lane + (uint32_t)r * stride;
            const uint32_t wp = from_lane_below(b.w[r].w, b.wp0[r]);
            const uint32_t sp = from_lane_below(b.s[r].y, b.sp0[r]) >> 31;
            const bool valid = !kTail || gb + (int64_t)o < nblk;
            // (a power-of-two chunk — the reference's 0x10000 — needs no 64-bit modulo)
            const bool cstart = kPow2 ? (((uint32_t)gb + o) & (uint32_t)(blk_per_chunk - 1)) == 0u
                                      : ((gb + (int64_t)o) % blk_per_chunk) == 0;
            if (valid && cstart) atomicAdd(&scnt[64 + cnt::init_state(b.w[r].x, b.s[r].x)], 1u);
            lc.block(b.w[r], b.s[r], wp, sp, cstart, scnt, valid);   // (every lane calls)
        }
    };
    // two batches in flight per lane: the next batch's loads are issued before the current
    // one is counted (ping-pong buffers)
    // a round is full when the wave's last block of it lies before the end (wave-uniform)
    const int64_t span = (int64_t)(kBatch - 1) * stride + 63;
    auto count_round = [&](const Batch& b, int64_t gb) {
        if (gb + span < nblk) count(b, gb, std::false_type{});
        else count(b, gb, std::true_type{});
    };
    uint32_t zv;
    asm volatile("v_mov_b32 %0, 0" : "=v"(zv));
    Batch A, B;
    load_batch(A, packed4, sign2, packed, sign, g, lane, stride, nblk, zv);
    while (g < nblk) {
        load_batch(B, packed4, sign2, packed, sign, g + step, lane, stride, nblk, zv);
        count_round(A, g);
        g += step;
        if (g < nblk) {
            load_batch(A, packed4, sign2, packed, sign, g + step, lane, stride, nblk, zv);
            count_round(B, g);
            g += step;
        }
    }
    lc.flush(scnt);   // (32-bit counters: a lane's blocks are far below their range)
    __syncthreads();
    cnt::pp_replicas_sum(spp, scnt, t);
    __syncthreads();
    if (t < kRaw) {
        const uint32_t v = cnt::raw_of(scnt, t);
        if (v)
            atomicAdd(gacc + (blockIdx.x % kCntRep) * kRaw + t, (unsigned long long)v);
    }
    if (done && last_workgroup(done, &s_last)) {
        if (t < kRaw) cnt::fin_load<true>(gacc, raw, t);
        __syncthreads();
        cnt::fin_store(gacc, raw, out, t, blockDim.x);
        reset_done(done);
    }
}

// One workgroup: the cpg_counts_i64 assembly from accumulators filled by earlier launches
// (the streamed genome), which it re-zeroes.
__global__ __launch_bounds__(128) void k_count_final(unsigned long long* __restrict__ gacc,
                                                     int64_t* __restrict__ out) {
    __shared__ uint64_t raw[kRaw];
    if (threadIdx.x < kRaw) cnt::fin_load<false>(gacc, raw, threadIdx.x);
    __syncthreads();
    cnt::fin_store(gacc, raw, out, threadIdx.x, blockDim.x);
}

}  // namespace

hipError_t launch_count(const uint32_t* packed, const uint32_t* sign, int64_t nchunks,
                        int64_t chunk_len, uint64_t* ws, int64_t* out, hipStream_t s, int parts) {
    const int64_t nblk = nchunks * chunk_len / 64;
    if (nblk <= 0 && parts == PART_ALL) return hipMemsetAsync(out, 0, 124 * sizeof(int64_t), s);
    if ((parts & PART_ACC) && nblk > 0) {
        // at most one batch per lane when the input is small (46 Mbp: ~0.7 batches per lane
        // of 1,024 workgroups), the grid cap when it is large
        int64_t grid = (nblk + (int64_t)kCountThreads * kBatch - 1) / ((int64_t)kCountThreads * kBatch);
        if (grid > kCntGrid) grid = kCntGrid;
        // the whole call in one launch: its last workgroup finalizes
        unsigned int* done = parts == PART_ALL ? (unsigned int*)(ws + kRaw * kCntRep) : nullptr;
        const int64_t bpc = chunk_len / 64;
        if ((bpc & (bpc - 1)) == 0)
            hipLaunchKernelGGL(k_count_main<true>, dim3((unsigned)grid), dim3(kCountThreads), 0, s,
                               (const uint4*)packed, (const uint2*)sign, packed, sign, nblk, bpc,
                               (unsigned long long*)ws, done, out);
        else
            hipLaunchKernelGGL(k_count_main<false>, dim3((unsigned)grid), dim3(kCountThreads), 0,
                               s, (const uint4*)packed, (const uint2*)sign, packed, sign, nblk, bpc,
                               (unsigned long long*)ws, done, out);
        if (done) return hipGetLastError();
    }
    if (parts & PART_FINAL)
        hipLaunchKernelGGL(k_count_final, dim3(1), dim3(128), 0, s, (unsigned long long*)ws, out);
    return hipGetLastError();
}

// + the done counters
size_t count_ws_bytes(int64_t) { return (size_t)kRaw * 8 * kCntRep + 4 * kDoneWords; }

}  // namespace cpg
