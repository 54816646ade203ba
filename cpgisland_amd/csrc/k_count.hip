// k_count.hip — labelled int64 counts on gfx950.
//
// Training-side counterpart of the BW mapper stripes (init / transition / emission rows,
// CpGIslandFinder.java:200) computed from hard labels: state s_t = base_t + (sign_t?0:4).
// Streams 2-bit packed bases (16 B per lane = 64 bases) and sign bits (8 B per lane) in
// grid-stride rounds, the next round's loads in flight while a round is counted, and counts
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
// the grid cap: 4 waves per SIMD (<= 128 VGPRs) hold 1,024 workgroups of 4 waves at once;
// every lane has two rounds in flight (the one being counted and the next one's loads)
constexpr int kCntGrid = 2048;
// s_waitcnt vmcnt(0) (gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15 — only the vector memory
// counter is waited for)
constexpr int kVmcnt0 = 0x0F70;
constexpr int kCntWavesPerEU = 4;

// the value of `v` in the lane below (wave_shr:1 DPP); lane 0 takes `old`
__device__ __forceinline__ uint32_t from_lane_below(uint32_t v, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xF, 0xF, false);
}

// One wave-round: the 64 consecutive blocks g .. g+63, block g + lane in lane `lane` (coalesced
// 16-B packed and 8-B label loads off a wave-uniform base), plus the packed word and the label
// word before block g (wave-uniform addresses); the other lanes' words before their block are
// the lane below's last words (DPP, no load).
struct Round {
    uint4 w;
    uint2 s;
    uint32_t wp0, sp0;
};
// a full round (every block < nblk): no clamp, no validity.  zv: an opaque zero in a VGPR, so
// that the wave-uniform loads stay VECTOR loads, counted in order with the round's other loads
// (as scalar loads they made every round wait lgkmcnt(0) — for the NEXT round's scalar loads
// too, which SMEM returns out of order)
__device__ __forceinline__ void load_round(Round& r, const uint4* __restrict__ packed4,
                                           const uint2* __restrict__ sign2,
                                           const uint32_t* __restrict__ packed,
                                           const uint32_t* __restrict__ sign, int64_t g, int lane,
                                           uint32_t zv) {
    r.w = (packed4 + g)[lane];
    r.s = (sign2 + g)[lane];
    const int64_t ip = g > 0 ? g - 1 : 0;   // (block 0 is a chunk start: its word is unused)
    r.wp0 = packed[4 * ip + 3 + zv];
    r.sp0 = sign[2 * ip + 1 + zv];
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
    __shared__ uint64_t raw[kRaw];
    __shared__ int s_last;
    const int t = threadIdx.x, lane = t & 63;
    if (t < kRaw) scnt[t] = 0u;
    __syncthreads();
    cnt::Lane lc;
    const int64_t step = (int64_t)gridDim.x * blockDim.x;   // blocks per grid round
    // the wave's first block (wave-uniform): every lane of a wave runs every round, so the
    // flush's shuffles see the whole wave
    int64_t g = (int64_t)blockIdx.x * blockDim.x + __builtin_amdgcn_readfirstlane(t & ~63);
    auto chunk_start = [&](int64_t b) {
        // (a power-of-two chunk — the reference's 0x10000 — needs no 64-bit modulo)
        return kPow2 ? ((uint32_t)b & (uint32_t)(blk_per_chunk - 1)) == 0u : (b % blk_per_chunk) == 0;
    };
    auto count_round = [&](const Round& r, int64_t gb, bool valid) {
        const uint32_t wp = from_lane_below(r.w.w, r.wp0);
        const uint32_t sp = from_lane_below(r.s.y, r.sp0) >> 31;
        const bool cstart = valid && chunk_start(gb + lane);
        if (cstart) atomicAdd(&scnt[64 + cnt::init_state(r.w.x, r.s.x)], 1u);
        lc.block(r.w, r.s, wp, sp, cstart, scnt, valid);   // (every lane calls)
    };
    uint32_t zv;
    asm volatile("v_mov_b32 %0, 0" : "=v"(zv));
    // full rounds, two per iteration (ping-pong buffers): the next round's loads are issued
    // before the current one is counted — and only once the current round's have landed
    // (vmcnt(0)), so that a wave holds exactly ONE round of loads in flight while it counts,
    // never two: on this chip a streaming read runs faster with fewer requests outstanding
    // (tools/loadshape.hip: one round in flight per wave 6.1-6.5 TB/s, two 5.4-5.8; the count
    // kernel 0.2435-0.2538 -> 0.2314-0.2330 ms at 3.1 Gbp, profiles/r06_count/).  A round is
    // full when the wave's last block of it lies before the end (wave-uniform).
    const int64_t gfull = nblk - 64;
    Round A, B;
    if (g <= gfull) load_round(A, packed4, sign2, packed, sign, g, lane, zv);
    while (g <= gfull) {
        __builtin_amdgcn_s_waitcnt(kVmcnt0);
        if (g + step <= gfull) load_round(B, packed4, sign2, packed, sign, g + step, lane, zv);
        count_round(A, g, true);
        g += step;
        if (g > gfull) break;
        __builtin_amdgcn_s_waitcnt(kVmcnt0);
        if (g + step <= gfull) load_round(A, packed4, sign2, packed, sign, g + step, lane, zv);
        count_round(B, g, true);
        g += step;
    }
    // the grid's last, partial round (at most one wave has it): lanes past the end count
    // nothing (every lane still calls: the wave reductions)
    if (g < nblk) {
        const bool valid = g + lane < nblk;
        const int64_t bb = valid ? g + lane : nblk - 1;
        Round r;
        r.w = packed4[bb];
        r.s = sign2[bb];
        const int64_t ip = g > 0 ? g - 1 : 0;
        r.wp0 = packed[4 * ip + 3 + zv];
        r.sp0 = sign[2 * ip + 1 + zv];
        count_round(r, g, valid);
    }
    lc.flush(scnt);   // (32-bit counters: a lane's blocks are far below their range)
    lc.flush_plus(scnt);
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
        // at most one round per lane when the input is small (46 Mbp: ~0.7 rounds per lane
        // of 1,024 workgroups), the grid cap when it is large
        int64_t grid = (nblk + (int64_t)kCountThreads - 1) / kCountThreads;
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
