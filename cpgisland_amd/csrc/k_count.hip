// k_count.hip — labelled int64 counts on gfx950.
//
// Training-side counterpart of the BW mapper stripes (init / transition / emission rows,
// CpGIslandFinder.java:200) computed from hard labels: state s_t = base_t + (sign_t?0:4).
// Streams 2-bit packed bases (16 B per lane = 64 bases) and sign bits (8 B per lane) in
// grid-stride batches whose loads are all in flight before any block is counted, and counts
// with v_bcnt over base bit-masks (count_dev.h; shared with the fused training pass in
// k_estep.hip).
//
// Per-workgroup partial counts (and the init states of the chunks starting in the
// workgroup) are added to 72 global 64-bit accumulators (integer atomics: exact and
// order-independent, one per counter per workgroup); the last workgroup to finish derives the
// emission/dinucleotide/mono counts from the transition + init counts (exact integer
// identities) and re-zeroes the accumulators.  One launch per call (a separate one-workgroup
// finalize launch for the streamed genome, which accumulates every window first).

#include "count_dev.h"

namespace cpg {
namespace {

using cnt::kRaw;
constexpr int kCountThreads = 256;
constexpr int kCntRep = cnt::kRep;
constexpr int kCntGrid = 512;   // measured: 2048 / 1024 / 512 workgroups 19.0 / 14.6 / 12.9 us at 46 Mbp
constexpr int kBatch = 6;       // blocks per lane in flight (46 Mbp: 5.5 blocks per lane at 512 x 256)
static_assert(kBatch <= cnt::Lane::kMaxBlocks, "16-bit wave sums");

// done != nullptr: the last workgroup to finish also finalizes (one launch per call)
__global__ __launch_bounds__(kCountThreads) void k_count_main(
    const uint4* __restrict__ packed4, const uint2* __restrict__ sign2,
    const uint32_t* __restrict__ packed, const uint32_t* __restrict__ sign, int64_t nblk,
    int64_t blk_per_chunk, unsigned long long* __restrict__ gacc, unsigned int* done,
    int64_t* __restrict__ out) {
    __shared__ uint32_t scnt[kRaw];   // the workgroup's counters (LDS atomics)
    __shared__ uint64_t raw[kRaw];
    __shared__ int s_last;
    const int t = threadIdx.x;
    const bool pow2 = (blk_per_chunk & (blk_per_chunk - 1)) == 0;
    if (t < kRaw) scnt[t] = 0u;
    __syncthreads();
    cnt::Lane lc;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    // grid-stride batches: all of a batch's words are loaded before any is counted, so a lane
    // waits for memory once per batch (the loop is latency-bound, not VALU-bound)
    // (the loop bound is the workgroup's first block: every lane runs every batch, so the
    // flush's shuffles see the whole wave)
    for (int64_t g0 = (int64_t)blockIdx.x * blockDim.x; g0 < nblk; g0 += kBatch * stride) {
        const int64_t i0 = g0 + t;
        uint4 w[kBatch];
        uint2 s[kBatch];
        uint32_t wp[kBatch], sp[kBatch];
        // unconditional loads (index clamped) and no arithmetic on their results here: a
        // load under a branch, or a shift of a loaded word, makes the compiler wait for it
        // before issuing the next — one memory round trip per block instead of per batch
#pragma unroll
        for (int r = 0; r < kBatch; ++r) {
            const int64_t i = min(i0 + r * stride, nblk - 1);
            const int64_t ip = i > 0 ? i - 1 : 0;
            w[r] = packed4[i];
            s[r] = sign2[i];
            wp[r] = packed[4 * ip + 3];
            sp[r] = sign[2 * ip + 1];
        }
#pragma unroll
        for (int r = 0; r < kBatch; ++r) {
            const int64_t i = i0 + r * stride;
            if (i < nblk) {
                // (a power-of-two chunk — the reference's 0x10000 — needs no 64-bit modulo)
                const bool cstart = pow2 ? (i & (blk_per_chunk - 1)) == 0 : (i % blk_per_chunk) == 0;
                if (cstart) atomicAdd(&scnt[64 + cnt::init_state(w[r].x, s[r].x)], 1u);
                lc.block(w[r], s[r], wp[r], sp[r] >> 31, cstart, scnt);
            }
        }
        lc.flush(scnt);   // per batch: kBatch <= Lane::kMaxBlocks
    }
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
        int grid = kCntGrid;
        if ((int64_t)grid * kCountThreads > nblk)
            grid = (int)((nblk + kCountThreads - 1) / kCountThreads);
        // the whole call in one launch: its last workgroup finalizes
        unsigned int* done = parts == PART_ALL ? (unsigned int*)(ws + kRaw * kCntRep) : nullptr;
        hipLaunchKernelGGL(k_count_main, dim3(grid), dim3(kCountThreads), 0, s,
                           (const uint4*)packed, (const uint2*)sign, packed, sign, nblk,
                           chunk_len / 64, (unsigned long long*)ws, done, out);
        if (done) return hipGetLastError();
    }
    if (parts & PART_FINAL)
        hipLaunchKernelGGL(k_count_final, dim3(1), dim3(128), 0, s, (unsigned long long*)ws, out);
    return hipGetLastError();
}

// + the done counters
size_t count_ws_bytes(int64_t) { return (size_t)kRaw * 8 * kCntRep + 4 * kDoneWords; }

}  // namespace cpg
