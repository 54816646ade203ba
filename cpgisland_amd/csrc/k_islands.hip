// k_islands.hip — island scan + filter (CpGIslandFinder.java:262-339) on gfx950.
//
// The reference walks each decoded 1 Mi chunk sequentially.  Its state is re-expressed as
// bit-parallel masks over 32-position words (sign bits + 2-bit packed bases):
//   start  = S & ~S_prev          (:319-337, inIsland false -> true)
//   close  = ~S & S_prev          (:273-289, the '-' that ends the island; end = i-1)
//   C, G   = base masks, CGm = G & C_prev (a G whose predecessor is a C)
// Island counts are differences of chunk-prefix counts taken at the run boundaries; CpG
// inside (beg, end] is exact from CGm.  The one serial quirk — `atC` is never cleared when an
// island closes (:325-331), so the first pair of an island can count a CpG against the
// previous island's last C — is a function stale_in -> stale_out per island (const 0 /
// const 1 / identity), resolved by a scan over the chunk's islands.  Islands still open at
// the chunk end are dropped (:269-339 never closes them).  Coordinates and
// (cgCount*islandLen) use Java int arithmetic.
//
// Kernels:
//   T (per tile of 1,024 words = 32,768 positions, all CUs streaming): counts, a workgroup
//     scan, and a record per run boundary with the tile-local prefix counts at it, written
//     at its tile-local rank into the tile's slice of the run lists; the tile totals;
//   R (per chunk): tile offsets (scan of the tile totals), per-run stats, stale-atC scan,
//     filter, kept ranks, the chunk's kept count;
//   W (per chunk): the chunk's first record = the kept counts of the chunks before it (summed
//     from R's per-chunk counts: a kernel boundary instead of a look-back, so no workgroup
//     ever waits for another), island records.
// (The fused decode, k_viterbi.hip, runs R for a chunk in its last traceback workgroup; W
// runs after the traceback.)
// A whole chunk per workgroup would stream at one CU's share of the memory system (≈25-70
// GB/s per CU): the tiles spread the one pass over the data on every CU.

#include <algorithm>
#include <atomic>

#include "cpg_internal.h"
#include "isl_dev.h"

namespace cpg {
namespace {

constexpr int kIT = 1024;    // lanes of the per-chunk kernels
constexpr int kTT = 256;     // lanes of the tile kernel
constexpr int kTRows = 1;           // rows of kTT * 4 words per tile (1: 1,376 tiles per
                                    // 46 Mbp — 7.3 us; 4 rows: 344 tiles — 11.0 us)
constexpr int64_t kTW = (int64_t)kTT * 4 * kTRows;   // words per tile (1,024 with one row)
// a fused decode's tiles: one traceback workgroup's 256 blocks of 256 positions
constexpr int64_t kFTW = 2048;

using namespace isl;

IslWs carve_isl(void* base, int64_t nchunks, int64_t C, int64_t tw) {
    const int64_t nw = C / 32, maxr = C / 2 + 1;
    IslWs w;
    w.ntile = std::max<int64_t>(1, (nw + tw - 1) / tw);
    w.cap_t = std::min<int64_t>(tw * 16 + 1, maxr);   // a tile holds <= 16 runs per word
    char* p = static_cast<char*>(base);
    size_t o = 0;
    auto take = [&](size_t b) {
        o = (o + 255) & ~size_t(255);
        char* r = p ? p + o : nullptr;
        o += b;
        return r;
    };
    const int64_t nt = nchunks * w.ntile;
    w.starts = (RunRec*)take(nt * w.cap_t * sizeof(RunRec));
    w.closes = (RunRec*)take(nt * w.cap_t * sizeof(RunRec));
    w.ttot = (Cnt5*)take(nt * sizeof(Cnt5));
    w.toff = (Cnt5*)take(nt * sizeof(Cnt5));
    w.kept = (int32_t*)take(nchunks * maxr * 4);
    w.cres = (int2*)take(nchunks * sizeof(int2));
    w.cbase = (long long*)take(nchunks * 8);
    w.bsum = (long long*)take(((nchunks + kBaseBlock - 1) / kBaseBlock) * 8);
    w.scanned = nchunks > kInlineBaseMax ? 1 : 0;
    w.bytes = o + 256;
    return w;
}

// the 4 words w0..w0+3 of a chunk (words >= nw read as 0) and the words before them
struct Quad {
    uint32_t S[4], P[8], sprev, pprev;
};
__device__ __forceinline__ Quad load_quad(const uint32_t* __restrict__ pk,
                                          const uint32_t* __restrict__ sg, int64_t w0,
                                          int64_t nw) {
    Quad q;
    if (w0 + 4 <= nw) {
        const uint4 s4 = *reinterpret_cast<const uint4*>(sg + w0);
        const uint4 p0 = *reinterpret_cast<const uint4*>(pk + 2 * w0);
        const uint4 p1 = *reinterpret_cast<const uint4*>(pk + 2 * w0 + 4);
        q.S[0] = s4.x; q.S[1] = s4.y; q.S[2] = s4.z; q.S[3] = s4.w;
        q.P[0] = p0.x; q.P[1] = p0.y; q.P[2] = p0.z; q.P[3] = p0.w;
        q.P[4] = p1.x; q.P[5] = p1.y; q.P[6] = p1.z; q.P[7] = p1.w;
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const bool in = w0 + i < nw;
            q.S[i] = in ? sg[w0 + i] : 0u;
            q.P[2 * i] = in ? pk[2 * (w0 + i)] : 0u;
            q.P[2 * i + 1] = in ? pk[2 * (w0 + i) + 1] : 0u;
        }
    }
    q.sprev = (w0 > 0 && w0 < nw) ? sg[w0 - 1] : 0u;
    q.pprev = (w0 > 0 && w0 < nw) ? pk[2 * w0 - 1] : 0u;
    return q;
}
__device__ __forceinline__ WordMasks quad_masks(const Quad& q, int i) {   // i compile-time
    return masks_reg(q.S[i], i ? q.S[i - 1] : q.sprev, q.P[2 * i], q.P[2 * i + 1],
                     i ? q.P[2 * i - 1] : q.pprev);
}

// T: one tile.  Lane t owns words 4t..4t+3 of each of the tile's 4 rows of 1,024 words
// (coalesced 16-B loads); the scan runs over (row, lane) in word order: the lane's four row
// counts are packed two fields per 32-bit word (a wave row sums to <= 8,192) and scanned by
// wave shuffles together, the wave totals of every row meet in LDS behind one barrier.
__global__ __launch_bounds__(kTT) void k_isl_tile(const uint32_t* packed, const uint32_t* sign,
                                                 int64_t C, IslWs ws) {
    const int64_t c = blockIdx.x / ws.ntile;
    const int64_t k = blockIdx.x - c * ws.ntile;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int64_t nw = C / 32;
    const uint32_t* pk = packed + c * (C / 16);
    const uint32_t* sg = sign + c * nw;
    Quad q[kTRows];
#pragma unroll
    for (int r = 0; r < kTRows; ++r) q[r] = load_quad(pk, sg, k * kTW + r * (kTT * 4) + 4 * t, nw);
    uint32_t x[kTRows][3], own[kTRows][3];
#pragma unroll
    for (int r = 0; r < kTRows; ++r) {
        Cnt5 s{0, 0, 0, 0, 0};
        const int64_t w0 = k * kTW + r * (kTT * 4) + 4 * t;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (w0 + i < nw) s = cadd(s, cnt_of(quad_masks(q[r], i)));
        own[r][0] = x[r][0] = (uint32_t)s.c | ((uint32_t)s.g << 16);
        own[r][1] = x[r][1] = (uint32_t)s.cg | ((uint32_t)s.st << 16);
        own[r][2] = x[r][2] = (uint32_t)s.cl;
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
#pragma unroll
        for (int r = 0; r < kTRows; ++r)
#pragma unroll
            for (int f = 0; f < 3; ++f) {
                const uint32_t y = __shfl_up(x[r][f], off);
                if (lane >= off) x[r][f] += y;
            }
    }
    __shared__ Cnt5 wt[kTRows][kTT / 64];
    if (lane == 63)
#pragma unroll
        for (int r = 0; r < kTRows; ++r)
            wt[r][wv] = Cnt5{(int32_t)(x[r][0] & 0xFFFFu), (int32_t)(x[r][0] >> 16),
                             (int32_t)(x[r][1] & 0xFFFFu), (int32_t)(x[r][1] >> 16),
                             (int32_t)x[r][2]};
    __syncthreads();
    RunRec* st = ws.starts + blockIdx.x * ws.cap_t;
    RunRec* cl = ws.closes + blockIdx.x * ws.cap_t;
    Cnt5 rowbase{0, 0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < kTRows; ++r) {
        Cnt5 e = rowbase;
#pragma unroll
        for (int w = 0; w < kTT / 64; ++w) {
            const Cnt5 s = wt[r][w];
            if (w < wv) e = cadd(e, s);
            rowbase = cadd(rowbase, s);
        }
        const uint32_t ex0 = x[r][0] - own[r][0], ex1 = x[r][1] - own[r][1], ex2 = x[r][2] - own[r][2];
        e = cadd(e, Cnt5{(int32_t)(ex0 & 0xFFFFu), (int32_t)(ex0 >> 16), (int32_t)(ex1 & 0xFFFFu),
                         (int32_t)(ex1 >> 16), (int32_t)ex2});
        if ((own[r][1] >> 16) | own[r][2]) {   // the lane's words hold a run boundary
            const int64_t w0 = k * kTW + r * (kTT * 4) + 4 * t;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (w0 + i < nw) emit_word(quad_masks(q[r], i), w0 + i, e, st, cl);
        }
    }
    if (t == 0) ws.ttot[blockIdx.x] = rowbase;
}

// R, two passes (no workgroup waits for another: two processes' decodes may share a GPU):
// the per-chunk resolve up to the kept words and counts (resolve_chunk), then the records
// (write_runs) once every chunk's kept count is in ws.cres
constexpr int kToffLds = 1024;
__global__ __launch_bounds__(kIT) void k_isl_resolve(const uint32_t* packed, int64_t C,
                                                    IslWs ws) {
    __shared__ ResolveLds L;
    __shared__ Cnt5 s_to[kToffLds];
    resolve_chunk<false, kToffLds>(packed, C, ws, blockIdx.x, L, s_to);
}
__global__ __launch_bounds__(kIT) void k_isl_write(const uint32_t* packed, int64_t C, IslWs ws,
                                                  IslOut o) {
    __shared__ long long s_part[kIT / 64];
    __shared__ int32_t sk[kIT / 64];
    write_runs(packed, C, ws, o, blockIdx.x, s_part, sk);
}

// Between the passes, past kInlineBaseMax chunks: every chunk's first record in two launches
// (O(chunks) work).  k_isl_base: per block of kBaseBlock chunks, the exclusive scan of their
// kept counts -> cbase, the block's total -> bsum (a block's total < 2^31: a chunk keeps at
// most chunk_len / 2 islands, 2^19 x 1,024 chunks).  k_isl_bscan: one workgroup, the block
// totals' exclusive scan in place (int64).
__global__ __launch_bounds__(kBaseBlock) void k_isl_base(IslWs ws, int64_t nchunks) {
    __shared__ int32_t sk[kBaseBlock / 64];
    const int64_t c = (int64_t)blockIdx.x * kBaseBlock + threadIdx.x;
    const int32_t v = c < nchunks ? ws.cres[c].x : 0;
    int32_t tot;
    const int32_t e = wg_scan_sum(v, sk, tot);
    if (c < nchunks) ws.cbase[c] = e;
    if (threadIdx.x == 0) ws.bsum[blockIdx.x] = tot;
}
__global__ __launch_bounds__(kBaseBlock) void k_isl_bscan(IslWs ws, int64_t nblocks) {
    __shared__ long long sw[2][kBaseBlock / 64];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    long long carry = 0;
    for (int64_t b0 = 0, it = 0; b0 < nblocks; b0 += kBaseBlock, ++it) {
        const int64_t i = b0 + t;
        const long long v = i < nblocks ? ws.bsum[i] : 0;
        long long x = v;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const long long y = __shfl_up(x, off);
            if (lane >= off) x += y;
        }
        if (lane == 63) sw[it & 1][wv] = x;   // double-buffered: one barrier per block
        __syncthreads();
        long long before = 0, tot = 0;
        for (int w = 0; w < kBaseBlock / 64; ++w) {
            const long long s = sw[it & 1][w];
            before += w < wv ? s : 0;
            tot += s;
        }
        if (i < nblocks) ws.bsum[i] = carry + before + x - v;
        carry += tot;
    }
}

// the second pass (and, past kInlineBaseMax chunks, the base scan before it)
void launch_write(const uint32_t* packed, const IslWs& ws, const IslOut& o, int64_t nchunks,
                  int64_t C, hipStream_t s) {
    if (ws.scanned) {
        const int64_t nb = (nchunks + kBaseBlock - 1) / kBaseBlock;
        hipLaunchKernelGGL(k_isl_base, dim3((unsigned)nb), dim3(kBaseBlock), 0, s, ws, nchunks);
        hipLaunchKernelGGL(k_isl_bscan, dim3(1), dim3(kBaseBlock), 0, s, ws, nb);
    }
    hipLaunchKernelGGL(k_isl_write, dim3((unsigned)nchunks), dim3(kIT), 0, s, packed, C, ws, o);
}
// both resolve passes
void launch_resolve(const uint32_t* packed, const IslWs& ws, const IslOut& o, int64_t nchunks,
                    int64_t C, hipStream_t s) {
    hipLaunchKernelGGL(k_isl_resolve, dim3((unsigned)nchunks), dim3(kIT), 0, s, packed, C, ws);
    launch_write(packed, ws, o, nchunks, C, s);
}

}  // namespace

size_t islands_ws_bytes(int64_t nchunks, int64_t chunk_len) {
    return std::max(carve_isl(nullptr, nchunks, chunk_len, kTW).bytes,
                    islands_fusable(nchunks, chunk_len)
                        ? carve_isl(nullptr, nchunks, chunk_len, kFTW).bytes : size_t(0));
}

// the traceback's workgroups are the tiles: 256 whole blocks of 256 positions, inside one
// chunk (vit_nsb(C) a multiple of 256)
bool islands_fusable(int64_t nchunks, int64_t chunk_len) {
    return nchunks > 0 && chunk_len % (kFTW * 32) == 0;
}

hipError_t islands_fuse(IslFuse* f, void* ws, size_t ws_bytes, int64_t nchunks,
                        int64_t chunk_len, int64_t first_chunk, cpg_island* out, int64_t cap,
                        int64_t* count, unsigned int* done, const int64_t* base_in) {
    if (!islands_fusable(nchunks, chunk_len) || !done) return hipErrorInvalidValue;
    f->ws = carve_isl(ws, nchunks, chunk_len, kFTW);
    if (f->ws.bytes > ws_bytes) return hipErrorInvalidValue;
    f->o = IslOut{out, cap, count, base_in, first_chunk, nchunks};
    f->done = done;
    return hipSuccess;
}
// the records of a fused decode whose traceback resolved every chunk (first pass)
hipError_t islands_write(const uint32_t* packed, const IslFuse& f, int64_t chunk_len,
                         hipStream_t s) {
    launch_write(packed, f.ws, f.o, f.o.nchunks, chunk_len, s);
    return hipGetLastError();
}

// past 256 chunks the fused decode's traceback writes the tiles (kFTW, plain stores: f->done
// stays null) and islands_resolve runs the two resolve passes after it
hipError_t islands_tiles(IslFuse* f, void* ws, size_t ws_bytes, int64_t nchunks,
                         int64_t chunk_len, int64_t first_chunk, cpg_island* out, int64_t cap,
                         int64_t* count, const int64_t* base_in) {
    if (!islands_fusable(nchunks, chunk_len)) return hipErrorInvalidValue;
    f->ws = carve_isl(ws, nchunks, chunk_len, kFTW);
    if (f->ws.bytes > ws_bytes) return hipErrorInvalidValue;
    f->o = IslOut{out, cap, count, base_in, first_chunk, nchunks};
    f->done = nullptr;
    return hipSuccess;
}
hipError_t islands_resolve(const uint32_t* packed, const IslFuse& f, int64_t chunk_len,
                           hipStream_t s) {
    launch_resolve(packed, f.ws, f.o, f.o.nchunks, chunk_len, s);
    return hipGetLastError();
}

hipError_t launch_islands(const uint32_t* packed, const uint32_t* sign, int64_t nchunks,
                          int64_t chunk_len, int64_t first_chunk, void* wsp, size_t ws_bytes,
                          cpg_island* out, int64_t cap, int64_t* count, hipStream_t s,
                          const int64_t* base_in) {
    IslWs ws = carve_isl(wsp, nchunks, chunk_len, kTW);
    if (ws.bytes > ws_bytes) return hipErrorInvalidValue;
    if (nchunks == 0)
        return base_in ? hipMemcpyAsync(count, base_in, sizeof(int64_t), hipMemcpyDeviceToDevice, s)
                       : hipMemsetAsync(count, 0, sizeof(int64_t), s);
    hipLaunchKernelGGL(k_isl_tile, dim3((unsigned)(nchunks * ws.ntile)), dim3(kTT), 0, s, packed,
                       sign, chunk_len, ws);
    const IslOut o{out, cap, count, base_in, first_chunk, nchunks};
    launch_resolve(packed, ws, o, nchunks, chunk_len, s);
    return hipGetLastError();
}

}  // namespace cpg
