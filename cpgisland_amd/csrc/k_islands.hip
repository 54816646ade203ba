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
//     filter, kept rank, the chunk's first record from a look-back over the earlier chunks'
//     published counts, island records.
// A whole chunk per workgroup would stream at one CU's share of the memory system (≈25-70
// GB/s per CU): the tiles spread the one pass over the data on every CU.

#include <algorithm>
#include <atomic>

#include "cpg_internal.h"

namespace cpg {
namespace {

constexpr int kIT = 1024;    // lanes of the per-chunk kernels
constexpr int kTT = 256;     // lanes of the tile kernel
#ifndef ISL_TROWS
#define ISL_TROWS 1
#endif
constexpr int kTRows = ISL_TROWS;   // rows of kTT * 4 words per tile (1: 1,376 tiles per
                                    // 46 Mbp — 7.3 us; 4 rows: 344 tiles — 11.0 us)
constexpr int64_t kTW = (int64_t)kTT * 4 * kTRows;   // words per tile (4,096)

__device__ __forceinline__ uint32_t compact16(uint32_t x) {   // even bits -> low 16 bits
    x &= 0x55555555u;
    x = (x | (x >> 1)) & 0x33333333u;
    x = (x | (x >> 2)) & 0x0F0F0F0Fu;
    x = (x | (x >> 4)) & 0x00FF00FFu;
    x = (x | (x >> 8)) & 0x0000FFFFu;
    return x;
}

struct WordMasks {
    uint32_t S, start, close, C, G, CG;
};

// masks of one sign word from registers: S, the previous sign word, its two packed words
// and the packed word before them (0 at the chunk start)
__device__ __forceinline__ WordMasks masks_reg(uint32_t S, uint32_t Sprev, uint32_t w0,
                                               uint32_t w1, uint32_t wprev) {
    WordMasks m;
    const uint32_t Sp = (S << 1) | (Sprev >> 31);
    m.S = S;
    m.start = S & ~Sp;
    m.close = ~S & Sp;
    const uint32_t h0 = w0 >> 1, h1 = w1 >> 1;
    const uint32_t c = compact16(w0 & ~h0) | (compact16(w1 & ~h1) << 16);
    const uint32_t g = compact16(h0 & ~w0) | (compact16(h1 & ~w1) << 16);
    m.C = c;
    m.G = g;
    m.CG = g & ((c << 1) | ((wprev >> 30) == 1u));
    return m;
}

struct Cnt5 {
    int32_t c, g, cg, st, cl;
};
__device__ __forceinline__ Cnt5 cnt_of(const WordMasks& m) {
    return Cnt5{(int32_t)__popc(m.C), (int32_t)__popc(m.G), (int32_t)__popc(m.CG),
                (int32_t)__popc(m.start), (int32_t)__popc(m.close)};
}
__device__ __forceinline__ Cnt5 cadd(Cnt5 a, const Cnt5& b) {
    a.c += b.c; a.g += b.g; a.cg += b.cg; a.st += b.st; a.cl += b.cl;
    return a;
}

// a run boundary with the prefix counts at it: start records carry C, G before `pos` and
// CpG up to and including `pos` (the run's first pair is (pos, pos+1)); close records carry
// C, G, CpG before `pos` (the first '-' after the run).  `pos` is chunk-relative; the counts
// are tile-relative in the lists (the tile offsets are added when a record is read).
struct RunRec {
    uint32_t pos;
    int32_t c, g, cg;
};

struct IslWs {
    RunRec* starts;     // per tile, cap_t records
    RunRec* closes;
    Cnt5* ttot;         // per tile: totals (kernel T)
    Cnt5* toff;         // per tile: exclusive prefix in its chunk (kernel R)
    int32_t* kept;      // per chunk, maxr: rank*2 | stale_in, or -1
    unsigned long long* flags;   // per chunk: epoch << 32 | kept islands (look-back)
    int64_t ntile;      // tiles per chunk
    int64_t cap_t;      // records per tile and kind
    size_t bytes;
};

IslWs carve_isl(void* base, int64_t nchunks, int64_t C) {
    const int64_t nw = C / 32, maxr = C / 2 + 1;
    IslWs w;
    w.ntile = std::max<int64_t>(1, (nw + kTW - 1) / kTW);
    w.cap_t = std::min<int64_t>(kTW * 16 + 1, maxr);   // a tile holds <= 16 runs per word
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
    w.flags = nullptr;   // WS_IFLG (launch_islands)
    w.bytes = o + 256;
    return w;
}

// the run boundaries of word w as records; e = the prefix counts before the word (advanced)
__device__ __forceinline__ void emit_word(const WordMasks& q, int64_t w, Cnt5& e,
                                          RunRec* __restrict__ st, RunRec* __restrict__ cl) {
    for (uint32_t x = q.start; x; x &= x - 1) {
        const int b = __ffs(x) - 1;
        const uint32_t lo = (1u << b) - 1u;
        st[e.st++] = RunRec{(uint32_t)(w * 32 + b), e.c + (int32_t)__popc(q.C & lo),
                            e.g + (int32_t)__popc(q.G & lo),
                            e.cg + (int32_t)__popc(q.CG & (lo | (1u << b)))};
    }
    for (uint32_t x = q.close; x; x &= x - 1) {
        const int b = __ffs(x) - 1;
        const uint32_t lo = (1u << b) - 1u;
        cl[e.cl++] = RunRec{(uint32_t)(w * 32 + b), e.c + (int32_t)__popc(q.C & lo),
                            e.g + (int32_t)__popc(q.G & lo), e.cg + (int32_t)__popc(q.CG & lo)};
    }
    e.c += __popc(q.C);
    e.g += __popc(q.G);
    e.cg += __popc(q.CG);
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

// workgroup scans (blockDim.x a multiple of 64, <= 1024): wave shuffles, the wave totals
// through LDS, one barrier each.  Every call uses its own LDS array (no reuse barrier).
__device__ __forceinline__ Cnt5 wg_scan5(const Cnt5 v, Cnt5* sw, Cnt5& total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    Cnt5 x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const Cnt5 y{__shfl_up(x.c, off), __shfl_up(x.g, off), __shfl_up(x.cg, off),
                     __shfl_up(x.st, off), __shfl_up(x.cl, off)};
        if (lane >= off) x = cadd(x, y);
    }
    if (lane == 63) sw[wv] = x;
    __syncthreads();
    Cnt5 before{0, 0, 0, 0, 0}, tot{0, 0, 0, 0, 0};
    for (int w = 0; w < nwv; ++w) {
        const Cnt5 s = sw[w];
        if (w < wv) before = cadd(before, s);
        tot = cadd(tot, s);
    }
    total = tot;
    return Cnt5{before.c + x.c - v.c, before.g + x.g - v.g, before.cg + x.cg - v.cg,
                before.st + x.st - v.st, before.cl + x.cl - v.cl};
}

__device__ __forceinline__ uint32_t isl_base(const uint32_t* pk, int64_t pos) {
    return (pk[pos >> 4] >> ((pos & 15) * 2)) & 3u;
}

// a chunk's tile offsets: in LDS, or in global memory written by this same kernel (read
// past this CU's L1: agent scope), or written by an earlier kernel (plain loads)
template <bool kAgent>
__device__ __forceinline__ int32_t ld_off(const int32_t* p) {
    if constexpr (kAgent) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
}

// the chunk's r-th start (kind 0) or close (kind 1) record with chunk-relative counts: the
// last tile whose exclusive offset is <= r (binary search over the chunk's tile offsets `to`)
template <bool kAgent>
__device__ __forceinline__ RunRec run_rec(const IslWs& ws, const Cnt5* to, int64_t c, int64_t r,
                                          int kind) {
    int64_t lo = 0, hi = ws.ntile - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        const int32_t v = ld_off<kAgent>(kind ? &to[mid].cl : &to[mid].st);
        if (v <= r) lo = mid; else hi = mid - 1;
    }
    const int32_t oc = ld_off<kAgent>(&to[lo].c), og = ld_off<kAgent>(&to[lo].g),
                  ocg = ld_off<kAgent>(&to[lo].cg),
                  ok = ld_off<kAgent>(kind ? &to[lo].cl : &to[lo].st);
    const int64_t tile = c * ws.ntile + lo;
    RunRec x = (kind ? ws.closes : ws.starts)[tile * ws.cap_t + (r - ok)];
    x.c += oc;
    x.g += og;
    x.cg += ocg;
    return x;
}

struct RunStat {
    int32_t beg, end, len, C, G, CGin;
    uint32_t b0, b1, last;
};
template <bool kAgent>
__device__ __forceinline__ RunStat run_stat(const uint32_t* pk, const IslWs& ws, const Cnt5* to,
                                            int64_t c, int64_t r) {
    const RunRec s = run_rec<kAgent>(ws, to, c, r, 0), e = run_rec<kAgent>(ws, to, c, r, 1);
    RunStat o;
    o.beg = (int32_t)s.pos;
    o.end = (int32_t)e.pos - 1;
    o.len = (int32_t)(e.pos - s.pos);
    o.C = e.c - s.c;
    o.G = e.g - s.g;
    o.CGin = o.len >= 2 ? e.cg - s.cg : 0;
    o.b0 = isl_base(pk, s.pos);
    o.b1 = o.len >= 2 ? isl_base(pk, s.pos + 1) : 0u;
    o.last = isl_base(pk, e.pos - 1);
    return o;
}
// stale atC map (bit x = output for input x): const0 0b00, const1 0b11, id 0b10
__device__ __forceinline__ uint32_t stale_map(const RunStat& r) {
    if (r.len >= 2) return r.last == 1u ? 0x3u : 0x0u;
    return r.b0 == 1u ? 0x3u : 0x2u;
}
__device__ __forceinline__ uint32_t mapply(uint32_t m, uint32_t x) { return (m >> x) & 1u; }
__device__ __forceinline__ uint32_t mcompose(uint32_t f, uint32_t g) {   // f o g
    return mapply(f, mapply(g, 0)) | (mapply(f, mapply(g, 1)) << 1);
}

struct Rec {
    double cg, oe;
    bool keep;
    int32_t cpg;
};
__device__ __forceinline__ Rec filter(const RunStat& r, uint32_t stale_in) {
    Rec o;
    o.cpg = r.CGin + ((r.len >= 2 && r.b1 == 2u && r.b0 != 1u && stale_in) ? 1 : 0);
    const double ccnt = (double)r.C, gcnt = (double)r.G;
    o.cg = (ccnt + gcnt) / (double)r.len;                          // :280
    o.oe = 0.0;
    if (r.C != 0 && r.G != 0) {                                     // :282-283
        const int32_t prod = (int32_t)((uint32_t)o.cpg * (uint32_t)r.len);   // int * int wraps
        o.oe = (double)prod / (ccnt * gcnt);
    }
    o.keep = (o.cg > 0.5) && (o.oe > 0.6);                          // :285
    return o;
}

// exclusive composition scan of stale maps (lane order = run order)
__device__ __forceinline__ uint32_t wg_scan_map(const uint32_t f, uint32_t* sw) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t x = f;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off);
        if (lane >= off) x = mcompose(x, y);
    }
    if (lane == 63) sw[wv] = x;
    __syncthreads();
    uint32_t before = 0x2u;   // identity
    for (int w = 0; w < wv; ++w) before = mcompose(sw[w], before);
    const uint32_t up = __shfl_up(x, 1);
    return lane > 0 ? mcompose(up, before) : before;
}
__device__ __forceinline__ int32_t wg_scan_sum(const int32_t v, int32_t* sw, int32_t& total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    int32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int32_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) sw[wv] = x;
    __syncthreads();
    int32_t before = 0, tot = 0;
    for (int w = 0; w < nwv; ++w) {
        const int32_t s = sw[w];
        before += w < wv ? s : 0;
        tot += s;
    }
    total = tot;
    return before + x - v;
}

// where the island records go (the former separate record kernel is fused into R)
struct IslOut {
    cpg_island* out;
    int64_t cap;
    int64_t* count;            // total records (with base_in)
    const int64_t* base_in;    // append mode: records already written before this call
    int64_t first_chunk;
    uint32_t epoch;            // tags this call's look-back flags
    uint32_t* status;          // ctx status word: ST_LOOKBACK_TIMEOUT when a spin gives up
};

__device__ __forceinline__ void put_island(const IslOut& o, const RunStat& rs, uint32_t stale_in,
                                           int64_t dst, int64_t gchunk, uint32_t cbase) {
    if (dst >= o.cap) return;
    const Rec f = filter(rs, stale_in);
    cpg_island isl;
    isl.beg1 = (int32_t)((uint32_t)rs.beg + cbase + 1u);          // :287
    isl.end1 = (int32_t)((uint32_t)rs.end + cbase + 1u);
    isl.len = rs.len;
    isl.chunk = (int32_t)gchunk;
    isl.cg = f.cg;
    isl.oe = f.oe;
    o.out[dst] = isl;
}

// kept islands of the chunks before c: a look-back over their flags (this call's epoch),
// one wave, windows of 64 chunks.  Workgroups start in chunk order, so every chunk waited
// on is running or done; the spin is bounded all the same (2 s of wall clock).  A spin that
// gives up sets ST_LOOKBACK_TIMEOUT in the status word (cpg_sync then fails the call: the
// offsets, and so every record and the count, are unusable) and counts nothing for that
// chunk.  CPG_ISL_SPIN_LIMIT (ticks of the 100 MHz wall clock) is a test hook.
#ifndef CPG_ISL_SPIN_LIMIT
#define CPG_ISL_SPIN_LIMIT 200000000ull
#endif
__device__ __forceinline__ long long kept_before(const IslWs& ws, int64_t c, uint32_t epoch,
                                                 uint32_t* status) {
    const int lane = threadIdx.x & 63;
    long long sum = 0;
    bool gave_up = false;
    const unsigned long long t0 = wall_clock64();
    for (int64_t j0 = c - 1; j0 >= 0; j0 -= 64) {
        const int64_t j = j0 - lane;
        if (j >= 0) {
            unsigned long long f;
            for (;;) {
                // deadline first: a limit of 0 gives up deterministically (the test hook)
                if (wall_clock64() - t0 >= (unsigned long long)(CPG_ISL_SPIN_LIMIT)) {
                    gave_up = true;
                    f = 0;
                    break;
                }
                f = __hip_atomic_load(ws.flags + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((uint32_t)(f >> 32) == epoch) break;
                __builtin_amdgcn_s_sleep(1);
            }
            sum += (long long)(uint32_t)f;
        }
    }
    if (gave_up) atomicOr(status, ST_LOOKBACK_TIMEOUT);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) sum += __shfl_xor(sum, off);
    return sum;
}

// the chunk's closed runs split over the lanes: stale-atC maps composed and scanned,
// filtered (:280-285), kept islands ranked, the chunk's first record found by the look-back,
// records written.  With <= 8 runs per lane the map and both filter outcomes (stale 0 / 1)
// of each run stay in registers: one pass of loads before the records.
template <bool kAgent>
__device__ __forceinline__ void resolve_runs(const uint32_t* pk, const IslWs& ws, const Cnt5* to,
                                             int64_t c, int64_t C, int64_t nr, int32_t* kept,
                                             uint32_t* sm, int32_t* sk, long long* sbase,
                                             const IslOut& o) {
    const int t = threadIdx.x, nl = blockDim.x;
    const int64_t per = (nr + nl - 1) / nl;
    const int64_t r0 = min((int64_t)t * per, nr), r1 = min(r0 + per, nr);
    constexpr int kCache = 8;
    const bool cached = per <= kCache;   // uniform
    uint32_t bits = 0;   // run j: bits 4j.. = map | keep(stale 0) << 2 | keep(stale 1) << 3
    uint32_t F = 0x2u;
    for (int64_t r = r0; r < r1; ++r) {
        const RunStat rs = run_stat<kAgent>(pk, ws, to, c, r);
        const uint32_t m = stale_map(rs);
        F = mcompose(m, F);
        if (cached)
            bits |= (m | ((uint32_t)filter(rs, 0u).keep << 2) | ((uint32_t)filter(rs, 1u).keep << 3))
                    << (4 * (r - r0));
    }
    const uint32_t stale0 = mapply(wg_scan_map(F, sm), 0u);   // atC = false at the chunk start (:268)
    uint32_t stale = stale0;
    int32_t nk = 0;
    if (cached) {
        for (int64_t j = 0; j < r1 - r0; ++j) {
            const uint32_t b = bits >> (4 * j);
            nk += (b >> (2 + stale)) & 1u;
            stale = mapply(b & 3u, stale);
        }
    } else {
        for (int64_t r = r0; r < r1; ++r) {
            const RunStat rs = run_stat<kAgent>(pk, ws, to, c, r);
            const Rec f = filter(rs, stale);
            kept[r] = f.keep ? (int32_t)stale : -1;
            nk += f.keep;
            stale = mapply(stale_map(rs), stale);
        }
    }
    int32_t nkt;
    int32_t rank = wg_scan_sum(nk, sk, nkt);
    // publish this chunk's count, then find the kept islands of the chunks before it
    if (t == 0)
        __hip_atomic_store(ws.flags + c, ((unsigned long long)o.epoch << 32) | (uint32_t)nkt,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t < 64) {
        const long long before = kept_before(ws, c, o.epoch, o.status);
        if (t == 0) *sbase = before;
    }
    __syncthreads();
    const int64_t base = *sbase + (o.base_in ? *o.base_in : 0);
    if (c == (int64_t)gridDim.x - 1 && t == 0) *o.count = base + nkt;
    const int64_t gchunk = o.first_chunk + c;
    const uint32_t cbase = (uint32_t)gchunk * (uint32_t)C;   // chunk*0x100000, Java int
    if (cached) {
        stale = stale0;
        for (int64_t j = 0; j < r1 - r0; ++j) {
            const uint32_t b = bits >> (4 * j);
            if ((b >> (2 + stale)) & 1u)
                put_island(o, run_stat<kAgent>(pk, ws, to, c, r0 + j), stale, base + rank++,
                           gchunk, cbase);
            stale = mapply(b & 3u, stale);
        }
    } else {
        for (int64_t r = r0; r < r1; ++r)
            if (kept[r] >= 0)
                put_island(o, run_stat<kAgent>(pk, ws, to, c, r), (uint32_t)(kept[r] & 1),
                           base + rank++, gchunk, cbase);
    }
}

// R: one chunk.  Tile offsets (exclusive scan of the tile totals, in blocks of kIT tiles;
// kept in LDS too for up to kToffLds tiles), then resolve_runs.
constexpr int kToffLds = 1024;
__global__ __launch_bounds__(kIT) void k_isl_resolve(const uint32_t* packed, int64_t C,
                                                    IslWs ws, IslOut o) {
    const int64_t c = blockIdx.x;
    const int t = threadIdx.x, nl = blockDim.x;
    const int64_t maxr = C / 2 + 1;
    const uint32_t* pk = packed + c * (C / 16);
    __shared__ Cnt5 s5[2][16];
    __shared__ uint32_t sm[16];
    __shared__ int32_t sk[16];
    __shared__ long long sbase;
    __shared__ Cnt5 s_to[kToffLds];
    const bool in_lds = ws.ntile <= kToffLds;
    Cnt5 carry{0, 0, 0, 0, 0};
    for (int64_t b = 0, it = 0; b < ws.ntile; b += nl, ++it) {
        const int64_t i = b + t;
        const Cnt5 v = i < ws.ntile ? ws.ttot[c * ws.ntile + i] : Cnt5{0, 0, 0, 0, 0};
        Cnt5 tot;
        const Cnt5 e = wg_scan5(v, s5[it & 1], tot);   // double-buffered: one barrier per block
        if (i < ws.ntile) {
            const Cnt5 oo = cadd(e, carry);
            if (in_lds) s_to[i] = oo;
            else ws.toff[c * ws.ntile + i] = oo;
        }
        carry = cadd(carry, tot);
    }
    if (!in_lds) __threadfence();   // read back past L1 below
    __syncthreads();
    // closed runs only: an island still open at the chunk end is dropped (:269-339)
    const int64_t nr = carry.cl;
    int32_t* kept = ws.kept + c * maxr;
    if (in_lds)
        resolve_runs<false>(pk, ws, s_to, c, C, nr, kept, sm, sk, &sbase, o);
    else
        resolve_runs<true>(pk, ws, ws.toff + c * ws.ntile, c, C, nr, kept, sm, sk, &sbase, o);
}

}  // namespace

size_t islands_ws_bytes(int64_t nchunks, int64_t chunk_len) {
    return carve_isl(nullptr, nchunks, chunk_len).bytes;
}

hipError_t launch_islands(const uint32_t* packed, const uint32_t* sign, int64_t nchunks,
                          int64_t chunk_len, int64_t first_chunk, void* wsp, size_t ws_bytes,
                          cpg_island* out, int64_t cap, int64_t* count, uint32_t* status,
                          hipStream_t s, unsigned long long* flags, const int64_t* base_in) {
    IslWs ws = carve_isl(wsp, nchunks, chunk_len);
    if (ws.bytes > ws_bytes || !flags) return hipErrorInvalidValue;
    ws.flags = flags;
    if (nchunks == 0)
        return base_in ? hipMemcpyAsync(count, base_in, sizeof(int64_t), hipMemcpyDeviceToDevice, s)
                       : hipMemsetAsync(count, 0, sizeof(int64_t), s);
    hipLaunchKernelGGL(k_isl_tile, dim3((unsigned)(nchunks * ws.ntile)), dim3(kTT), 0, s, packed,
                       sign, chunk_len, ws);
    // a fresh tag per call for the look-back flags (their own workspace slot: stale words are
    // earlier calls' flags, whose tags never match)
    const IslOut o{out, cap, count, base_in, first_chunk, lookback_epoch(), status};
    hipLaunchKernelGGL(k_isl_resolve, dim3((unsigned)nchunks), dim3(kIT), 0, s, packed,
                       chunk_len, ws, o);
    return hipGetLastError();
}

}  // namespace cpg
