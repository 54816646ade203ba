// k_islands.hip — island scan + filter (CpGIslandFinder.java:262-339) on gfx950.
//
// The reference walks each decoded 1 Mi chunk sequentially.  Its state is re-expressed as
// bit-parallel masks over 32-position words (sign bits + 2-bit packed bases):
//   start  = S & ~S_prev          (:319-337, inIsland false -> true)
//   close  = ~S & S_prev          (:273-289, the '-' that ends the island; end = i-1)
//   C, G   = base masks, CGm = G & C_prev (a G whose predecessor is a C)
// Island counts are differences of per-word prefix sums; CpG inside (beg, end] is exact
// from CGm.  The one serial quirk — `atC` is never cleared when an island closes (:325-331),
// so the first pair of an island can count a CpG against the previous island's last C — is
// a function stale_in -> stale_out per island (const 0 / const 1 / identity), resolved by a
// scan over the chunk's islands.  Islands still open at the chunk end are dropped (:269-339
// never closes them).  Coordinates and (cgCount*islandLen) use Java int arithmetic.
//
// Kernels: A1 (per 1024-word tile) tile totals; A3 (per tile) word prefixes + run
// boundaries, offset = sum of earlier tiles; B (per chunk) per-run stats, stale scan, filter,
// kept rank; D (per chunk) records at offset = kept islands of earlier chunks.

#include "cpg_internal.h"

namespace cpg {
namespace {

constexpr int kIT = 1024;

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

// the 4 sign words a lane owns (w0..w0+3), all loads vectorised; words >= nw read as 0
__device__ __forceinline__ void masks4(const uint32_t* __restrict__ pk,
                                       const uint32_t* __restrict__ sg, int64_t w0, int64_t nw,
                                       WordMasks (&m)[4]) {
    uint32_t S[4], P[8], sprev, pprev;
    if (w0 + 4 <= nw) {
        const uint4 s4 = *reinterpret_cast<const uint4*>(sg + w0);
        const uint4 p0 = *reinterpret_cast<const uint4*>(pk + 2 * w0);
        const uint4 p1 = *reinterpret_cast<const uint4*>(pk + 2 * w0 + 4);
        S[0] = s4.x; S[1] = s4.y; S[2] = s4.z; S[3] = s4.w;
        P[0] = p0.x; P[1] = p0.y; P[2] = p0.z; P[3] = p0.w;
        P[4] = p1.x; P[5] = p1.y; P[6] = p1.z; P[7] = p1.w;
    } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const bool in = w0 + i < nw;
            S[i] = in ? sg[w0 + i] : 0u;
            P[2 * i] = in ? pk[2 * (w0 + i)] : 0u;
            P[2 * i + 1] = in ? pk[2 * (w0 + i) + 1] : 0u;
        }
    }
    sprev = w0 > 0 ? sg[w0 - 1] : 0u;
    pprev = w0 > 0 ? pk[2 * w0 - 1] : 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        m[i] = masks_reg(S[i], i == 0 ? sprev : S[i - 1], P[2 * i], P[2 * i + 1],
                         i == 0 ? pprev : P[2 * i - 1]);
}

// masks of sign word w (positions 32w..32w+31) of a chunk; nw = words in the chunk
__device__ __forceinline__ WordMasks word_masks(const uint32_t* __restrict__ pk,
                                                const uint32_t* __restrict__ sg, int64_t w) {
    WordMasks m;
    const uint32_t S = sg[w];
    const uint32_t sprev = w > 0 ? (sg[w - 1] >> 31) : 0u;
    const uint32_t Sp = (S << 1) | sprev;
    m.S = S;
    m.start = S & ~Sp;
    m.close = ~S & Sp;
    const uint32_t w0 = pk[2 * w], w1 = pk[2 * w + 1];
    const uint32_t h0 = w0 >> 1, h1 = w1 >> 1;
    const uint32_t c = compact16(w0 & ~h0) | (compact16(w1 & ~h1) << 16);   // base == 1
    const uint32_t g = compact16(h0 & ~w0) | (compact16(h1 & ~w1) << 16);   // base == 2
    const uint32_t cprev = w > 0 ? ((pk[2 * w - 1] >> 30) == 1u) : 0u;
    m.C = c;
    m.G = g;
    m.CG = g & ((c << 1) | cprev);
    return m;
}

struct Cnt5 {
    int32_t c, g, cg, st, cl;
};

struct IslWs {
    int32_t* Cp;        // per word exclusive prefix (chunk-local)
    int32_t* Gp;
    int32_t* CGp;
    uint32_t* starts;   // per run
    uint32_t* closes;
    int32_t* kept;      // per run: rank*2 | stale_in, or -1
    int32_t* nruns;     // per chunk
    int32_t* ncloses;
    int64_t* nkept;
    void* tiles;        // Cnt5 per (chunk, tile)
    size_t bytes;
};

IslWs carve_isl(void* base, int64_t nchunks, int64_t C) {
    const int64_t nw = (C + 31) / 32, maxr = C / 2 + 1;
    char* p = static_cast<char*>(base);
    size_t o = 0;
    auto take = [&](size_t b) {
        o = (o + 255) & ~size_t(255);
        char* r = p ? p + o : nullptr;
        o += b;
        return r;
    };
    IslWs w;
    w.Cp = (int32_t*)take(nchunks * nw * 4);
    w.Gp = (int32_t*)take(nchunks * nw * 4);
    w.CGp = (int32_t*)take(nchunks * nw * 4);
    w.starts = (uint32_t*)take(nchunks * maxr * 4);
    w.closes = (uint32_t*)take(nchunks * maxr * 4);
    w.kept = (int32_t*)take(nchunks * maxr * 4);
    w.nruns = (int32_t*)take(nchunks * 4);
    w.ncloses = (int32_t*)take(nchunks * 4);
    w.nkept = (int64_t*)take(nchunks * 8);
    w.tiles = take(nchunks * ((nw + 1023) / 1024) * 20 + 16);
    w.bytes = o + 256;
    return w;
}


// Pass A, tiled: a tile = 1024 sign words (32,768 positions) of one chunk, 4 words per lane.
constexpr int kTileW = 1024;
constexpr int kAT = 256;

__device__ __forceinline__ Cnt5 cnt_of(const WordMasks& m) {
    return Cnt5{(int32_t)__popc(m.C), (int32_t)__popc(m.G), (int32_t)__popc(m.CG),
                (int32_t)__popc(m.start), (int32_t)__popc(m.close)};
}
__device__ __forceinline__ Cnt5 cadd(Cnt5 a, const Cnt5& b) {
    a.c += b.c; a.g += b.g; a.cg += b.cg; a.st += b.st; a.cl += b.cl;
    return a;
}

// block-wide exclusive scan of one Cnt5 per lane; returns (exclusive, total)
__device__ __forceinline__ Cnt5 block_scan(Cnt5 v, Cnt5* sb, Cnt5& total) {
    const int t = threadIdx.x;
    sb[t] = v;
    __syncthreads();
    for (int off = 1; off < kAT; off <<= 1) {
        Cnt5 x = sb[t];
        if (t >= off) x = cadd(x, sb[t - off]);
        __syncthreads();
        sb[t] = x;
        __syncthreads();
    }
    total = sb[kAT - 1];
    const Cnt5 e = t > 0 ? sb[t - 1] : Cnt5{0, 0, 0, 0, 0};
    __syncthreads();
    return e;
}

// A1: tile totals
__global__ __launch_bounds__(kAT) void k_isl_a1(const uint32_t* packed, const uint32_t* sign,
                                               int64_t C, int ntiles, Cnt5* __restrict__ tiles) {
    const int64_t c = blockIdx.x / ntiles;
    const int tile = blockIdx.x - (int)c * ntiles;
    const int64_t nw = C / 32;
    const uint32_t* pk = packed + c * (C / 16);
    const uint32_t* sg = sign + c * nw;
    Cnt5 s{0, 0, 0, 0, 0};
    const int64_t w0 = (int64_t)tile * kTileW + threadIdx.x * 4;
    WordMasks m[4];
    if (w0 < nw) masks4(pk, sg, w0, nw, m);
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (w0 + i < nw) s = cadd(s, cnt_of(m[i]));
    __shared__ Cnt5 sb[kAT];
    Cnt5 tot;
    block_scan(s, sb, tot);
    if (threadIdx.x == 0) tiles[blockIdx.x] = tot;
}

// A3: word prefixes and run boundaries
__global__ __launch_bounds__(kAT) void k_isl_a3(const uint32_t* packed, const uint32_t* sign,
                                               int64_t C, int ntiles,
                                               const Cnt5* __restrict__ tiles, IslWs ws) {
    const int64_t c = blockIdx.x / ntiles;
    const int tile = blockIdx.x - (int)c * ntiles;
    const int64_t nw = C / 32, maxr = C / 2 + 1;
    const uint32_t* pk = packed + c * (C / 16);
    const uint32_t* sg = sign + c * nw;
    const int64_t w0 = (int64_t)tile * kTileW + threadIdx.x * 4;
    WordMasks m[4];
    Cnt5 s{0, 0, 0, 0, 0};
    if (w0 < nw) masks4(pk, sg, w0, nw, m);
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (w0 + i < nw) s = cadd(s, cnt_of(m[i]));
    __shared__ Cnt5 sb[kAT];
    // this tile's offset in the chunk: the sum of the earlier tiles' A1 totals
    Cnt5 before{0, 0, 0, 0, 0}, off, tot;
    for (int i = threadIdx.x; i < tile; i += kAT) before = cadd(before, tiles[c * ntiles + i]);
    block_scan(before, sb, off);
    Cnt5 e = cadd(block_scan(s, sb, tot), off);
    if (tile == ntiles - 1 && threadIdx.x == 0) {   // chunk totals: runs opened / closed
        ws.nruns[c] = off.st + tot.st;
        ws.ncloses[c] = off.cl + tot.cl;
    }
    int32_t* Cp = ws.Cp + c * nw;
    int32_t* Gp = ws.Gp + c * nw;
    int32_t* CGp = ws.CGp + c * nw;
    uint32_t* st = ws.starts + c * maxr;
    uint32_t* cl = ws.closes + c * maxr;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int64_t w = w0 + i;
        if (w >= nw) break;
        Cp[w] = e.c;
        Gp[w] = e.g;
        CGp[w] = e.cg;
        e.c += __popc(m[i].C);
        e.g += __popc(m[i].G);
        e.cg += __popc(m[i].CG);
        for (uint32_t x = m[i].start; x; x &= x - 1) st[e.st++] = (uint32_t)(w * 32 + __ffs(x) - 1);
        for (uint32_t x = m[i].close; x; x &= x - 1) cl[e.cl++] = (uint32_t)(w * 32 + __ffs(x) - 1);
    }
}

__device__ __forceinline__ uint32_t isl_base(const uint32_t* pk, int64_t pos) {
    return (pk[pos >> 4] >> ((pos & 15) * 2)) & 3u;
}
// prefix count of a mask kind (0 C, 1 G, 2 CG) over chunk positions [0, pos)
__device__ __forceinline__ int32_t pref(const uint32_t* pk, const uint32_t* sg, const int32_t* P,
                                        int kind, int64_t pos, int64_t nw) {
    const int64_t w = pos >> 5;
    if (w >= nw) return P[nw - 1] + __popc(kind == 0 ? word_masks(pk, sg, nw - 1).C
                                           : kind == 1 ? word_masks(pk, sg, nw - 1).G
                                                       : word_masks(pk, sg, nw - 1).CG);
    const WordMasks m = word_masks(pk, sg, w);
    const uint32_t x = kind == 0 ? m.C : kind == 1 ? m.G : m.CG;
    const uint32_t lowmask = (pos & 31) ? ((1u << (pos & 31)) - 1u) : 0u;
    return P[w] + __popc(x & lowmask);
}

struct RunStat {
    int32_t beg, end, len, C, G, CGin;
    uint32_t b0, b1, last;
};
__device__ __forceinline__ RunStat run_stat(const uint32_t* pk, const uint32_t* sg, IslWs ws,
                                            int64_t c, int64_t nw, uint32_t beg, uint32_t close) {
    RunStat r;
    r.beg = (int32_t)beg;
    r.end = (int32_t)close - 1;
    r.len = (int32_t)(close - beg);
    const int32_t* Cp = ws.Cp + c * nw;
    const int32_t* Gp = ws.Gp + c * nw;
    const int32_t* CGp = ws.CGp + c * nw;
    r.C = pref(pk, sg, Cp, 0, close, nw) - pref(pk, sg, Cp, 0, beg, nw);
    r.G = pref(pk, sg, Gp, 1, close, nw) - pref(pk, sg, Gp, 1, beg, nw);
    r.CGin = r.len >= 2 ? pref(pk, sg, CGp, 2, close, nw) - pref(pk, sg, CGp, 2, beg + 1, nw) : 0;
    r.b0 = isl_base(pk, beg);
    r.b1 = r.len >= 2 ? isl_base(pk, beg + 1) : 0u;
    r.last = isl_base(pk, close - 1);
    return r;
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

__global__ __launch_bounds__(kIT) void k_isl_b(const uint32_t* packed, const uint32_t* sign,
                                               int64_t C, IslWs ws) {
    const int64_t c = blockIdx.x;
    const int t = threadIdx.x;
    const int64_t nw = C / 32, maxr = C / 2 + 1;
    const uint32_t* pk = packed + c * (C / 16);
    const uint32_t* sg = sign + c * nw;
    const int64_t nr = ws.ncloses[c];   // closed runs only; an open last run is dropped
    const uint32_t* st = ws.starts + c * maxr;
    const uint32_t* cl = ws.closes + c * maxr;
    int32_t* kept = ws.kept + c * maxr;
    const int64_t per = (nr + kIT - 1) / kIT;
    const int64_t r0 = min((int64_t)t * per, nr), r1 = min(r0 + per, nr);
    uint32_t F = 0x2u;
    for (int64_t r = r0; r < r1; ++r) F = mcompose(stale_map(run_stat(pk, sg, ws, c, nw, st[r], cl[r])), F);
    __shared__ uint32_t sF[kIT];
    __shared__ int32_t sK[kIT];
    sF[t] = F;
    __syncthreads();
    for (int off = 1; off < kIT; off <<= 1) {
        uint32_t x = sF[t];
        if (t >= off) x = mcompose(x, sF[t - off]);
        __syncthreads();
        sF[t] = x;
        __syncthreads();
    }
    uint32_t stale = t > 0 ? mapply(sF[t - 1], 0u) : 0u;   // atC = false at chunk start (:268)
    int32_t nk = 0;
    for (int64_t r = r0; r < r1; ++r) {
        const RunStat rs = run_stat(pk, sg, ws, c, nw, st[r], cl[r]);
        const Rec o = filter(rs, stale);
        kept[r] = o.keep ? (int32_t)(stale) : -1;   // rank added below
#ifdef CPG_DEBUG_ISL
        if (c == 0 && r < 8)
            printf("run %d beg %d end %d len %d C %d G %d CGin %d b0 %u b1 %u last %u cg %f oe %f keep %d\n",
                   (int)r, rs.beg, rs.end, rs.len, rs.C, rs.G, rs.CGin, rs.b0, rs.b1, rs.last, o.cg, o.oe, (int)o.keep);
#endif
        nk += o.keep;
        stale = mapply(stale_map(rs), stale);
    }
    sK[t] = nk;
    __syncthreads();
    for (int off = 1; off < kIT; off <<= 1) {
        int32_t x = sK[t];
        if (t >= off) x += sK[t - off];
        __syncthreads();
        sK[t] = x;
        __syncthreads();
    }
    int32_t rank = t > 0 ? sK[t - 1] : 0;
    for (int64_t r = r0; r < r1; ++r)
        if (kept[r] >= 0) kept[r] |= (rank++) << 1;
    if (t == kIT - 1) ws.nkept[c] = sK[kIT - 1];
}

__global__ __launch_bounds__(kIT) void k_isl_d(const uint32_t* packed, const uint32_t* sign,
                                               int64_t C, int64_t first_chunk, IslWs ws,
                                               cpg_island* out, int64_t cap, int64_t* count,
                                               const int64_t* base_in) {
    const int64_t c = blockIdx.x;
    // the chunk's first record: kept islands of all earlier chunks (fixed-order sum)
    __shared__ int64_t sb[kIT];
    {
        int64_t a = 0;
        for (int64_t i = threadIdx.x; i < c; i += kIT) a += ws.nkept[i];
        sb[threadIdx.x] = a;
        __syncthreads();
        for (int o = kIT / 2; o > 0; o >>= 1) {
            if ((int)threadIdx.x < o) sb[threadIdx.x] += sb[threadIdx.x + o];
            __syncthreads();
        }
    }
    // append mode (streamed windows): records continue after *base_in earlier ones and
    // *count receives the running total
    const int64_t base = sb[0] + (base_in ? *base_in : 0);
    if (c == (int64_t)gridDim.x - 1 && threadIdx.x == 0) *count = base + ws.nkept[c];
    const int64_t nw = C / 32, maxr = C / 2 + 1;
    const uint32_t* pk = packed + c * (C / 16);
    const uint32_t* sg = sign + c * nw;
    const int64_t nr = ws.ncloses[c];
    const uint32_t* st = ws.starts + c * maxr;
    const uint32_t* cl = ws.closes + c * maxr;
    const int32_t* kept = ws.kept + c * maxr;
    const int64_t gchunk = first_chunk + c;
    const uint32_t cbase = (uint32_t)gchunk * (uint32_t)C;   // chunk*0x100000, Java int
    for (int64_t r = threadIdx.x; r < nr; r += kIT) {
        const int32_t k = kept[r];
        if (k < 0) continue;
        const int64_t dst = base + (k >> 1);
        if (dst >= cap) continue;
        const RunStat rs = run_stat(pk, sg, ws, c, nw, st[r], cl[r]);
        const Rec o = filter(rs, (uint32_t)(k & 1));
        cpg_island isl;
        isl.beg1 = (int32_t)((uint32_t)rs.beg + cbase + 1u);          // :287
        isl.end1 = (int32_t)((uint32_t)rs.end + cbase + 1u);
        isl.len = rs.len;
        isl.chunk = (int32_t)gchunk;
        isl.cg = o.cg;
        isl.oe = o.oe;
        out[dst] = isl;
    }
}

}  // namespace

size_t islands_ws_bytes(int64_t nchunks, int64_t chunk_len) {
    return carve_isl(nullptr, nchunks, chunk_len).bytes;
}

hipError_t launch_islands(const uint32_t* packed, const uint32_t* sign, int64_t nchunks,
                          int64_t chunk_len, int64_t first_chunk, void* wsp, size_t ws_bytes,
                          cpg_island* out, int64_t cap, int64_t* count, hipStream_t s,
                          const int64_t* base_in) {
    IslWs ws = carve_isl(wsp, nchunks, chunk_len);
    if (ws.bytes > ws_bytes) return hipErrorInvalidValue;
    if (nchunks == 0)
        return base_in ? hipMemcpyAsync(count, base_in, sizeof(int64_t), hipMemcpyDeviceToDevice, s)
                       : hipMemsetAsync(count, 0, sizeof(int64_t), s);
    const int ntiles = (int)((chunk_len / 32 + kTileW - 1) / kTileW);
    Cnt5* tiles = static_cast<Cnt5*>(ws.tiles);
    hipLaunchKernelGGL(k_isl_a1, dim3((unsigned)(nchunks * ntiles)), dim3(kAT), 0, s, packed,
                       sign, chunk_len, ntiles, tiles);
    hipLaunchKernelGGL(k_isl_a3, dim3((unsigned)(nchunks * ntiles)), dim3(kAT), 0, s, packed,
                       sign, chunk_len, ntiles, tiles, ws);
    hipLaunchKernelGGL(k_isl_b, dim3((unsigned)nchunks), dim3(kIT), 0, s, packed, sign,
                       chunk_len, ws);
    hipLaunchKernelGGL(k_isl_d, dim3((unsigned)nchunks), dim3(kIT), 0, s, packed, sign,
                       chunk_len, first_chunk, ws, out, cap, count, base_in);
    return hipGetLastError();
}

}  // namespace cpg
