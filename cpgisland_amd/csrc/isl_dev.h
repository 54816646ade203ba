// isl_dev.h — the island scan's word-parallel run boundaries (CpGIslandFinder.java:262-339),
// shared by the island tile kernel (k_islands.hip) and the Viterbi traceback (k_viterbi.hip),
// which emits the same tile records straight from the sign words it has just produced when
// one decode call runs both (cpg_decode_d).
//
// Per 32-position word: S = sign bits ('+' = 1), start = S & ~S_prev (:319-337), close =
// ~S & S_prev (:273-289; the '-' that ends the island), C / G base masks, CG = G & C_prev.
// A run boundary is written as a record with the tile-relative prefix counts at it; the
// per-chunk resolve kernel adds the tile offsets.

#pragma once

#include "cpg_internal.h"

namespace cpg {
namespace isl {

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

// kAgent: the record is read by another workgroup of the same kernel (fused decode): two
// agent-scope atomic stores, read back with ld_rec<true> after the chunk's done counter
template <bool kAgent>
__device__ __forceinline__ void st_rec(RunRec* p, const RunRec& v) {
    if constexpr (kAgent) {
        unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
        __hip_atomic_store(q, (unsigned long long)v.pos | ((unsigned long long)(uint32_t)v.c << 32),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(q + 1, (unsigned long long)(uint32_t)v.g | ((unsigned long long)(uint32_t)v.cg << 32),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        *p = v;
    }
}

// the run boundaries of word w as records; e = the prefix counts before the word (advanced)
template <bool kAgent = false>
__device__ __forceinline__ void emit_word(const WordMasks& q, int64_t w, Cnt5& e,
                                          RunRec* __restrict__ st, RunRec* __restrict__ cl) {
    for (uint32_t x = q.start; x; x &= x - 1) {
        const int b = __ffs(x) - 1;
        const uint32_t lo = (1u << b) - 1u;
        st_rec<kAgent>(st + e.st++, RunRec{(uint32_t)(w * 32 + b), e.c + (int32_t)__popc(q.C & lo),
                                          e.g + (int32_t)__popc(q.G & lo),
                                          e.cg + (int32_t)__popc(q.CG & (lo | (1u << b)))});
    }
    for (uint32_t x = q.close; x; x &= x - 1) {
        const int b = __ffs(x) - 1;
        const uint32_t lo = (1u << b) - 1u;
        st_rec<kAgent>(cl + e.cl++, RunRec{(uint32_t)(w * 32 + b), e.c + (int32_t)__popc(q.C & lo),
                                          e.g + (int32_t)__popc(q.G & lo),
                                          e.cg + (int32_t)__popc(q.CG & lo)});
    }
    e.c += __popc(q.C);
    e.g += __popc(q.G);
    e.cg += __popc(q.CG);
}

constexpr int64_t kInlineBaseMax = 4096;   // chunks: write_runs sums cres inline up to here
constexpr int kBaseBlock = 1024;            // chunks per k_isl_base workgroup

struct IslWs {
    RunRec* starts;     // per tile, cap_t records
    RunRec* closes;
    Cnt5* ttot;         // per tile: totals (kernel T)
    Cnt5* toff;         // per tile: exclusive prefix in its chunk (kernel R)
    int32_t* kept;      // per chunk, maxr: rank*2 | stale_in, or -1
    // the two-pass resolve (no look-back): per chunk {kept islands, closed runs}; per run its
    // kept[] word (stale_in, or -1: filtered out)
    int2* cres;
    // past kInlineBaseMax chunks (the split path): every chunk's first record, scanned once
    // from cres between the two passes (k_isl_base: per block of 1,024 chunks -> cbase and the
    // block totals bsum; k_isl_bscan: the block totals' exclusive scan in place), so that
    // write_runs reads its base instead of summing every chunk before it (O(chunks^2) work)
    long long* cbase;
    long long* bsum;
    int scanned;        // 1: write_runs reads cbase[c] + bsum[c / kBaseBlock]
    int64_t ntile;      // tiles per chunk
    int64_t cap_t;      // records per tile and kind
    size_t bytes;
};

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
// a run record: written by an earlier kernel (plain load) or by another workgroup of this
// one (agent-scope atomic loads: the fused decode's resolve, see st_rec)
template <bool kAgent>
__device__ __forceinline__ RunRec ld_rec(const RunRec* p) {
    if constexpr (kAgent) {
        const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
        const unsigned long long a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                                 b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return RunRec{(uint32_t)a, (int32_t)(a >> 32), (int32_t)(uint32_t)b, (int32_t)(b >> 32)};
    } else {
        return *p;
    }
}
template <bool kAgent, bool kAgentRec>
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
    RunRec x = ld_rec<kAgentRec>((kind ? ws.closes : ws.starts) + tile * ws.cap_t + (r - ok));
    x.c += oc;
    x.g += og;
    x.cg += ocg;
    return x;
}

struct RunStat {
    int32_t beg, end, len, C, G, CGin;
    uint32_t b0, b1, last;
};
template <bool kAgent, bool kAgentRec>
__device__ __forceinline__ RunStat run_stat(const uint32_t* pk, const IslWs& ws, const Cnt5* to,
                                            int64_t c, int64_t r) {
    const RunRec s = run_rec<kAgent, kAgentRec>(ws, to, c, r, 0),
                 e = run_rec<kAgent, kAgentRec>(ws, to, c, r, 1);
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
    int64_t nchunks;           // the last chunk writes the count
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

// The first pass of a chunk's resolve (k_isl_resolve, or the chunk's last traceback workgroup
// in a fused decode): the chunk's closed runs split over the lanes, stale-atC maps composed
// and scanned, filtered (:280-285); every run's kept[] word (stale_in, or -1: filtered out)
// and the chunk's {kept islands, closed runs} in ws.cres.  The records are placed by the
// second pass (write_runs, a later kernel) once every chunk's count is known: no workgroup
// waits for another.  With <= 8 runs per lane the map and both filter outcomes (stale 0 / 1)
// of each run stay in registers: one pass of loads.
template <bool kAgent, bool kAgentRec>
__device__ __forceinline__ void resolve_runs(const uint32_t* pk, const IslWs& ws, const Cnt5* to,
                                             int64_t c, int64_t nr, int32_t* kept, uint32_t* sm,
                                             int32_t* sk) {
    const int t = threadIdx.x, nl = blockDim.x;
    const int64_t per = (nr + nl - 1) / nl;
    const int64_t r0 = min((int64_t)t * per, nr), r1 = min(r0 + per, nr);
    constexpr int kCache = 8;
    const bool cached = per <= kCache;   // uniform
    uint32_t bits = 0;   // run j: bits 4j.. = map | keep(stale 0) << 2 | keep(stale 1) << 3
    uint32_t F = 0x2u;
    for (int64_t r = r0; r < r1; ++r) {
        const RunStat rs = run_stat<kAgent, kAgentRec>(pk, ws, to, c, r);
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
            const bool keep = (b >> (2 + stale)) & 1u;
            kept[r0 + j] = keep ? (int32_t)stale : -1;
            nk += keep;
            stale = mapply(b & 3u, stale);
        }
    } else {
        for (int64_t r = r0; r < r1; ++r) {
            const RunStat rs = run_stat<kAgent, kAgentRec>(pk, ws, to, c, r);
            const Rec f = filter(rs, stale);
            kept[r] = f.keep ? (int32_t)stale : -1;
            nk += f.keep;
            stale = mapply(stale_map(rs), stale);
        }
    }
    int32_t nkt;
    (void)wg_scan_sum(nk, sk, nkt);
    if (t == 0) ws.cres[c] = make_int2(nkt, (int32_t)nr);
}


// tile totals: plain, or agent-scope atomics when another workgroup of the same kernel reads
// them (fused decode)
template <bool kAgent>
__device__ __forceinline__ void st_cnt5(Cnt5* p, const Cnt5& v) {
    if constexpr (kAgent) {
        int32_t* q = reinterpret_cast<int32_t*>(p);
        const int32_t f[5] = {v.c, v.g, v.cg, v.st, v.cl};
#pragma unroll
        for (int i = 0; i < 5; ++i)
            __hip_atomic_store(q + i, f[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        *p = v;
    }
}
template <bool kAgent>
__device__ __forceinline__ Cnt5 ld_cnt5(const Cnt5* p) {
    if constexpr (kAgent) {
        const int32_t* q = reinterpret_cast<const int32_t*>(p);
        int32_t f[5];
#pragma unroll
        for (int i = 0; i < 5; ++i)
            f[i] = __hip_atomic_load(q + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return Cnt5{f[0], f[1], f[2], f[3], f[4]};
    } else {
        return *p;
    }
}

struct ResolveLds {
    Cnt5 s5[2][16];
    uint32_t sm[16];
    int32_t sk[16];
};

// The per-chunk resolve (kernel R, or the last traceback workgroup of a chunk in a fused
// decode): tile offsets (exclusive scan of the chunk's tile totals in blocks of blockDim.x
// tiles; kept in LDS `s_to` for up to kToff tiles for the runs' stats, and written to ws.toff
// for the second pass), then resolve_runs.  kAgentRec: the tile lists and totals were written
// by other workgroups of this kernel.
template <bool kAgentRec, int kToff>
__device__ __forceinline__ void resolve_chunk(const uint32_t* packed, int64_t C, const IslWs& ws,
                                              int64_t c, ResolveLds& L, Cnt5* s_to) {
    const int t = threadIdx.x, nl = blockDim.x;
    const int64_t maxr = C / 2 + 1;
    const uint32_t* pk = packed + c * (C / 16);
    const bool in_lds = ws.ntile <= kToff;
    Cnt5 carry{0, 0, 0, 0, 0};
    for (int64_t b = 0, it = 0; b < ws.ntile; b += nl, ++it) {
        const int64_t i = b + t;
        const Cnt5 v = i < ws.ntile ? ld_cnt5<kAgentRec>(ws.ttot + c * ws.ntile + i)
                                    : Cnt5{0, 0, 0, 0, 0};
        Cnt5 tot;
        const Cnt5 e = wg_scan5(v, L.s5[it & 1], tot);   // double-buffered: one barrier per block
        if (i < ws.ntile) {
            const Cnt5 oo = cadd(e, carry);
            if (in_lds) s_to[i] = oo;
            ws.toff[c * ws.ntile + i] = oo;   // (write_runs, the next kernel, reads them here)
        }
        carry = cadd(carry, tot);
    }
    if (!in_lds) __threadfence();   // read back past L1 below
    __syncthreads();
    // closed runs only: an island still open at the chunk end is dropped (:269-339)
    const int64_t nr = carry.cl;
    int32_t* kept = ws.kept + c * maxr;
    if (in_lds)
        resolve_runs<false, kAgentRec>(pk, ws, s_to, c, nr, kept, L.sm, L.sk);
    else
        resolve_runs<true, kAgentRec>(pk, ws, ws.toff + c * ws.ntile, c, nr, kept, L.sm, L.sk);
}

// The second pass of the two-pass resolve: chunk c's first record = the kept islands of the
// chunks before it (written by earlier kernels, so no workgroup waits for another: up to
// kInlineBaseMax chunks a workgroup sum over ws.cres, past it the scanned ws.cbase + ws.bsum),
// then every lane ranks and writes its kept islands from the runs' kept[] words (run stats
// re-read for the kept runs only).
__device__ __forceinline__ void write_runs(const uint32_t* packed, int64_t C, const IslWs& ws,
                                           const IslOut& o, int64_t c, long long* s_part,
                                           int32_t* sk) {
    const int t = threadIdx.x, nl = blockDim.x, lane = t & 63, wv = t >> 6;
    long long base = 0;
    if (ws.scanned) {
        base = ws.cbase[c] + ws.bsum[c / kBaseBlock];
    } else {
        long long before = 0;
        for (int64_t j = t; j < c; j += nl) before += ws.cres[j].x;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) before += __shfl_xor(before, off);
        if (lane == 0) s_part[wv] = before;
        __syncthreads();
        for (int w = 0; w < (nl >> 6); ++w) base += s_part[w];
    }
    base += o.base_in ? *o.base_in : 0;
    const int2 cr = ws.cres[c];
    if (c == o.nchunks - 1 && t == 0) *o.count = base + cr.x;
    if (cr.x == 0) return;
    const int64_t nr = cr.y;
    const int64_t per = (nr + nl - 1) / nl;
    const int64_t r0 = min((int64_t)t * per, nr), r1 = min(r0 + per, nr);
    const int32_t* kept = ws.kept + c * (C / 2 + 1);
    int32_t nk = 0;
    for (int64_t r = r0; r < r1; ++r) nk += kept[r] >= 0;
    int32_t nkt;
    const int32_t rank = wg_scan_sum(nk, sk, nkt);   // (uniform: every lane reaches it)
    if (!nk) return;
    const uint32_t* pk = packed + c * (C / 16);
    const Cnt5* to = ws.toff + c * ws.ntile;
    const int64_t gchunk = o.first_chunk + c;
    const uint32_t cbase = (uint32_t)gchunk * (uint32_t)C;   // chunk*0x100000, Java int
    int64_t dst = base + rank;
    for (int64_t r = r0; r < r1; ++r)
        if (kept[r] >= 0)
            put_island(o, run_stat<false, false>(pk, ws, to, c, r), (uint32_t)(kept[r] & 1),
                       dst++, gchunk, cbase);
}

}  // namespace isl

// a fused decode (cpg_decode_d): the traceback kernel's workgroups are the island tiles
// (256 blocks = 2,048 sign words each), and a chunk's last workgroup to finish (done counter,
// reset by it for the next call) resolves the chunk
struct IslFuse {
    isl::IslWs ws;
    isl::IslOut o;
    unsigned int* done;   // per chunk (WS_IDONE: zero between calls)
};

}  // namespace cpg
