// k_ingest.hip — device-side ASCII ingest with the reference's quirks (SURVEY.md §8(f) 1,
// Appendix A.1) on gfx950: CpGIslandFinder.java:112-145 (training reader) and :238-259
// (decode reader) as ONE streaming pass over the raw text in HBM.
//
// The reference reads the file character by character: A/a C/c G/g T/t become 0..3
// (:114-128, :240-254), every other byte is skipped, and after EVERY byte the Java int
// `count` of bases read is tested against the chunk cadence:
//   count != 0 && count % chunk == 0  ->  the pending list (exactly `chunk` bases) is a
//   chunk (training: a SequenceFile record, :130-141; decode: one Viterbi call, :256-259).
// A non-ACGT byte read while `count` still sits on the multiple finds the list EMPTY: the
// training reader writes an extra all-A (zero-padded) chunk, the decode reader throws
// (observedSequence.get(i) on an empty list).  Those bytes are the "quirk" bytes here.
//
// Per 32 KiB tile (one 256-lane workgroup, coalesced 16-B loads):
//   * SWAR byte classification: fold case (x & 0xDF), code = ((f>>1)^(f>>2)) & 3 gives
//     A,C,G,T -> 0,1,2,3, and a byte is valid iff f equals perm({A,C,G,T}, code)
//     (v_perm_b32 as a 4-entry byte table);
//   * per-lane compaction of the 2-bit codes of its 16 bytes (one shift-merge per invalid
//     byte: usually none or one), a wave/tile scan of the valid counts, and the codes
//     assembled as a bit array in LDS;
//   * decoupled look-back (Merrill & Garland) over the tiles for the number of valid
//     bases before the tile; the quirk bytes of the tile follow from it (a tile holds fewer
//     than `chunk` bases, so at most one residue point l* falls inside it) and, for the
//     training reader with quirks, a second look-back chains the extra-chunk counts;
//   * the tile's bases are written as packed words at their final positions (a quirk gap of
//     q * chunk all-A bases inside the tile splits them in two runs); full words are plain
//     stores, the partial words at run edges integer atomicOr into the zeroed output.
// The look-back descriptors are 8-byte {flag, value} granules stored and polled with
// agent-scope relaxed atomics (the data is the flag); every spin is bounded.
// `count` is a Java int (:107, :236): at 2^32 bases it wraps to 0 and the test is skipped, so
// the list keeps its chunk.  At the next multiple the training reader's chunk vector gets two
// chunks (DenseVector.set(0x10000) throws at :134: a crash at that valid byte), the decode
// reader decodes the held chunk and clear() drops the 2^20 bases read after the wrap (a
// dropped window: the tile's bases are written as two runs around it, later bases shifted).
// Algorithmic bytes: 1 B/byte read + 0.25 B/base written.

#include "cpg_internal.h"


namespace cpg {
namespace {

constexpr int kIT = 256;                       // lanes per tile
constexpr int kIRows = 8;                      // rows of 1 KiB per wave (8: 32 KiB tiles)
constexpr int kTileBytes = kIT * 16 * kIRows;  // <= 32 KiB: one residue point per tile
static_assert(kIRows % 2 == 0 && kTileBytes <= 32768, "2..8 rows of 1 KiB per wave");
constexpr int kTileWords = kTileBytes / 16;    // packed words for a tile of valid bytes
constexpr unsigned long long kFlagAgg = 1ull << 62, kFlagInc = 2ull << 62;
constexpr unsigned long long kValMask = (1ull << 62) - 1;
constexpr uint64_t kWrap = 1ull << 32;         // Java int `count` wraps to 0 here

typedef unsigned long long __attribute__((address_space(1))) gu64;

struct IngestWs {
    unsigned long long* stV;   // [ntiles] look-back granules: valid bases
    unsigned long long* stQ;   // [ntiles] look-back granules: extra all-A chunks
    unsigned int* ticket;      // dynamic tile id
    unsigned int* crash_tile;  // first tile with a crash (0xFFFFFFFF: none)
    unsigned int* timeout;     // a bounded spin gave up
    long long* crash_k;        // [ntiles] crash byte index of a crashing tile
    long long* crash_c;        // [ntiles] bases committed before it
    long long* tot;            // [2] valid bases, extra chunks (written by the last tile)
};

__device__ __forceinline__ void gstore(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long gload(const unsigned long long* p) {
    return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Exclusive prefix of the granules before `tile` (one wave, uniform).  Each pass reads a
// window of 64 * kLbw granules (lane l, slot k: distance 64 k + l); it waits only for the
// granules up to the nearest inclusive one.  Wide windows matter: every tile of a dispatch
// round publishes its aggregate at about the same time, so the nearest inclusive granule is
// typically a round (~2,000 tiles) back, and each pass costs one device-scope round trip.
constexpr int kLbw = 1;   // wider windows were slower (polling traffic)
__device__ unsigned long long lookback(const unsigned long long* st, long long tile, int lane,
                                       unsigned int* timeout) {
    unsigned long long excl = 0;
    long long j = tile - 1;
    const unsigned long long t0 = wall_clock64();
    while (j >= 0) {
        unsigned long long s[kLbw];
        int first;   // distance of the nearest inclusive granule in the window (or last)
        for (;;) {
#pragma unroll
            for (int k = 0; k < kLbw; ++k) {
                const long long idx = j - 64 * k - lane;
                s[k] = idx >= 0 ? gload(st + idx) : kFlagInc;
            }
            first = 64 * kLbw - 1;
            bool ok = true;
#pragma unroll
            for (int k = kLbw - 1; k >= 0; --k) {
                const unsigned long long inc = __ballot((s[k] >> 62) == 2);
                if (inc) first = 64 * k + __ffsll((long long)inc) - 1;
            }
#pragma unroll
            for (int k = 0; k < kLbw; ++k) {
                const int d = 64 * k + lane;
                ok = ok && (d > first || (s[k] >> 62) != 0);
            }
            if (__all(ok)) break;
            // bounded: 0.5 s of wall clock (100 MHz) -> give up, flag the call
            if (wall_clock64() - t0 > 50000000ull) {
                if (lane == 0) atomicOr(timeout, 1u);
                return excl;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        unsigned long long v = 0;
#pragma unroll
        for (int k = 0; k < kLbw; ++k)
            if (64 * k + lane <= first) v += s[k] & kValMask;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
        excl += v;
        bool found = false;
#pragma unroll
        for (int k = 0; k < kLbw; ++k) found = found || (64 * k + lane == first && (s[k] >> 62) == 2);
        if (__ballot(found)) break;
        j -= 64 * kLbw;
    }
    return excl;
}

// 16 bytes -> 16-bit valid mask, the 16 2-bit codes in place, and the bytes' validity
__device__ __forceinline__ void classify(uint4 q, uint32_t& vmask, uint32_t& codes) {
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
    vmask = 0u;
    codes = 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t f = w[i] & 0xDFDFDFDFu;
        const uint32_t c = ((f >> 1) ^ (f >> 2)) & 0x03030303u;
        const uint32_t e = __builtin_amdgcn_perm(0u, 0x54474341u, c);   // 'A' 'C' 'G' 'T'
        const uint32_t d = f ^ e;                                         // 0 byte: valid
        const uint32_t z = ~(((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d) & 0x80808080u;
        const uint32_t nib = ((z >> 7) * 0x10204080u) >> 28;              // bits 7,15,23,31
        uint32_t p = c | (c >> 6);
        p = (p | (p >> 12)) & 0xFFu;                                      // 4 codes, 8 bits
        vmask |= nib << (4 * i);
        codes |= p << (8 * i);
    }
}

// chunks committed by the firings at the multiples of C in (c0, G] (G, c0: unwrapped counts):
// every multiple fires except the wraps k 2^32 (count == 0), and each firing commits one chunk
// (past a wrap, the held one)
__device__ __forceinline__ long long commits(unsigned long long G, unsigned long long c0,
                                             long long C) {
    return (long long)(G / (unsigned long long)C) - (long long)(G >> 32) -
           ((long long)(c0 / (unsigned long long)C) - (long long)(c0 >> 32));
}

struct IngestArgs {
    const uint8_t* txt;
    int64_t n;
    int64_t chunk;
    int64_t cap;        // output capacity in bases
    int64_t ntiles;
    int mode;           // 0 training, 1 decode
    int quirks;
    uint32_t* out;
    unsigned long long c0;   // Java count before the first byte (a chunk multiple < 2^32)
};

__global__ __launch_bounds__(kIT) void k_ingest(IngestArgs a, IngestWs ws) {
    __shared__ uint32_t sb[kTileWords + 2];   // code bit array (+1 guard word each side)
    __shared__ uint32_t srow[4][kIRows];          // per wave per row valid counts
    __shared__ long long s_tile;
    __shared__ unsigned long long s_vex, s_qp;
    __shared__ int s_q;
    __shared__ long long s_qmin;                  // first quirk byte of the tile
    __shared__ long long s_wrapk;                 // byte of the wrap crash (if here)
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (t == 0) {
        // tile id = blockIdx: workgroups are dispatched in increasing order, so every
        // predecessor a tile waits on is resident or done (a global ticket counter measured
        // ~4x slower: one device-scope atomic per tile on one address)
        s_tile = (long long)blockIdx.x;
        s_q = 0;
        s_qmin = 0x7FFFFFFFFFFFFFFFll;
        s_wrapk = -1;
    }
    for (int i = t; i < kTileWords + 2; i += kIT) sb[i] = 0u;
    __syncthreads();
    const long long tile = s_tile;
    const long long base = tile * (long long)kTileBytes;
    uint32_t vm[kIRows], cw[kIRows], real[kIRows];
#pragma unroll
    for (int r = 0; r < kIRows; ++r) {
        const long long off = base + wv * (kIRows * 1024) + r * 1024 + lane * 16;
        uint4 q = make_uint4(0u, 0u, 0u, 0u);
        real[r] = 0xFFFFu;
        if (off + 16 <= a.n) {
            q = *reinterpret_cast<const uint4*>(a.txt + off);
        } else {
            uint32_t b[4] = {0u, 0u, 0u, 0u};
            for (int k = 0; k < 16; ++k)
                if (off + k < a.n) b[k >> 2] |= (uint32_t)a.txt[off + k] << (8 * (k & 3));
            q = make_uint4(b[0], b[1], b[2], b[3]);
            const long long left = a.n - off;
            real[r] = left <= 0 ? 0u : (left >= 16 ? 0xFFFFu : ((1u << left) - 1u));
        }
        classify(q, vm[r], cw[r]);
        vm[r] &= real[r];
    }
    // per-lane compaction: drop the fields of invalid bytes, highest first
    uint32_t cnt[kIRows];
#pragma unroll
    for (int r = 0; r < kIRows; ++r) {
        uint32_t inv = ~vm[r] & 0xFFFFu, u = cw[r];
        while (inv) {
            const int k = 31 - __builtin_clz(inv);
            const uint32_t lo = k ? (0xFFFFFFFFu >> (32 - 2 * k)) : 0u;
            u = (u & lo) | ((u >> 2) & ~lo);
            inv &= ~(1u << k);
        }
        cnt[r] = __builtin_popcount(vm[r]);
        cw[r] = cnt[r] == 16 ? u : (u & ((1u << (2 * cnt[r])) - 1u));
    }
    // scans: two rows packed per 32-bit word (counts <= 1024 per row per wave)
    uint32_t xs[kIRows / 2];
#pragma unroll
    for (int h = 0; h < kIRows / 2; ++h) xs[h] = cnt[2 * h] | (cnt[2 * h + 1] << 16);
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
#pragma unroll
        for (int h = 0; h < kIRows / 2; ++h) {
            const uint32_t y = __shfl_up(xs[h], off);
            if (lane >= off) xs[h] += y;
        }
    }
    if (lane == 63) {
#pragma unroll
        for (int h = 0; h < kIRows / 2; ++h) {
            srow[wv][2 * h] = xs[h] & 0xFFFFu;
            srow[wv][2 * h + 1] = xs[h] >> 16;
        }
    }
    __syncthreads();
    uint32_t o[kIRows];   // tile-local index of the lane's first valid byte in each row
    uint32_t agg = 0;
    {
        uint32_t before = 0;
        for (int w = 0; w < 4; ++w)
#pragma unroll
            for (int r = 0; r < kIRows; ++r) {
                if (w == wv) {
                    const uint32_t incl = (r & 1) ? (xs[r >> 1] >> 16) : (xs[r >> 1] & 0xFFFFu);
                    o[r] = before + incl - cnt[r];
                }
                before += srow[w][r];
            }
        agg = before;
    }
    // codes -> LDS bit array (guard word at sb[0])
#pragma unroll
    for (int r = 0; r < kIRows; ++r) {
        if (!cnt[r]) continue;
        const uint32_t bit = 2 * o[r], wi = 1 + (bit >> 5), sh = bit & 31;
        atomicOr(&sb[wi], cw[r] << sh);
        if (sh && sh + 2 * cnt[r] > 32) atomicOr(&sb[wi + 1], cw[r] >> (32 - sh));
    }
    // look-back 1: valid bases before this tile
    if (wv == 0) {
        unsigned long long vex = 0;
        if (tile == 0) {
            if (lane == 0) gstore(ws.stV, kFlagInc | agg);
        } else {
            if (lane == 0) gstore(ws.stV + tile, kFlagAgg | agg);
            vex = lookback(ws.stV, tile, lane, ws.timeout);
            if (lane == 0) gstore(ws.stV + tile, kFlagInc | ((vex + agg) & kValMask));
        }
        if (lane == 0) s_vex = vex;
    }
    __syncthreads();
    const unsigned long long vex = s_vex;
    const long long C = a.chunk;
    // residue point: local index l* with (vex + l*) % chunk == 0, l* <= agg
    const long long ls = (C - (long long)(vex % (unsigned long long)C)) % C;   // c0 % C == 0
    const unsigned long long gq = a.c0 + vex + (unsigned long long)ls;   // count at the quirk bytes
    const bool qlive = a.quirks && ls <= (long long)agg && gq != 0 && (gq % kWrap) != 0;
    if (qlive) {
#pragma unroll
        for (int r = 0; r < kIRows; ++r) {
            const uint32_t inv = ~vm[r] & real[r] & 0xFFFFu;
            if (!inv || (long long)o[r] > ls || (long long)(o[r] + cnt[r]) < ls) continue;
            int q = 0;
            long long kmin = 0x7FFFFFFFFFFFFFFFll;
            uint32_t before = o[r];
            for (int k = 0; k < 16; ++k) {
                if ((inv >> k) & 1u) {
                    if ((long long)before == ls) {
                        ++q;
                        const long long kb = base + wv * (kIRows * 1024) + r * 1024 + lane * 16 + k;
                        kmin = kb < kmin ? kb : kmin;
                    }
                } else if ((vm[r] >> k) & 1u) {
                    ++before;
                }
            }
            if (q) {
                atomicAdd(&s_q, q);
                atomicMin(&s_qmin, kmin);
            }
        }
    }
    // the training reader's crash past a count wrap: the valid byte that brings the count to
    // W + chunk (W = 2^32, the first wrap after c0: the stream ends there)
    if (a.mode == 0) {
        const unsigned long long jc = kWrap + (unsigned long long)C - 1ull - a.c0;  // its index
        if (vex <= jc && jc < vex + agg) {
            const uint32_t jw = (uint32_t)(jc - vex);
#pragma unroll
            for (int r = 0; r < kIRows; ++r) {
                if (jw < o[r] || jw >= o[r] + cnt[r]) continue;
                uint32_t m = vm[r];
                for (uint32_t s = o[r]; s < jw; ++s) m &= m - 1;   // drop lower valid bytes
                s_wrapk = base + wv * (kIRows * 1024) + r * 1024 + lane * 16 + (__builtin_ffs(m) - 1);
            }
        }
    }
    __syncthreads();
    const int qt = s_q;
    // look-back 2 (training reader with quirks): extra chunks before this tile
    const bool qchain = a.quirks && a.mode == 0;
    if (qchain) {
        if (wv == 0) {
            unsigned long long qp = 0;
            if (tile == 0) {
                if (lane == 0) gstore(ws.stQ, kFlagInc | (unsigned)qt);
            } else {
                if (lane == 0) gstore(ws.stQ + tile, kFlagAgg | (unsigned)qt);
                qp = lookback(ws.stQ, tile, lane, ws.timeout);
                if (lane == 0) gstore(ws.stQ + tile, kFlagInc | (qp + (unsigned)qt));
            }
            if (lane == 0) s_qp = qp;
        }
        __syncthreads();
    } else if (t == 0) {
        s_qp = 0;
    }
    if (!qchain) __syncthreads();
    const unsigned long long qp = s_qp;
    if (t == 0) {
        // crashes: decode reader at a quirk byte; either reader at the count wrap
        long long ck = -1, cc = 0;
        if (a.mode == 1 && qt > 0) {
            ck = s_qmin;
            cc = commits(gq, a.c0, C) * C;   // the chunks committed before it
        }
        if (s_wrapk >= 0 && (ck < 0 || s_wrapk < ck)) {
            ck = s_wrapk;
            cc = (commits(kWrap, a.c0, C) + (long long)(qchain ? qp : 0)) * C;
        }
        if (ck >= 0) {
            ws.crash_k[tile] = ck;
            ws.crash_c[tile] = cc;
            __threadfence();
            atomicMin(ws.crash_tile, (unsigned)tile);
        }
        if (tile == a.ntiles - 1) {
            ws.tot[0] = (long long)(vex + agg);
            ws.tot[1] = (long long)(qp + (qchain ? (unsigned)qt : 0u));
        }
    }
    // write the tile's bases as two runs (local start, length, output position): with a quirk
    // gap (training reader) run A = local [0, min(agg, ls)) at P, run B = local [ls, agg) at
    // P + ls + qt * chunk; past a count wrap (decode reader) the bases of the dropped window
    // (count in (W, W + chunk], W = k 2^32) are skipped and every later base moves down a chunk
    const long long P = (long long)vex + (long long)qp * C;
    long long sA = 0, lenA = (long long)agg, gA = P, sB = 0, lenB = 0, gB = 0;
    if (qchain && qt > 0) {
        lenA = ls < (long long)agg ? ls : (long long)agg;
        sB = lenA;
        lenB = (long long)agg - lenA;
        gB = P + ls + (long long)qt * C;
    } else if (a.mode == 1) {
        // base l of the tile (global valid index vex + l) is dropped iff v0 + l lies in
        // [W_k, W_k + C) for some W_k = k 2^32, k >= 1; `done` windows end at or before v0
        const long long v0 = (long long)(a.c0 + vex);          // count before the tile
        const long long done = v0 >= C ? (long long)((unsigned long long)(v0 - C) >> 32) : 0;
        const long long W = (done + 1) << 32;                  // the next window's start
        const long long wa = W - v0, wb = wa + C;              // its local range [wa, wb)
        const long long a0 = wa < 0 ? 0 : (wa < (long long)agg ? wa : (long long)agg);
        const long long b0 = wb < (long long)agg ? wb : (long long)agg;   // wb > 0
        lenA = a0;
        gA = (long long)vex - done * C;
        sB = b0;
        lenB = (long long)agg - b0;
        gB = (long long)vex + b0 - (done + 1) * C;
    }
    for (int run = 0; run < 2; ++run) {
        const long long s0 = run == 0 ? sA : sB;
        const long long len = run == 0 ? lenA : lenB;
        if (len <= 0) continue;
        const long long g0 = run == 0 ? gA : gB;
        const long long gend = g0 + len < a.cap ? g0 + len : a.cap;
        if (gend <= g0) continue;
        const long long w0 = g0 >> 4, w1 = (gend - 1) >> 4;
        for (long long gw = w0 + t; gw <= w1; gw += kIT) {
            // 32 bits of the bit array from local code index (16 gw - g0 + s0)
            const long long lb = 2 * (16 * gw - g0 + s0) + 32;   // +32: the guard word
            const long long wi = lb >> 5;
            const int sh = (int)(lb & 31);
            const uint32_t lo = sb[wi], hi = sb[wi + 1];
            uint32_t v = sh ? __builtin_amdgcn_alignbit(hi, lo, sh) : lo;
            const long long p0 = 16 * gw > g0 ? 16 * gw : g0;
            const long long p1 = 16 * gw + 16 < gend ? 16 * gw + 16 : gend;
            const int b0 = (int)(p0 - 16 * gw), b1 = (int)(p1 - 16 * gw);
            const uint32_t m = (b1 == 16 ? 0xFFFFFFFFu : ((1u << (2 * b1)) - 1u)) &
                               ~((1u << (2 * b0)) - 1u);
            if (m == 0xFFFFFFFFu)
                a.out[gw] = v;
            else
                atomicOr(&a.out[gw], v & m);
        }
    }
}

// One thread: totals + crash info -> the cpg_ingest_result fields (host rules of cpg_ingest)
__global__ void k_ingest_final(IngestWs ws, int64_t chunk, int64_t cap, int mode, int quirks,
                               unsigned long long c0, long long* __restrict__ res) {
    if (threadIdx.x != 0) return;
    const long long V = ws.tot[0], Q = ws.tot[1], C = chunk;
    long long committed = (commits(c0 + (unsigned long long)V, c0, C) + Q) * C;
    long long status = CPG_OK, crash_byte = -1;
    const unsigned ct = *ws.crash_tile;
    if (ct != 0xFFFFFFFFu) {
        crash_byte = ws.crash_k[ct];
        committed = ws.crash_c[ct];
        status = CPG_E_REF_CRASH;
    }
    const long long capc = cap / C * C;
    if (committed > cap) {   // the first commit past the capacity fails first
        committed = capc;
        status = CPG_E_CAPACITY;
        crash_byte = -1;
    }
    if (*ws.timeout) status = CPG_E_DEVICE;
    res[0] = committed;
    res[1] = status;
    res[2] = crash_byte;
    res[3] = V;
    res[4] = Q;
    res[5] = ws.crash_tile[0] == 0xFFFFFFFFu ? 0 : 1;
    res[6] = mode;
    res[7] = quirks;
}

}  // namespace

// workspace: [stV | stQ] granules (zeroed every call) | 16 B of counters | per-tile crash
size_t ingest_ws_bytes(int64_t n) {
    const int64_t nt = (n + kTileBytes - 1) / kTileBytes;
    return (size_t)(nt * 16 + 64 + nt * 16 + 64);
}

hipError_t launch_ingest(const uint8_t* txt, int64_t n, int mode, int quirks, int64_t chunk,
                         uint32_t* out, int64_t cap, void* wsp, size_t ws_bytes,
                         long long* res, hipStream_t s, uint32_t count0) {
    const int64_t nt = (n + kTileBytes - 1) / kTileBytes;
    if (ws_bytes < ingest_ws_bytes(n) || nt >= (1ll << 31)) return hipErrorInvalidValue;
    char* w = static_cast<char*>(wsp);
    IngestWs ws;
    ws.stV = reinterpret_cast<unsigned long long*>(w);
    ws.stQ = ws.stV + nt;
    unsigned int* ctr = reinterpret_cast<unsigned int*>(w + nt * 16);
    ws.ticket = ctr;
    ws.timeout = ctr + 1;
    ws.crash_tile = ctr + 2;
    ws.tot = reinterpret_cast<long long*>(w + nt * 16 + 16);
    ws.crash_k = reinterpret_cast<long long*>(w + nt * 16 + 64);
    ws.crash_c = ws.crash_k + nt;
    hipError_t e;
    if ((e = hipMemsetAsync(w, 0, (size_t)(nt * 16 + 64), s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(ws.crash_tile, 0xFF, 4, s)) != hipSuccess) return e;
    if (cap > 0 && (e = hipMemsetAsync(out, 0, (size_t)((cap + 15) / 16) * 4, s)) != hipSuccess)
        return e;
    if (nt > 0) {
        IngestArgs a{txt, n, chunk, cap, nt, mode, quirks, out, (unsigned long long)count0};
        hipLaunchKernelGGL(k_ingest, dim3((unsigned)nt), dim3(kIT), 0, s, a, ws);
    }
    hipLaunchKernelGGL(k_ingest_final, dim3(1), dim3(64), 0, s, ws, chunk, cap, mode, quirks,
                       (unsigned long long)count0, res);
    return hipGetLastError();
}

}  // namespace cpg
