// count_dev.h — labelled-count device code, shared by the standalone count
// launch (k_count.hip) and the fused training pass (k_estep.hip): one lane counts one block
// of 64 bases.
//
// The counts are those of the BW mapper's init / transition / emission stripes
// (CpGIslandFinder.java:200) taken from hard labels: state s_t = base_t + (sign_t ? 0 : 4).
// Only 72 raw sums are accumulated — per dinucleotide d = p*4 + b (p the previous base):
// every transition (tot), the '+'->'+' ones (pp), '+'->'-' (pm), '-'->'+' (mp), and the 8
// init states; everything else is an exact integer identity of them (final_counts).
#pragma once
#include "cpg_internal.h"

namespace cpg {
namespace cnt {

constexpr int kRaw = 72;        // tot[16] pp[16] pm[16] mp[16] init[8]
constexpr int kRep = 16;        // replicated accumulator sets (workgroup b adds into b % kRep)
constexpr uint32_t M55 = 0x55555555u;

struct Masks {
    uint32_t e[4];   // bit 2k set iff base k == b
};
__device__ __forceinline__ Masks base_masks(uint32_t w) {
    const uint32_t h = w >> 1;
    Masks m;
    m.e[0] = ~(w | h) & M55;
    m.e[1] = w & ~h & M55;
    m.e[2] = h & ~w & M55;
    m.e[3] = w & h & M55;
    return m;
}
// 16 bits (bit k) -> even bit positions (bit 2k)
__device__ __forceinline__ uint32_t spread16(uint32_t x) {
    x &= 0xFFFFu;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x;
}

// even bit positions (bit 2k) -> 16 bits (bit k)
__device__ __forceinline__ uint32_t compact16(uint32_t x) {
    x &= 0x55555555u;
    x = (x | (x >> 1)) & 0x33333333u;
    x = (x | (x >> 2)) & 0x0F0F0F0Fu;
    x = (x | (x >> 4)) & 0x00FF00FFu;
    x = (x | (x >> 8)) & 0x0000FFFFu;
    return x;
}

// One lane's register counters.  The 16 dinucleotide counts of a set of transitions are
// kept in a BASIS of 16 sums from which they follow exactly (class_of): the 9 counts with
// p, b < 3 (p the previous base), the 3 row sums (previous base p < 3), the 3 column sums
// (base b < 3) and the number of transitions — 9 AND+popcounts and 6 popcounts per word pair
// instead of 16 ANDs + 16 popcounts per word, and masks for three base values, not four.
// Two words are counted at once: a word's base masks sit on the even bits, the next word's
// are shifted onto the odd bits of the same register (popcounts do not care about order).
// Two 16-bit fields per basis sum: all transitions (low half) and the '+'->'+' ones (high
// half); a block without a '+' state skips the sign work.  Sign changes (island borders: a
// few per island) go to the LDS counters lds[32 .. 64) one by one.  A field grows by at most
// 64 per block and flush() sums 64 lanes, so a lane flushes at least every 15 blocks.
struct Lane {
    static constexpr int kMaxBlocks = 15;
    uint32_t c[16];
    __device__ __forceinline__ Lane() {
#pragma unroll
        for (int d = 0; d < 16; ++d) c[d] = 0u;
    }
    struct M3 {
        uint32_t e[3];   // bit 2k set iff base k == b (b < 3)
    };
    static __device__ __forceinline__ M3 masks3(uint32_t w) {
        const uint32_t h = w >> 1;
        return M3{{~(w | h) & M55, w & ~h & M55, h & ~w & M55}};
    }
    // w: the block's 4 packed words; s: its 2 sign words; wprev / sprev: the packed word and
    // the sign bit before the block (ignored at a chunk start: no transition into position 0).
    // Two code paths chosen per lane (a wave runs the '+' path only if one of its lanes needs
    // it): as selects, the compiler computed the '+' path's 16-bit high fields always.
    __device__ __forceinline__ void block(uint4 w, uint2 s, uint32_t wprev, uint32_t sprev,
                                          bool cstart, uint32_t* lds) {
        if (cstart) sprev = 0u;
        if ((s.x | s.y | sprev) != 0u) block_t<true>(w, s, wprev, sprev, cstart, lds);
        else block_t<false>(w, s, wprev, sprev, cstart, lds);
    }
    template <bool kPlus>
    __device__ __forceinline__ void block_t(uint4 w, uint2 s, uint32_t wprev, uint32_t sprev,
                                            bool cstart, uint32_t* lds) {
        const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
        const uint32_t sw[4] = {s.x & 0xFFFFu, s.x >> 16, s.y & 0xFFFFu, s.y >> 16};
        M3 last = masks3(wprev);
        uint32_t sprv = sprev & 1u;
        uint64_t ch = 0u;   // positions whose sign differs from the previous position's
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
            const M3 ea = masks3(ww[2 * pr]), eb = masks3(ww[2 * pr + 1]);
            uint32_t P[3], E[3], Ec[3];
#pragma unroll
            for (int b = 0; b < 3; ++b) {
                uint32_t pa = __builtin_amdgcn_alignbit(ea.e[b], last.e[b], 30);
                if (pr == 0 && cstart) pa &= ~1u;   // no transition into position 0
                const uint32_t pb = __builtin_amdgcn_alignbit(eb.e[b], ea.e[b], 30);
                P[b] = pa | (pb << 1);
                E[b] = ea.e[b] | (eb.e[b] << 1);
                Ec[b] = (pr == 0 && cstart) ? (E[b] & ~1u) : E[b];   // column: positions with a transition
            }
            last = eb;
            uint32_t PP = 0u;
            if (kPlus) {
                uint32_t pp2[2];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int k = 2 * pr + h;
                    const uint32_t S = spread16(sw[k]);
                    const uint32_t Sp = (S << 2) | sprv;   // sign of the previous position
                    sprv = sw[k] >> 15;
                    pp2[h] = Sp & S;   // bit 0 of a chunk's first word: Sp = 0
                    uint32_t chg = (Sp ^ S) & M55;
                    if (k == 0 && cstart) chg &= ~1u;
                    ch |= (uint64_t)compact16(chg) << (16 * k);
                }
                PP = pp2[0] | (pp2[1] << 1);
            }
            auto add = [&](int j, uint32_t x) {
                c[j] += kPlus ? __popc(x) + (__popc(x & PP) << 16) : __popc(x);
            };
#pragma unroll
            for (int p = 0; p < 3; ++p)
#pragma unroll
                for (int b = 0; b < 3; ++b) add(p * 3 + b, P[p] & E[b]);
#pragma unroll
            for (int p = 0; p < 3; ++p) add(9 + p, P[p]);
#pragma unroll
            for (int b = 0; b < 3; ++b) add(12 + b, Ec[b]);
            if (kPlus) c[15] += __popc(PP) << 16;
        }
        c[15] += cstart ? 63u : 64u;
        if (kPlus) {
            // sign changes, position by position (rare: island borders); a loop over the
            // block's 64-bit change mask, not inside the per-word code, so that it unrolls
            while (ch) {
                const int q = (int)__builtin_ctzll(ch);
                ch &= ch - 1u;
                const uint32_t d = (q ? base_at(w, q - 1) : wprev >> 30) * 4u + base_at(w, q);
                const uint32_t sq = ((q < 32 ? s.x : s.y) >> (q & 31)) & 1u;
                atomicAdd(&lds[sq ? 48u + d : 32u + d], 1u);
            }
        }
    }
    // base q (0..63) of a block (selects, no indexed array)
    static __device__ __forceinline__ uint32_t base_at(uint4 w, int q) {
        const uint32_t x = q < 32 ? (q < 16 ? w.x : w.y) : (q < 48 ? w.z : w.w);
        return (x >> (2 * (q & 15))) & 3u;
    }
    // the wave's basis sums -> lds[0 .. 16) (all transitions) and lds[16 .. 32) ('+'->'+');
    // every lane of the wave calls; counters re-zeroed.  Recursive halving (after 4 levels
    // lane L holds sum L & 15 of its 16-lane row, 15 shuffles instead of 16 x 4), then the rows.
    __device__ __forceinline__ void flush(uint32_t* lds) {
        const int lane = threadIdx.x & 63;
#pragma unroll
        for (int lvl = 0; lvl < 4; ++lvl) {
            const int o = 8 >> lvl;
            // the halves chosen by masks, not by `up ? c[i] : c[i + o]`: that select becomes an
            // indexed (scratch) array access
            const uint32_t m = (lane & o) ? ~0u : 0u;
#pragma unroll
            for (int i = 0; i < o; ++i) {
                const uint32_t send = (c[i] & m) | (c[i + o] & ~m);
                const uint32_t keep = (c[i + o] & m) | (c[i] & ~m);
                c[i] = keep + (uint32_t)__shfl_xor((int)send, o);
            }
        }
        uint32_t x = c[0];
        x += (uint32_t)__shfl_xor((int)x, 16);
        x += (uint32_t)__shfl_xor((int)x, 32);
        if (lane < 16) {
            if (x & 0xFFFFu) atomicAdd(&lds[lane], x & 0xFFFFu);
            if (x >> 16) atomicAdd(&lds[16 + lane], x >> 16);
        }
#pragma unroll
        for (int d = 0; d < 16; ++d) c[d] = 0u;
    }
};

// raw sum i (< kRaw, the accumulators' layout tot[16] pp[16] pm[16] mp[16] init[8]) from a
// workgroup's LDS counters: tot and pp from their basis (Lane), exact integer identities
__device__ __forceinline__ uint32_t raw_of(const uint32_t* lds, int i) {
    if (i >= 32) return lds[i];
    const uint32_t* B = lds + (i & 16);
    const int p = (i & 15) >> 2, b = i & 3;
    if (p < 3 && b < 3) return B[p * 3 + b];
    if (p < 3) return B[9 + p] - B[p * 3] - B[p * 3 + 1] - B[p * 3 + 2];
    if (b < 3) return B[12 + b] - B[b] - B[3 + b] - B[6 + b];
    uint32_t v = B[15];
#pragma unroll
    for (int j = 0; j < 9; ++j) v += B[j];
#pragma unroll
    for (int j = 9; j < 15; ++j) v -= B[j];
    return v;
}

// the init state of a chunk's first base
__device__ __forceinline__ uint32_t init_state(uint32_t w0, uint32_t s0) {
    return (w0 & 3u) + ((s0 & 1u) ? 0u : 4u);
}

// cpg_counts_i64 from the 72 raw sums; one output word per thread t < 124
// (layout init[8] trans[8][8] emit[8][4] dinuc[4][4] mono[4])
__device__ __forceinline__ void final_counts(const uint64_t* raw, int t, int64_t* __restrict__ out) {
    auto trans = [&](int i, int j) {
        const int d = (i & 3) * 4 + (j & 3), si = i >> 2, sj = j >> 2;
        const int64_t tt = (int64_t)raw[d], ppv = (int64_t)raw[16 + d],
                      pmv = (int64_t)raw[32 + d], mpv = (int64_t)raw[48 + d];
        return si == 0 ? (sj == 0 ? ppv : pmv) : (sj == 0 ? mpv : tt - ppv - pmv - mpv);
    };
    int64_t v = 0;
    if (t < 8) {
        v = (int64_t)raw[64 + t];
    } else if (t < 72) {
        v = trans((t - 8) >> 3, (t - 8) & 7);
    } else if (t < 104) {
        const int s = (t - 72) >> 2, k = (t - 72) & 3;     // emit[s][k]: every visit of s
        if (k == (s & 3)) {
            v = (int64_t)raw[64 + s];
            for (int r = 0; r < 8; ++r) v += trans(r, s);
        }
    } else if (t < 120) {
        v = (int64_t)raw[t - 104];                         // dinuc[p][b]
    } else {
        // mono[b]: every base at a chunk position > 0 is the current base of one transition,
        // position 0 is counted by init
        const int b = t - 120;
        for (int p = 0; p < 4; ++p) v += (int64_t)raw[p * 4 + b];
        v += (int64_t)raw[64 + b] + (int64_t)raw[64 + b + 4];
    }
    out[t] = v;
}

// Finalize in two halves so that a caller can run it beside another finalize: load (thread
// i < kRaw: the replicas' sum into raw[i]), a workgroup barrier, then store (threads
// [0, nthr): re-zero the accumulators, write the 124 outputs).  kAgent: the accumulators were
// written by workgroups of the same launch (device-scope loads).
template <bool kAgent>
__device__ __forceinline__ void fin_load(unsigned long long* gacc, uint64_t* raw, int i) {
    uint64_t v = 0;
#pragma unroll
    for (int r = 0; r < kRep; ++r) v += kAgent ? load_agent(gacc + r * kRaw + i) : gacc[r * kRaw + i];
    raw[i] = v;
}
__device__ __forceinline__ void fin_store(unsigned long long* gacc, const uint64_t* raw,
                                          int64_t* out, int t, int nthr) {
    for (int i = t; i < kRaw * kRep; i += nthr) gacc[i] = 0ull;
    for (int i = t; i < 124; i += nthr) final_counts(raw, i, out);
}

}  // namespace cnt
}  // namespace cpg
