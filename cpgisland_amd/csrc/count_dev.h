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

// (m & x) | (~m & y) as v_bitop3_b32 (truth table 0xCA): a full-rate instruction on gfx950,
// where v_bfi_b32 issues at half rate (tools/ubench_bits.hip: 2.6 against 4.4 cycles per
// wave-instruction per SIMD at 4 waves per SIMD)
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t x, uint32_t y) {
#if defined(__gfx950__)
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(r) : "v"(m), "v"(x), "v"(y));
    return r;
#else   // (other targets: v_bitop3 is gfx950's; the compiler's v_bfi_b32)
    return (m & x) | (~m & y);
#endif
}
// c + popcount(x) as ONE v_bcnt_u32_b32 (its second operand is the addend): the compiler pairs
// two popcounts with a v_add3 instead, three instructions where two do
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t c) {
#if defined(__gfx950__)
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(c));
    return r;
#else
    return c + __popc(x);
#endif
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

// One lane's register counters.  The 16 dinucleotide counts of a set of transitions are kept
// as their 16 MOMENTS: with the four bit-planes of a transition — lo / hi bit of the current
// base b and lo / hi bit of the previous base p — moment S (S = a subset of the planes, bit 0
// lo, bit 1 hi, bit 2 previous lo, bit 3 previous hi) counts the transitions whose planes in S
// are all 1, moment 0 the transitions themselves.  The count of dinucleotide d = p * 4 + b
// follows by Moebius inversion, N(d) = sum over S containing d of (-1)^|S \ d| m_S (raw_of):
// 11 ANDs + 15 v_bcnt per 32 positions on four planes, which cost 11 instructions to form
// (two words at once: a word's positions on the even bits, the next word's on the odd bits
// of the same register — popcounts do not care about order).  The registers hold the moments
// of ALL transitions (32-bit: flushed once per kernel or per caller's batch); the moments of
// the '+'->'+' transitions and the sign changes (island borders: a few per island) occur in
// few blocks and go to the LDS counters at once (lds[16 .. 32) and lds[32 .. 64)), so the
// common block — no '+' state — adds each popcount straight into its register.
struct Lane {
    uint32_t c[16];
    // the '+'->'+' moments: in the standalone count kernel (kSplit below) per-lane registers
    // too, added by the lanes that have '+' states and flushed once (flush_plus); in the
    // E-step's fused counts the whole wave runs the '+' work when one lane needs it and adds one
    // wave sum per moment to lds[16 .. 32) (registers there are the E-step's)
    uint32_t cp[16];
    __device__ __forceinline__ Lane() {
#pragma unroll
        for (int d = 0; d < 16; ++d) c[d] = cp[d] = 0u;
    }
    // w: the block's 4 packed words; s: its 2 sign words; wprev / sprev: the packed word and
    // the sign bit before the block (ignored at a chunk start: no transition into position 0);
    // valid = false: a lane without a block (counts nothing).  EVERY lane of the wave calls
    // (the '+' work below reduces over the wave).
    // the 15 all-transition moments of the block's 64 positions into c[1..15]; kMask: pair 0's
    // planes masked by pm0 (a chunk start: no transition into position 0), pair 1's by vm
    template <bool kMask, bool kAsm>
    __device__ __forceinline__ void moments(const uint32_t (&ww)[4], uint32_t wprev, uint32_t pm0,
                                            uint32_t vm) {
        uint32_t last = wprev;
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
            const uint32_t a = ww[2 * pr], b = ww[2 * pr + 1];
            // planes of the 32 positions: word a's position k at bit 2k, word b's at 2k+1
            uint32_t LO = bfi(M55, a, b << 1);
            uint32_t HI = bfi(M55, a >> 1, b);
            // the previous base's planes: position k-1 of the same word two bits below; bit 0
            // (a[0]) from the word before a (its position 15: bits 30 / 31), bit 1 (b[0]) from
            // a[15] (bit 30 of the planes) — through bits 30 / 31 of an aligned pair
            uint32_t PLO = __builtin_amdgcn_alignbit(LO, bfi(0x80000000u, LO << 1, last), 30);
            uint32_t PHI = __builtin_amdgcn_alignbit(HI, bfi(0x80000000u, HI << 1, last >> 1), 30);
            if constexpr (kMask) {
                const uint32_t pm = pr == 0 ? pm0 : vm;
                LO &= pm; HI &= pm; PLO &= pm; PHI &= pm;
            }
            last = b;
            const uint32_t lh = LO & HI, pq = PLO & PHI;
            const uint32_t x[16] = {0u, LO, HI, lh, PLO, LO & PLO, HI & PLO, lh & PLO,
                                    PHI, LO & PHI, HI & PHI, lh & PHI, pq, LO & pq, HI & pq, lh & pq};
#pragma unroll
            for (int j = 1; j < 16; ++j) c[j] = kAsm ? bcnt_acc(x[j], c[j]) : c[j] + __popc(x[j]);
        }
    }
    // kSplit: the masks only in a wave with a masked lane (a wave-uniform branch around two
    // copies of the moments: the standalone count kernel, where chunk starts are 1 in 1,024
    // blocks at the reference's chunk length), and the accumulating v_bcnt; otherwise always
    // masked and the compiler's popcounts (the E-step's fused counts: inside its 128-VGPR
    // budget the inline-asm popcounts cost 6 spills)
    template <bool kSplit = true>
    __device__ __forceinline__ void block(uint4 w, uint2 s, uint32_t wprev, uint32_t sprev,
                                          bool cstart, uint32_t* lds, bool valid = true) {
        if (cstart) sprev = 0u;
        const uint32_t vm = valid ? ~0u : 0u;
        const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
        // no transition into a chunk's position 0, nothing from a lane without a block
        if (!kSplit || __builtin_amdgcn_ballot_w64(cstart || !valid))
            moments<true, kSplit>(ww, wprev, cstart ? (vm & ~1u) : vm, vm);
        else
            moments<false, kSplit>(ww, wprev, ~0u, ~0u);
        c[0] += valid ? (cstart ? 63u : 64u) : 0u;
        // the '+' work (rare: island blocks)
        const bool plus = valid && (s.x | s.y | sprev) != 0u;
        if constexpr (kSplit) {
            if (plus) plus_block<true>(w, s, wprev, sprev, cstart, lds);
        } else if (__builtin_amdgcn_ballot_w64(plus)) {
            plus_block<false>(w, plus ? s : make_uint2(0u, 0u), wprev, plus ? sprev : 0u, cstart,
                              lds);
        }
    }
    // the '+'->'+' moments (the same planes masked by the '+'->'+' positions: kReg into cp[],
    // else one wave sum per moment to LDS) and the sign changes, straight to LDS
    template <bool kReg>
    __device__ __forceinline__ void plus_block(uint4 w, uint2 s, uint32_t wprev,
                                               uint32_t sprev, bool cstart, uint32_t* lds) {
        const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
        const uint32_t sw[4] = {s.x & 0xFFFFu, s.x >> 16, s.y & 0xFFFFu, s.y >> 16};
        uint32_t last = wprev;
        uint32_t sprv = sprev & 1u;
        uint64_t ch = 0u;   // positions whose sign differs from the previous position's
        // both pairs' planes masked by their '+'->'+' positions (PP), then the moments one at a
        // time (few registers live: this runs beside the counters and the loaded batches)
        uint32_t lo[2], hi[2], plo[2], phi[2], pp[2];
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
            const uint32_t a = ww[2 * pr], b = ww[2 * pr + 1];
            const uint32_t LO = bfi(M55, a, b << 1);
            const uint32_t HI = bfi(M55, a >> 1, b);
            const uint32_t PLO = __builtin_amdgcn_alignbit(LO, bfi(0x80000000u, LO << 1, last), 30);
            const uint32_t PHI = __builtin_amdgcn_alignbit(HI, bfi(0x80000000u, HI << 1, last >> 1), 30);
            last = b;
            uint32_t pp2[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int k = 2 * pr + h;
                const uint32_t S = spread16(sw[k]);
                const uint32_t Sp = (S << 2) | sprv;   // sign of the previous position
                sprv = sw[k] >> 15;
                pp2[h] = Sp & S;   // bit 0 of a chunk's first word: Sp = 0 (sprev = 0)
                uint32_t chg = (Sp ^ S) & M55;
                if (k == 0 && cstart) chg &= ~1u;
                ch |= (uint64_t)compact16(chg) << (16 * k);
            }
            pp[pr] = pp2[0] | (pp2[1] << 1);   // '+'->'+' transitions
            lo[pr] = LO & pp[pr]; hi[pr] = HI & pp[pr]; plo[pr] = PLO & pp[pr]; phi[pr] = PHI & pp[pr];
        }
        auto mom = [&](int pr, int j) {   // moment j's mask of pair pr (j compile-time)
            uint32_t x = pp[pr];
            if (j & 1) x &= lo[pr];
            if (j & 2) x &= hi[pr];
            if (j & 4) x &= plo[pr];
            if (j & 8) x &= phi[pr];
            return x;
        };
        if constexpr (kReg) {   // per-lane registers (two accumulating v_bcnt per moment)
#pragma unroll
            for (int j = 0; j < 16; ++j) cp[j] = bcnt_acc(mom(1, j), bcnt_acc(mom(0, j), cp[j]));
        } else {       // the whole wave is here: one reduction, one atomic per moment
            uint32_t m[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) m[j] = __popc(mom(0, j)) + __popc(mom(1, j));
            wave_sum16(m, lds + 16);   // (a lane without '+' states adds zeros)
        }
        // sign changes, position by position (rare: island borders)
        while (ch) {
            const int q = (int)__builtin_ctzll(ch);
            ch &= ch - 1u;
            const uint32_t d = (q ? base_at(w, q - 1) : wprev >> 30) * 4u + base_at(w, q);
            const uint32_t sq = ((q < 32 ? s.x : s.y) >> (q & 31)) & 1u;
            atomicAdd(&lds[sq ? 48u + d : 32u + d], 1u);
        }
    }
    // base q (0..63) of a block (selects, no indexed array)
    static __device__ __forceinline__ uint32_t base_at(uint4 w, int q) {
        const uint32_t x = q < 32 ? (q < 16 ? w.x : w.y) : (q < 48 ? w.z : w.w);
        return (x >> (2 * (q & 15))) & 3u;
    }
    // the wave's moment sums -> lds[0 .. 16); every lane of the wave calls; counters
    // re-zeroed
    __device__ __forceinline__ void flush(uint32_t* lds) {
        wave_sum16(c, lds);
#pragma unroll
        for (int d = 0; d < 16; ++d) c[d] = 0u;
    }
    // the '+'->'+' moment registers (the standalone count kernel) -> lds[16 .. 32)
    __device__ __forceinline__ void flush_plus(uint32_t* lds) {
        wave_sum16(cp, lds + 16);
#pragma unroll
        for (int d = 0; d < 16; ++d) cp[d] = 0u;
    }
    // lds[0 .. 16) += the wave's sums of c[0 .. 16) (c is clobbered).  Recursive halving (after
    // 4 levels lane L holds sum L & 15 of its 16-lane row, 15 shuffles instead of 16 x 4), then
    // the rows; one LDS atomic per sum (a per-lane atomic on a shared address would become the
    // compiler's lane-by-lane reduction loop)
    static __device__ __forceinline__ void wave_sum16(uint32_t (&c)[16], uint32_t* lds) {
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
        if (lane < 16 && x) atomicAdd(&lds[lane], x);
    }
};

// raw sum i (< kRaw, the accumulators' layout tot[16] pp[16] pm[16] mp[16] init[8]) from a
// workgroup's LDS counters: tot and pp from their moments (Lane) by Moebius inversion — the
// cell d = p * 4 + b has exactly the planes of the bits of d (bit 0 lo, 1 hi of b; 2 lo, 3 hi
// of p), so N(d) = sum over S containing d of (-1)^|S \ d| m_S, m_0 = the transitions (exact
// integer identities, modulo 2^32 with a non-negative result)
__device__ __forceinline__ uint32_t raw_of(const uint32_t* lds, int i) {
    if (i >= 32) return lds[i];
    const uint32_t* B = lds + (i & 16);
    const int d = i & 15;
    uint32_t v = 0u;
#pragma unroll
    for (int S = 0; S < 16; ++S)
        if ((S & d) == d) v += (__popc((uint32_t)(S ^ d)) & 1) ? 0u - B[S] : B[S];
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
