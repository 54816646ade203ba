// cpg_host.cpp — host-side parts of libcpg.so: error state, ASCII ingest, synthetic
// genome, reducer normalisation, model checks and the Viterbi constant tables.
//
// Reference: /root/reference/CpGIslandFinder.java (cited per function).

#include <cfenv>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "cpg_internal.h"

namespace cpg {

static thread_local char g_err[512] = "";

int set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

int model_check_deterministic(const cpg_model* m) {
    for (int i = 0; i < 8; ++i)
        for (int k = 0; k < 4; ++k) {
            double want = (k == i % 4) ? 1.0 : 0.0;
            if (m->b[i][k] != want)
                return set_error(CPG_E_UNSUPPORTED,
                                 "emission b[%d][%d]=%.17g: the GPU path needs the "
                                 "deterministic emission matrix of :166-173",
                                 i, k, m->b[i][k]);
        }
    return CPG_OK;
}

bool vit_fast_ok(const cpg_model* m) {
    for (int i = 0; i < 8; ++i) {
        for (int k = 0; k < 4; ++k)
            if (m->b[i][k] != ((k == i % 4) ? 1.0 : 0.0)) return false;
        if (!(m->pi[i] >= 0.0 && m->pi[i] <= 1.0)) return false;
        for (int j = 0; j < 8; ++j)
            if (!(m->a[i][j] > 0.0 && m->a[i][j] <= 1.0)) return false;
    }
    return true;
}

// the general path's constants: every log Mahout's loop takes, C library log
void gen_prepare(const cpg_model* m, GenConsts* gc) {
    for (int j = 0; j < 8; ++j)
        for (int i = 0; i < 8; ++i) gc->L[j][i] = std::log(m->a[j][i]);
    for (int i = 0; i < 8; ++i)
        for (int k = 0; k < 4; ++k) {
            gc->LB[i][k] = std::log(m->b[i][k]);
            gc->LP[i][k] = std::log(m->pi[i] * m->b[i][k]);
        }
}

// Viterbi constants.  L = log a exactly as Mahout evaluates Math.log(a.getQuick(j, i))
// (here: the C library log, shared by every kernel and by the oracle).
int vit_prepare(const cpg_model* m, int64_t chunk_len, VitConsts* vc, VitTables* vt) {
    int rc = model_check_deterministic(m);
    if (rc) return rc;
    for (int i = 0; i < 8; ++i) {
        if (!(m->pi[i] >= 0.0 && m->pi[i] <= 1.0))
            return set_error(CPG_E_UNSUPPORTED, "pi[%d]=%.17g outside [0,1]", i, m->pi[i]);
        for (int j = 0; j < 8; ++j)
            if (!(m->a[i][j] > 0.0 && m->a[i][j] <= 1.0))
                return set_error(CPG_E_UNSUPPORTED,
                                 "a[%d][%d]=%.17g: the GPU Viterbi needs 0 < a <= 1", i, j,
                                 m->a[i][j]);
    }
    std::memset(vc, 0, sizeof *vc);
    double maxabs = 0.0;
    for (int p = 0; p < 4; ++p)
        for (int b = 0; b < 4; ++b) {
            double* l = vc->L[p + 4 * b];   // d = prev | cur << 2 (one bfe of the packed word)
            l[0] = std::log(m->a[p][b]);
            l[1] = std::log(m->a[p + 4][b]);
            l[2] = std::log(m->a[p][b + 4]);
            l[3] = std::log(m->a[p + 4][b + 4]);
            for (int k = 0; k < 4; ++k) maxabs = std::fmax(maxabs, -l[k]);
        }
    double minlogpi = 0.0;
    for (int i = 0; i < 8; ++i) {
        vc->logpi[i] = std::log(m->pi[i] * m->b[i][i % 4]);   // log(pi_i * b_i(o_0))
        if (std::isfinite(vc->logpi[i])) minlogpi = std::fmin(minlogpi, vc->logpi[i]);
    }
    if (maxabs <= 0.0) maxabs = 1e-300;
    // fixed point: kSB steps of the largest constant stay below 2^29
    int f = 24;
    while (f > 0 && (double)kSB * maxabs * std::ldexp(1.0, f) > std::ldexp(1.0, 29)) --f;
    vc->qshift = f;
    for (int d = 0; d < 16; ++d)
        for (int k = 0; k < 4; ++k)
            vc->Q[d][k] = (int32_t)std::llround(std::ldexp(vc->L[d][k], f));
    // |approx - exact| bound: constant rounding + fp64 drift of the sequential recurrence
    double vmax = -minlogpi + (double)chunk_len * maxabs + 1.0;
    int Emax = (int)std::floor(std::log2(vmax)) + 1;
    vc->eps = ((double)chunk_len + 1.0) * std::ldexp(1.0, -(f + 1)) +
              (double)chunk_len * std::ldexp(1.0, Emax - 53);
    vc->eps = vc->eps * 1.01 + 1e-9;
    vc->spread = 2.0 * maxabs;
    int emin = 4;
    while (std::ldexp(1.0, emin + 1) <= 64.0 * maxabs) ++emin;
    vc->emin = emin;
    vc->emax = std::max(std::min(Emax + 1, kMaxBinade - 2), vc->emin);
    std::memset(vt, 0, sizeof *vt);
    vc->tie_mask = 0;
    // tables for every binade >= emin (model-only, so a device copy can be cached)
    for (int e = vc->emin; e < kMaxBinade - 1; ++e) {
        double u = std::ldexp(1.0, e - 52);
        for (int d = 0; d < 16; ++d)
            for (int k = 0; k < 4; ++k) {
                double r = vc->L[d][k] / u;          // exact (power-of-two scaling)
                double fl = std::floor(r);
                if (r - fl == 0.5) vc->tie_mask |= (1ull << e);
                vt->Le[e][d][k] = std::nearbyint(r) * u;   // exact multiple of u
            }
    }
    return CPG_OK;
}

// ---------------------------------------------------------------------------------
// Host utilities
// ---------------------------------------------------------------------------------
static inline int sym_of(unsigned char ch) {   // :114-123 / :240-249
    switch (ch) {
        case 'A': case 'a': return 0;
        case 'C': case 'c': return 1;
        case 'G': case 'g': return 2;
        case 'T': case 't': return 3;
        default: return -1;
    }
}

}  // namespace cpg

using namespace cpg;

extern "C" {

const char* cpg_last_error(void) { return g_err; }
int cpg_abi_version(void) { return CPG_ABI_VERSION; }

// CpGIslandFinder.java:155-173
int cpg_initial_model(cpg_model* m) {
    if (!m) return set_error(CPG_E_INVALID, "null model");
    static const double pi[8] = {0.05, 0.05, 0.05, 0.05, 0.2, 0.2, 0.2, 0.2};
    static const double a[8][8] = {
        {0.170, 0.274, 0.426, 0.120, 0.0025, 0.0025, 0.0025, 0.0025},
        {0.170, 0.358, 0.274, 0.188, 0.0025, 0.0025, 0.0025, 0.0025},
        {0.161, 0.329, 0.375, 0.125, 0.0025, 0.0025, 0.0025, 0.0025},
        {0.079, 0.345, 0.384, 0.182, 0.0025, 0.0025, 0.0025, 0.0025},
        {0.0025, 0.0025, 0.0025, 0.0025, 0.300, 0.205, 0.275, 0.210},
        {0.0025, 0.0025, 0.0025, 0.0025, 0.393, 0.137, 0.088, 0.372},
        {0.0025, 0.0025, 0.0025, 0.0025, 0.248, 0.246, 0.288, 0.208},
        {0.0025, 0.0025, 0.0025, 0.0025, 0.177, 0.239, 0.282, 0.292}};
    std::memcpy(m->pi, pi, sizeof pi);
    std::memcpy(m->a, a, sizeof a);
    std::memset(m->b, 0, sizeof m->b);
    for (int i = 0; i < 8; ++i) m->b[i][i % 4] = 1.0;
    return CPG_OK;
}

// CpGIslandFinder.java:112-145 (mode 0) and :238-259 (mode 1), from Java `count` = count0
// with an empty list (cpg_ingest: 0; the test hook cpgx_ingest_at: a multiple of the chunk).
// `count` is a Java int: at 2^32 bases it wraps to 0 and the chunk test is skipped, so the
// list keeps its chunk and grows by another chunk until the next multiple.  There the
// training reader's DenseVector(0x10000).set(0x10000, …) throws (:133-134: a crash at the
// valid byte that brings count to 2^32 + 65,536), while the decode reader copies get(0 ..
// 2^20-1) — the held chunk — and clear() silently drops the 2^20 bases read after the wrap
// (:257-259); a non-ACGT byte read while count == 0 fires nothing.
static int ingest_host(const char* txt, size_t n, int mode, int compat_quirks, uint32_t* packed,
                       int64_t cap_bases, int64_t* nbases, uint32_t count0) {
    if (!txt || !packed || !nbases || (mode != 0 && mode != 1) || cap_bases < 0)
        return set_error(CPG_E_INVALID, "cpg_ingest: bad argument");
    const uint32_t mask = mode == 0 ? 0xFFFFu : 0xFFFFFu;
    const int64_t chunk = mode == 0 ? CPG_TRAIN_CHUNK : CPG_DECODE_CHUNK;
    if (count0 & mask) return set_error(CPG_E_INVALID, "ingest: count0 not a chunk multiple");
    uint32_t count = count0;     // Java int count (wraps)
    int64_t listlen = 0;         // bases pending in observedSequence
    int64_t out = 0;             // bases committed (whole chunks)
    *nbases = 0;
    // Committed + pending bases are written in place; a chunk boundary commits them.
    auto put = [&](int64_t pos, int v) {
        uint32_t& w = packed[pos >> 4];
        int sh = (int)(pos & 15) * 2;
        w = (w & ~(3u << sh)) | ((uint32_t)v << sh);
    };
    for (size_t k = 0; k < n; ++k) {
        int v = sym_of((unsigned char)txt[k]);
        if (v != -1) {
            // past a wrap the decode reader's bases beyond the held chunk are dropped at the
            // next multiple (or stay an undecoded tail): not written
            if (out + listlen < cap_bases && (mode == 0 || listlen < chunk))
                put(out + listlen, v);
            listlen++;
            count++;
        }
        if (count != 0 && (count & mask) == 0) {
            if (listlen > chunk && mode == 0) {
                *nbases = out;
                return set_error(CPG_E_REF_CRASH,
                                 "reference throws IndexOutOfBoundsException at input byte "
                                 "%zu (:133-134: the base count wrapped past 2^32, the chunk "
                                 "vector gets %lld bases)", k, (long long)listlen);
            }
            if (listlen >= chunk) {      // == chunk, or 2 chunks after a wrap (mode 1)
                if (out + chunk > cap_bases) {
                    *nbases = out;
                    return set_error(CPG_E_CAPACITY, "cpg_ingest: capacity %lld bases exceeded",
                                     (long long)cap_bases);
                }
                out += chunk;
                listlen = 0;
            } else if (compat_quirks) {          // list is empty here (count unchanged)
                if (mode == 1) {
                    *nbases = out;
                    return set_error(CPG_E_REF_CRASH,
                                     "reference throws IndexOutOfBoundsException at input "
                                     "byte %zu (:257-258 on an empty list)", k);
                }
                if (out + chunk > cap_bases) {
                    *nbases = out;
                    return set_error(CPG_E_CAPACITY, "cpg_ingest: capacity exceeded");
                }
                for (int64_t i = 0; i < chunk; i += 16) packed[(out + i) >> 4] = 0u;  // all-A
                out += chunk;
            }
        }
    }
    *nbases = out;          // tail (listlen bases) is never processed by the reference
    return CPG_OK;
}

int cpg_ingest(const char* txt, size_t n, int mode, int compat_quirks, uint32_t* packed,
               int64_t cap_bases, int64_t* nbases) {
    return ingest_host(txt, n, mode, compat_quirks, packed, cap_bases, nbases, 0u);
}

// test hook (cpg_internal.h, not part of cpg.h): the reader from Java count = count0
int cpgx_ingest_at(const char* txt, size_t n, int mode, int compat_quirks, uint32_t* packed,
                   int64_t cap_bases, int64_t* nbases, uint32_t count0) {
    return ingest_host(txt, n, mode, compat_quirks, packed, cap_bases, nbases, count0);
}

// ---------------------------------------------------------------------------------
// Synthetic genome: counter-based per 65,536-base segment, reproducible anywhere.
// ---------------------------------------------------------------------------------
namespace {
struct Rng {
    uint64_t s[4];
    static uint64_t splitmix(uint64_t& x) {
        uint64_t z = (x += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    Rng(uint64_t seed, uint64_t stream) {
        uint64_t x = seed ^ (stream * 0xD1B54A32D192ED03ull);
        for (auto& v : s) v = splitmix(x);
    }
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {   // xoshiro256**
        uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
        s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t;
        s[3] = rotl(s[3], 45);
        return r;
    }
    double uni() { return (double)(next() >> 11) * 0x1.0p-53; }
};

constexpr int64_t kSeg = 65536;
constexpr double kMeanGap = 100000.0;

struct SynthTables {
    double cdf[2][4][4];    // [island][prev][next] cumulative
};

SynthTables make_tables() {
    cpg_model m;
    cpg_initial_model(&m);
    SynthTables t;
    for (int isl = 0; isl < 2; ++isl)
        for (int p = 0; p < 4; ++p) {
            int row = isl ? p : p + 4, c0 = isl ? 0 : 4;
            double s = 0.0;
            for (int b = 0; b < 4; ++b) s += m.a[row][c0 + b];
            double c = 0.0;
            for (int b = 0; b < 4; ++b) {
                c += m.a[row][c0 + b] / s;
                t.cdf[isl][p][b] = c;
            }
            t.cdf[isl][p][3] = 1.0;
        }
    return t;
}

void synth_segment(uint64_t seed, int64_t seg, const SynthTables& T, uint8_t* base,
                   uint8_t* sign) {
    Rng r(seed, (uint64_t)seg);
    auto geom = [&]() {   // Geometric(mean kMeanGap)
        double u = r.uni();
        return (int64_t)std::floor(std::log1p(-u) / std::log1p(-1.0 / kMeanGap));
    };
    int prev = (int)(r.next() & 3);
    int64_t gap = geom(), left = 0;
    for (int64_t i = 0; i < kSeg; ++i) {
        int isl = 0;
        if (left > 0) {
            isl = 1;
            --left;
        } else if (gap-- <= 0) {
            left = 300 + (int64_t)(r.next() % 2701) - 1;   // U[300,3000]
            gap = geom();
            isl = 1;
        }
        double u = r.uni();
        const double* c = T.cdf[isl][prev];
        int b = (u < c[0]) ? 0 : (u < c[1]) ? 1 : (u < c[2]) ? 2 : 3;
        if (i == 0) b = prev;
        base[i] = (uint8_t)b;
        sign[i] = (uint8_t)isl;
        prev = b;
    }
}
}  // namespace

int cpg_synth(uint64_t seed, int64_t start, int64_t n, uint32_t* packed, uint32_t* sign_bits,
              int nthreads) {
    if (!packed || n < 0 || start < 0 || (start & 31))
        return set_error(CPG_E_INVALID, "cpg_synth: bad argument (start %% 32 == 0)");
    if (n == 0) return CPG_OK;
    static const SynthTables T = make_tables();
    const int64_t s0 = start / kSeg, s1 = (start + n - 1) / kSeg;
    const int64_t nseg = s1 - s0 + 1;
    int nt = nthreads > 0 ? nthreads : (int)std::thread::hardware_concurrency();
    if (nt > 64) nt = 64;
    if (nt < 1) nt = 1;
    if (nt > nseg) nt = (int)nseg;
    std::memset(packed, 0, (size_t)((n + 15) / 16) * 4);
    if (sign_bits) std::memset(sign_bits, 0, (size_t)((n + 31) / 32) * 4);
    auto work = [&](int tid) {
        std::vector<uint8_t> b(kSeg), g(kSeg);
        for (int64_t s = s0 + tid; s <= s1; s += nt) {
            synth_segment(seed, s, T, b.data(), g.data());
            int64_t lo = std::max(start, s * kSeg), hi = std::min(start + n, (s + 1) * kSeg);
            // segment boundaries are multiples of 32 relative to start: words never shared
            for (int64_t p = lo; p < hi; ++p) {
                int64_t q = p - start;
                packed[q >> 4] |= (uint32_t)b[p - s * kSeg] << ((q & 15) * 2);
                if (sign_bits && g[p - s * kSeg]) sign_bits[q >> 5] |= 1u << (q & 31);
            }
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    return CPG_OK;
}

// Reducer: MAHOUT-627 sums the mapper stripes and row-normalises (unvendored; :200-203).
int cpg_bw_normalize(const cpg_counts_f64* c, cpg_model* out) {
    if (!c || !out) return set_error(CPG_E_INVALID, "null argument");
    double s = 0.0;
    for (int i = 0; i < 8; ++i) s += c->init[i];
    for (int i = 0; i < 8; ++i) out->pi[i] = c->init[i] / s;
    for (int i = 0; i < 8; ++i) {
        double r = 0.0, e = 0.0;
        for (int j = 0; j < 8; ++j) r += c->trans[i][j];
        for (int j = 0; j < 8; ++j) out->a[i][j] = c->trans[i][j] / r;
        for (int k = 0; k < 4; ++k) e += c->emit[i][k];
        for (int k = 0; k < 4; ++k) out->b[i][k] = c->emit[i][k] / e;
    }
    return CPG_OK;
}

int cpg_counts_normalize(const cpg_counts_i64* c, cpg_model* out) {
    if (!c || !out) return set_error(CPG_E_INVALID, "null argument");
    cpg_counts_f64 f;
    std::memset(&f, 0, sizeof f);
    for (int i = 0; i < 8; ++i) f.init[i] = (double)c->init[i];
    for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j) f.trans[i][j] = (double)c->trans[i][j];
    for (int i = 0; i < 8; ++i)
        for (int k = 0; k < 4; ++k) f.emit[i][k] = (double)c->emit[i][k];
    return cpg_bw_normalize(&f, out);
}

}  // extern "C"
