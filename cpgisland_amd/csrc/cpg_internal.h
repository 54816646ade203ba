// cpg_internal.h — shared declarations of libcpg.so (host side + kernel launchers).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <string>

#include "../../include/cpg.h"

namespace cpg {

// ---- error state (thread-local message behind cpg_last_error) ---------------------
int set_error(int code, const char* fmt, ...);
#define CPG_HIP(expr)                                                                  \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess)                                                          \
            return ::cpg::set_error(CPG_E_DEVICE, "%s failed: %s (%s:%d)", #expr,      \
                                    hipGetErrorString(e_), __FILE__, __LINE__);        \
    } while (0)

// ---- geometry ----------------------------------------------------------------------
constexpr int kSB = 256;            // Viterbi sub-block: positions per lane
constexpr int kSBWords = kSB / 16;  // packed words per sub-block

// Device status word bits (ctx->d_status), collected by cpg_sync.
enum : uint32_t {
    ST_VERIFY_ENTRY = 1u << 0,   // K5 exit value != K4 entry of the next block
    ST_VERIFY_MAG = 1u << 1,     // K3 composite outside the exact range
    ST_VERIFY_CHAIN = 1u << 2,   // K7 traceback start state mismatch
    ST_CONTIG_LAYOUT = 1u << 3,  // a contig breaks the batch layout contract (skipped)
    // (bits 4 and 5 reported the bounded look-back spins of rounds 2-5: no kernel waits for
    // another workgroup any more)
    ST_GEN_NOT_SIGN = 1u << 6,       // general-model path: a state is not its base's (the path
                                     // is not representable as sign bits)
};

// ---- Viterbi constants (host-computed, shared by every kernel) ---------------------
constexpr int kMaxBinade = 64;
struct IslFuse;   // a fused decode's island state (isl_dev.h)

struct VitConsts {
    double L[16][4];        // per dinucleotide d = p | b<<2: log a for +->+, -->+, +->-, -->-
    double logpi[8];
    int32_t Q[16][4];       // fixed-point L * 2^qshift (rounded)
    int qshift;
    double eps;             // bound |approx - exact| on every value of a chunk
    double spread;          // 2*|min L|: lower slack inside a block
    int emin, emax;         // binades with exact tables
    uint64_t tie_mask;      // binade e has a rounding tie -> never regular
};
// the general-model Viterbi's constants (k_vit_general.hip): Math.log of every model entry
// Mahout's loop takes the log of, computed on the host (C library log, as the oracle's)
struct GenConsts {
    double L[8][8];     // log a[j][i]
    double LB[8][4];    // log b[i][k]
    double LP[8][4];    // log(pi[i] * b[i][k])
};
// per-binade rounded constants Le[e][16][4], e in [0, kMaxBinade)
struct VitTables {
    double Le[kMaxBinade][16][4];
};

// Block plan (K2 -> K3/K4)
enum : int8_t { PLAN_REGULAR = 0, PLAN_SPLIT = 1, PLAN_SEQ = 2, PLAN_DEGEN = 3 };
struct __attribute__((aligned(8))) VitPlan {
    int8_t type;
    int8_t e_pre;
    int8_t e_post;
    int8_t pad;
    uint16_t t1;     // offset (in steps from block's first step) where the window starts
    uint16_t t2;     // offset where the post composite starts
};

// ---- last-workgroup finalize (device) ----------------------------------------------
// The accumulating kernels (counts, E-step) fold their one-workgroup finalize into the main
// launch: every workgroup's accumulator atomics are device-scope RMWs (performed at the
// device coherence point, past the XCD-private L2s) and have completed once the workgroup has
// drained its memory counters; then thread 0 counts the workgroup in, and the workgroup that
// counts last reads the accumulators with device-scope loads.  No L2 writeback fence is
// needed (the only data exchanged is atomics): a release per workgroup would write back the
// XCD's L2, including what concurrent kernels on the other stream have written.
// The count is two-level: one device-scope word takes ~88 returning atomics per us, so 512
// workgroups finishing together would queue ~6 us on a single counter; workgroup b counts
// into group word b % kDoneGroups, and the last of each group into the top word
// done[kDoneGroups].  The finalizer re-zeroes all of them (kDoneWords u32 of workspace).
constexpr int kDoneGroups = 16;
constexpr int kDoneWords = kDoneGroups + 1;
#ifdef __HIPCC__
__device__ __forceinline__ bool last_workgroup(unsigned int* done, int* s_flag) {
    __builtin_amdgcn_s_waitcnt(0);   // this wave's atomics have completed
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned G = gridDim.x, g = blockIdx.x % kDoneGroups;
        const unsigned gsize = (G - g + kDoneGroups - 1) / kDoneGroups;
        bool last = false;
        if (__hip_atomic_fetch_add(done + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            gsize - 1) {
            const unsigned ngroups = G < kDoneGroups ? G : kDoneGroups;
            last = __hip_atomic_fetch_add(done + kDoneGroups, 1u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT) == ngroups - 1;
        }
        *s_flag = last;
    }
    __syncthreads();
    return *s_flag != 0;
}
__device__ __forceinline__ void reset_done(unsigned int* done) {
    if (threadIdx.x < kDoneWords)
        __hip_atomic_store(done + threadIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long load_agent(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The E-step's 128-bit fixed-point accumulators (k_estep.hip, k_contigs.hip) as SPLIT sums:
// a slot pair (w0, w1) accumulates the low 32 bits of each addend in w0 and the rest (the
// addend >> 32, two's complement) in w1, so the value is w1 * 2^32 + w0 — two non-returning
// 64-bit atomics per addend, no carry to wait for (a returning atomic's round trip had been
// most of the E-step's epilogue).  No overflow: w0 gains < 2^32 per addend (< 2^48 for 2^16
// addends per replica), |w1| < 2^63 for sums below 2^95.  acc_sum128 is the finalize's side.
__device__ __forceinline__ void acc_split_add(unsigned long long* w, unsigned long long lo,
                                              unsigned long long hi) {   // addend = hi 2^64 + lo
    const unsigned long long p0 = lo & 0xFFFFFFFFull, p1 = (lo >> 32) | (hi << 32);
    if (p0) atomicAdd(w, p0);
    if (p1) atomicAdd(w + 1, p1);
}
// sum of (w0, w1) pairs, as a 128-bit two's complement value (lo, hi)
__device__ __forceinline__ void acc_sum128(unsigned long long s0, unsigned long long s1,
                                           unsigned long long& lo, unsigned long long& hi) {
    lo = (s1 << 32) + s0;
    hi = (unsigned long long)((long long)s1 >> 32) + (lo < s0 ? 1ull : 0ull);
}
#endif

// ---- context -----------------------------------------------------------------------
struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
};

// ---- workspace slots (cpg_ctx::ws) ------------------------------------------------
enum { WS_COUNT = 0, WS_VIT = 1, WS_ISL = 2, WS_EST = 3, WS_IN0 = 4, WS_IN1 = 5, WS_OUT0 = 6,
       WS_OUT1 = 7, WS_OUT2 = 8, WS_ING = 9, WS_GEN = 10, WS_GISL = 11, WS_CSORT = 12,
       WS_CBP = 13, WS_CISL = 14, WS_CCK = 15,
       // K1's segment products (read by the next launch, k_vit_segplan); 17: unused (the
       // island look-back flags of rounds 2-5)
       WS_VAGG = 16,
       // per-chunk done counters of the fused decode: zero between calls (zero-filled when
       // allocated, reset by the workgroup that completes a chunk), so a slot of their own
       WS_IDONE = 18,
       // the general-model Viterbi (backpointer ballots, states, state-packed words)
       WS_VGEN = 19, WS_NSLOT = 20 };

}  // namespace cpg

struct cpg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    uint32_t* d_status = nullptr;     // device status word
    // workspace (grown on demand; cpg_reserve pre-sizes)
    cpg::Buf ws[cpg::WS_NSLOT];
    // host staging (pinned)
    cpg::Buf pin[4];
    // device copies of per-model Viterbi tables
    static constexpr int kVtSlots = 4;
    struct VtSlot {
        cpg_model model;
        cpg::VitTables* d;
    } vtc[kVtSlots];
    int vtn = 0, vtnext = 0;
    // device copies of per-model E-step one-step tables (rows TA | TB, 32 x double2)
    struct EtSlot {
        cpg_model model;
        double2* d;
    } etc_[kVtSlots];
    int etn = 0, etnext = 0;
    // streamed-genome pipeline (cpg_genome_run): copy-in, train, decode, copy-out streams
    // and per-buffer events, created on first use
    hipStream_t ps[4] = {};
    static constexpr int kMaxBuf = 8;
    hipEvent_t pev[4 * kMaxBuf] = {};
};

namespace cpg {
int ws_get(cpg_ctx* ctx, int slot, size_t bytes, void** out);
int pin_get(cpg_ctx* ctx, int slot, size_t bytes, void** out);
int model_check_deterministic(const cpg_model* m);
bool aligned16(const void* p);
int vit_tables(cpg_ctx* ctx, const cpg_model* m, const VitConsts& vc, const VitTables& vt,
               const VitTables** out);
int est_tables(cpg_ctx* ctx, const cpg_model* m, const double2** out);
int vit_prepare(const cpg_model* m, int64_t chunk_len, VitConsts* vc, VitTables* vt);
// the exact parallel Viterbi's model contract (deterministic emissions, 0 < a <= 1,
// 0 <= pi <= 1); models outside it decode through the general path
bool vit_fast_ok(const cpg_model* m);
void gen_prepare(const cpg_model* m, GenConsts* gc);

// kernel launchers (defined in the .hip files); all asynchronous on `s`
// parts: bit 0 = accumulate the chunks into the context's fixed-point accumulators, bit 1 =
// finalize (convert to the output struct and re-zero).  A streamed genome accumulates every
// window and finalizes once: bit-identical to one call over the whole genome.
enum { PART_ACC = 1, PART_FINAL = 2, PART_ALL = 3 };
hipError_t launch_count(const uint32_t* packed, const uint32_t* sign, int64_t nchunks,
                        int64_t chunk_len, uint64_t* ws, int64_t* out /*124*/, hipStream_t s,
                        int parts = PART_ALL);
size_t count_ws_bytes(int64_t nchunks);
hipError_t launch_viterbi(const VitConsts& vc, const VitTables* d_vt, const uint32_t* packed,
                          int64_t nchunks, int64_t chunk_len, void* ws, size_t ws_bytes,
                          uint32_t* sign_out, double* score, uint8_t* degen,
                          uint32_t* status, hipStream_t s, unsigned long long* agg,
                          uint32_t* zero_at = nullptr, int64_t zero_n = 0,
                          const IslFuse* fuse = nullptr,    // fused decode: K7 resolves
                          unsigned int* done5 = nullptr);   // nchunks zeroed words: K5 runs K6
size_t viterbi_ws_bytes(int64_t nchunks, int64_t chunk_len);
// the general-model Viterbi (any model: k_vit_general.hip): states_out (nchunks * C bytes, or
// the workspace when null), score (may be null), sign_out (state < 4; may be null), *spk_out
// (state & 3 in the packed layout, in the workspace; may be null); check_sign: status bit
// ST_GEN_NOT_SIGN when a state is not its position's base (state & 3 != base)
size_t vitg_ws_bytes(int64_t nchunks, int64_t C);
hipError_t launch_vitg(const GenConsts& gc, const uint32_t* packed, int64_t nchunks, int64_t C,
                       void* ws, size_t ws_bytes, uint8_t* states_out, double* score,
                       uint32_t* sign_out, uint32_t** spk_out, uint32_t* status,
                       bool check_sign, hipStream_t s);
size_t viterbi_agg_bytes(int64_t nchunks, int64_t chunk_len);   // WS_VAGG
// model-derived LDS tables of K1/K3, built once per model right after the VitTables copy
size_t vit_derived_bytes();
hipError_t launch_vit_tables(const VitConsts& vc, VitTables* d_vt, hipStream_t s);
int64_t vit_nsb(int64_t chunk_len);
hipError_t launch_islands(const uint32_t* packed, const uint32_t* sign, int64_t nchunks,
                          int64_t chunk_len, int64_t first_chunk, void* ws, size_t ws_bytes,
                          cpg_island* out, int64_t cap, int64_t* count, hipStream_t s,
                          const int64_t* base_in = nullptr);
size_t islands_ws_bytes(int64_t nchunks, int64_t chunk_len);
// fused decode (cpg_decode_d): the traceback writes the island tile lists and a chunk's last
// traceback workgroup runs the chunk's first resolve pass (done: nchunks zeroed words,
// WS_IDONE); islands_write places the records after it (no island tile / resolve kernels)
bool islands_fusable(int64_t nchunks, int64_t chunk_len);
// Per-chunk tail work folded into the last workgroup of a chunk (K6 into K5, the island tiles
// and the chunk resolve into K7) pays while the chunks are few: it saves a launch and the
// grid-wide boundary, and the tails run on an otherwise draining GPU.  With many chunks the
// GPU is full when each tail runs, so a latency-bound tail shares a busy CU: at 2,956 chunks
// (3.1 Gbp) K5 + K6 as two launches took 1,269 against 1,365 us and the separate traceback +
// tile + resolve kernels 648 against 1,013 us (decode 3.735 against 4.040 ms); at 43 chunks
// the fused decode is 4 % faster, at 256 they are equal, at 1,024 the separate one 3 %
// faster (profiles/r04_dec2/).  One chunk per compute unit is the crossover.
constexpr int64_t kTailFuseMaxChunks = 256;
inline bool tail_fusion_pays(int64_t nchunks) { return nchunks <= kTailFuseMaxChunks; }
hipError_t islands_fuse(IslFuse* f, void* ws, size_t ws_bytes, int64_t nchunks,
                        int64_t chunk_len, int64_t first_chunk, cpg_island* out, int64_t cap,
                        int64_t* count, unsigned int* done, const int64_t* base_in = nullptr);
hipError_t islands_write(const uint32_t* packed, const IslFuse& f, int64_t chunk_len,
                         hipStream_t s);
// the fused decode past kTailFuseMaxChunks chunks: the traceback writes the island tiles
// (IslFuse with done == null) and islands_resolve runs both resolve passes after it
hipError_t islands_tiles(IslFuse* f, void* ws, size_t ws_bytes, int64_t nchunks,
                         int64_t chunk_len, int64_t first_chunk, cpg_island* out, int64_t cap,
                         int64_t* count, const int64_t* base_in = nullptr);
hipError_t islands_resolve(const uint32_t* packed, const IslFuse& f, int64_t chunk_len,
                           hipStream_t s);
// gtab: the model's one-step tables in device memory (est_tables); needed with PART_ACC
hipError_t launch_estep(const cpg_model& model, const uint32_t* packed, int64_t nchunks,
                        int64_t chunk_len, unsigned long long* acc, double* out,
                        hipStream_t s, int parts = PART_ALL, const double2* gtab = nullptr);
size_t estep_ws_bytes(int64_t nchunks, int64_t chunk_len);
// the reducer over ranks: gathered records -> summed outputs (k_reduce.hip)
hipError_t launch_merge_train(const void* gathered, int world, double* estep, int64_t* counts,
                              hipStream_t s);
// the fused training pass (E-step + labelled counts in one launch; k_estep.hip)
bool train_fusable(int64_t chunk_len);
hipError_t launch_train(const cpg_model& model, const uint32_t* packed, const uint32_t* sign,
                        int64_t nchunks, int64_t chunk_len, unsigned long long* acc, double* out,
                        unsigned long long* cacc, int64_t* cout, hipStream_t s,
                        const double2* gtab);

// ragged contig batches (k_contigs.hip)
size_t contigs_sort_ws_bytes(int64_t n);
hipError_t launch_contigs_order(const int32_t* lens, int64_t n, int32_t* order, void* ws,
                                size_t ws_bytes, hipStream_t s);
hipError_t launch_contigs_count(const uint32_t* packed, const uint32_t* sign, int64_t nbases,
                                const int64_t* offs, const int32_t* lens, const int32_t* order,
                                int64_t n, uint64_t* ws, int64_t* out, uint32_t* status,
                                hipStream_t s);
hipError_t launch_contigs_viterbi(const VitConsts& vc, const uint32_t* packed, int64_t nbases,
                                  const int64_t* offs, const int32_t* lens, const int32_t* order,
                                  int64_t n, uint32_t* bp, uint32_t* sign_out, double* score,
                                  uint32_t* status, hipStream_t s);
hipError_t launch_contigs_estep(const cpg_model& model, const uint32_t* packed, int64_t nbases,
                                const int64_t* offs, const int32_t* lens, const int32_t* order,
                                int64_t n, void* ck, unsigned long long* acc, double* out,
                                uint32_t* status, hipStream_t s);
hipError_t launch_contigs_islands(const uint32_t* packed, const uint32_t* sign, int64_t nbases,
                                  const int64_t* offs, const int32_t* lens, const int32_t* order,
                                  int64_t n, void* ws, size_t ws_bytes, cpg_island* out,
                                  int64_t cap, int64_t* count, uint32_t* status, hipStream_t s);

// count0: the Java `count` before the first byte (0; the test hooks below: a chunk multiple)
hipError_t launch_ingest(const uint8_t* txt, int64_t n, int mode, int quirks, int64_t chunk,
                         uint32_t* out, int64_t cap, void* ws, size_t ws_bytes,
                         long long* res, hipStream_t s, uint32_t count0 = 0);
size_t ingest_ws_bytes(int64_t n);

}  // namespace cpg

// Test hooks, exported but not part of the C-ABI (include/cpg.h): the readers of cpg_ingest /
// cpg_ingest_gpu started from Java `count` = count0 (a multiple of the chunk below 2^32) with
// an empty list, so that the int counter's wrap at 2^32 bases (:127, :253) is reached with a
// few MB of text (tests/test_ingest_wrap.py, tests/test_gpu_ingest.py).
extern "C" {
int cpgx_ingest_at(const char* txt, size_t n, int mode, int compat_quirks, uint32_t* packed,
                   int64_t cap_bases, int64_t* nbases, uint32_t count0);
int cpgx_ingest_gpu_at(cpg_ctx* ctx, const char* txt, size_t n, int mode, int compat_quirks,
                       uint32_t* packed, int64_t cap_bases, int64_t* nbases, uint32_t count0);
}
