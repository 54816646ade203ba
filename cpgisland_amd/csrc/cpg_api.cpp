// cpg_api.cpp — the C-ABI of libcpg.so (include/cpg.h): context, device workspace,
// the HBM-resident "_d" entry points and the host-buffer wrappers that mirror the
// reference call sites (CpGIslandFinder.java:200 training, :260 decode, :262-339 islands).

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <vector>

#include <atomic>

#include "cpg_internal.h"
#include "isl_dev.h"

namespace cpg {

int ws_get(cpg_ctx* ctx, int slot, size_t bytes, void** out) {
    Buf& b = ctx->ws[slot];
    if (b.bytes < bytes) {
        // the whole device, not only the context's stream: calls run on callers' streams
        // (torch streams, the streamed genome's non-blocking streams), and a kernel still
        // reading the old buffer there must finish before it is freed
        if (b.p) {
            CPG_HIP(hipDeviceSynchronize());
            CPG_HIP(hipFree(b.p));
            b.p = nullptr;
            b.bytes = 0;
        }
        size_t sz = bytes + bytes / 8 + 4096;
        CPG_HIP(hipMalloc(&b.p, sz));
        // zero-filled once: the count / E-step accumulators rely on it (their final kernels
        // re-zero them after reading); the fill is on the null stream, which non-blocking
        // streams do not wait for: wait for it here
        CPG_HIP(hipMemset(b.p, 0, sz));
        CPG_HIP(hipDeviceSynchronize());
        b.bytes = sz;
    }
    *out = b.p;
    return CPG_OK;
}

int pin_get(cpg_ctx* ctx, int slot, size_t bytes, void** out) {
    Buf& b = ctx->pin[slot];
    if (b.bytes < bytes) {
        if (b.p) {
            CPG_HIP(hipStreamSynchronize(ctx->stream));
            CPG_HIP(hipHostFree(b.p));
            b.p = nullptr;
            b.bytes = 0;
        }
        CPG_HIP(hipHostMalloc(&b.p, bytes, hipHostMallocDefault));
        b.bytes = bytes;
    }
    *out = b.p;
    return CPG_OK;
}

namespace {


// NULL is the HIP null stream (torch's default stream handle is 0 too); the host-buffer
// wrappers pass the context's own stream explicitly
hipStream_t pick(cpg_ctx*, void* stream) { return static_cast<hipStream_t>(stream); }

}  // namespace

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// device copy of the per-binade tables of one model (model-only; cached per context)
int vit_tables(cpg_ctx* ctx, const cpg_model* m, const VitConsts& vc, const VitTables& vt,
               const VitTables** out) {
    for (int i = 0; i < ctx->vtn; ++i)
        if (std::memcmp(&ctx->vtc[i].model, m, sizeof *m) == 0) {
            *out = ctx->vtc[i].d;
            return CPG_OK;
        }
    cpg_ctx::VtSlot* sl;
    if (ctx->vtn < cpg_ctx::kVtSlots) {
        sl = &ctx->vtc[ctx->vtn++];
        CPG_HIP(hipMalloc(&sl->d, sizeof(VitTables) + vit_derived_bytes()));
    } else {
        sl = &ctx->vtc[ctx->vtnext];
        ctx->vtnext = (ctx->vtnext + 1) % cpg_ctx::kVtSlots;
        CPG_HIP(hipDeviceSynchronize());   // the evicted slot may still be read
    }
    std::memset(&sl->model, 0xFF, sizeof sl->model);   // NaN bytes: no model matches a half-built slot
    CPG_HIP(hipMemcpy(sl->d, &vt, sizeof(VitTables), hipMemcpyHostToDevice));
    // K1's 4-step and K3's per-binade tables, computed once here instead of by every
    // workgroup of every call (they depend on the model only: qshift and Le do)
    CPG_HIP(launch_vit_tables(vc, sl->d, nullptr));
    CPG_HIP(hipStreamSynchronize(nullptr));
    sl->model = *m;
    *out = sl->d;
    return CPG_OK;
}

// the E-step's tables, cached per model like the Viterbi tables: one-step rows
// TA[d] = (a[p][b], a[p][b+4]), TB[d] = (a[p+4][b], a[p+4][b+4]) for d = p | b << 2 (p the
// previous base, b the current one); then the two-step rows of the trinucleotide keys
// tau = x0 | x1 << 2 | x2 << 4, P_tau = M_{x0 x1} M_{x1 x2} (T2A: row +, T2B: row -), and
// keys 64 + d = the one-step M_d (k_estep.hip 3b) — written once per model
constexpr int kEstKeys = 80;
constexpr int kEstTabRows = 32 + 2 * kEstKeys;
int est_tables(cpg_ctx* ctx, const cpg_model* m, const double2** out) {
    for (int i = 0; i < ctx->etn; ++i)
        if (std::memcmp(&ctx->etc_[i].model, m, sizeof *m) == 0) {
            *out = ctx->etc_[i].d;
            return CPG_OK;
        }
    cpg_ctx::EtSlot* sl;
    if (ctx->etn < cpg_ctx::kVtSlots) {
        sl = &ctx->etc_[ctx->etn++];
        CPG_HIP(hipMalloc(&sl->d, kEstTabRows * sizeof(double2)));
    } else {
        sl = &ctx->etc_[ctx->etnext];
        ctx->etnext = (ctx->etnext + 1) % cpg_ctx::kVtSlots;
        CPG_HIP(hipDeviceSynchronize());   // the evicted slot may still be read
    }
    double2 h[kEstTabRows];
    auto M = [&](int d, int s, int s2) { return m->a[(d & 3) + 4 * s][(d >> 2) + 4 * s2]; };
    for (int d = 0; d < 16; ++d) {
        h[d] = make_double2(M(d, 0, 0), M(d, 0, 1));
        h[16 + d] = make_double2(M(d, 1, 0), M(d, 1, 1));
    }
    for (int k = 0; k < kEstKeys; ++k) {
        double P[2][2];
        for (int s = 0; s < 2; ++s)
            for (int s2 = 0; s2 < 2; ++s2) {
                if (k >= 64) {
                    P[s][s2] = M(k - 64, s, s2);
                } else {
                    const int d1 = k & 15, d2 = k >> 2;
                    P[s][s2] = M(d1, s, 0) * M(d2, 0, s2) + M(d1, s, 1) * M(d2, 1, s2);
                }
            }
        h[32 + k] = make_double2(P[0][0], P[0][1]);
        h[32 + kEstKeys + k] = make_double2(P[1][0], P[1][1]);
    }
    sl->model = *m;
    CPG_HIP(hipMemcpy(sl->d, h, sizeof(double2) * kEstTabRows, hipMemcpyHostToDevice));
    *out = sl->d;
    return CPG_OK;
}

namespace {

// the general-model Viterbi (k_vit_general.hip) over nch whole chunks of C bases
int vit_general(cpg_ctx* ctx, const cpg_model* model, const uint32_t* d_packed, int64_t nch,
                int64_t C, uint8_t* d_states, double* d_score, uint32_t* d_sign, uint32_t** spk,
                bool check_sign, hipStream_t s) {
    if (nch > 1 && C % 16)
        return set_error(CPG_E_INVALID, "chunk_len must be a multiple of 16 for >1 chunk");
    GenConsts gc;
    gen_prepare(model, &gc);
    void* ws;
    int rc;
    if ((rc = ws_get(ctx, WS_VGEN, vitg_ws_bytes(nch, C), &ws))) return rc;
    CPG_HIP(launch_vitg(gc, d_packed, nch, C, ws, ctx->ws[WS_VGEN].bytes, d_states, d_score,
                        d_sign, spk, ctx->d_status, check_sign, s));
    return CPG_OK;
}

int check_layout(const void* packed, int64_t nbases, int64_t chunk_len) {
    if (!packed && nbases > 0) return set_error(CPG_E_INVALID, "null packed buffer");
    if (nbases < 0 || chunk_len <= 0)
        return set_error(CPG_E_INVALID, "nbases=%lld chunk_len=%lld", (long long)nbases,
                         (long long)chunk_len);
    if (!aligned16(packed)) return set_error(CPG_E_INVALID, "packed buffer not 16-byte aligned");
    return CPG_OK;
}

}  // namespace
}  // namespace cpg

using namespace cpg;

extern "C" {

int cpg_open(int device, cpg_ctx** out) {
    if (!out) return set_error(CPG_E_INVALID, "null out");
    *out = nullptr;
    // Kernel arguments in device memory instead of host memory: every kernel's first
    // argument fetch otherwise crosses PCIe (measured ~1 us per launch on MI355X).  Takes
    // effect only if this is the process's first HIP call (e.g. a JVM host); Python hosts
    // that initialise HIP through torch first set it in the environment (bench.py).
    setenv("HIP_FORCE_DEV_KERNARG", "1", 0);
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0)
        return set_error(CPG_E_DEVICE, "no HIP device available (%s)", hipGetErrorString(e));
    if (device < 0 || device >= n) return set_error(CPG_E_INVALID, "device %d of %d", device, n);
    CPG_HIP(hipSetDevice(device));
    cpg_ctx* ctx = new cpg_ctx();
    ctx->device = device;
    CPG_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
    CPG_HIP(hipMalloc(&ctx->d_status, 256));
    CPG_HIP(hipMemset(ctx->d_status, 0, 256));
    *out = ctx;
    return CPG_OK;
}

void cpg_close(cpg_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    for (auto& b : ctx->ws)
        if (b.p) (void)hipFree(b.p);
    for (auto& b : ctx->pin)
        if (b.p) (void)hipHostFree(b.p);
    if (ctx->d_status) (void)hipFree(ctx->d_status);
    for (int i = 0; i < ctx->vtn; ++i) (void)hipFree(ctx->vtc[i].d);
    for (int i = 0; i < ctx->etn; ++i) (void)hipFree(ctx->etc_[i].d);
    for (auto& ps : ctx->ps)
        if (ps) (void)hipStreamDestroy(ps);
    for (auto& ev : ctx->pev)
        if (ev) (void)hipEventDestroy(ev);
    (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int cpg_reserve(cpg_ctx* ctx, int64_t nbases) { return cpg_reserve_ex(ctx, nbases, 0); }

// the workspace every entry point needs for inputs of up to nbases bases, at the decode chunk
// lengths C in [c_lo, c_hi] stepping c_step (host arithmetic only)
static int reserve_lengths(cpg_ctx* ctx, int64_t nbases, int flags, int64_t c_lo, int64_t c_hi,
                           int64_t c_step) {
    void* p;
    int rc;
    size_t vit = 0, isl = 0, agg = 0, per_chunk = 0;
    for (int64_t C = c_lo; C <= c_hi; C += c_step) {
        const int64_t nd = nbases / C + 1;
        // (the Viterbi: several chunks of a multiple of 256, or one chunk of any length)
        const int64_t ndv = C % 256 == 0 ? nd : 1;
        vit = std::max(vit, viterbi_ws_bytes(ndv, C));
        agg = std::max(agg, viterbi_agg_bytes(ndv, C));
        isl = std::max(isl, islands_ws_bytes(nd, C));
        per_chunk = std::max(per_chunk, (size_t)(nd + 1) * 8);
    }
    const int64_t nt = nbases / 256 + 1;
    if ((rc = ws_get(ctx, WS_COUNT, count_ws_bytes(nt), &p))) return rc;
    if ((rc = ws_get(ctx, WS_VIT, vit, &p))) return rc;
    if ((rc = ws_get(ctx, WS_ISL, isl, &p))) return rc;
    if ((rc = ws_get(ctx, WS_VAGG, agg, &p))) return rc;
    if ((rc = ws_get(ctx, WS_IDONE, per_chunk, &p))) return rc;
    if ((rc = ws_get(ctx, WS_EST, estep_ws_bytes(nt, CPG_TRAIN_CHUNK), &p))) return rc;
    if (flags & CPG_RESERVE_GENERAL) {
        // the general path: any chunk length that is a multiple of 16 (several chunks) or the
        // whole input as one chunk (cpg_decode_states); its ballots are sized per group of 8
        // chunks, so the largest need is at long chunks
        size_t gen = vitg_ws_bytes(1, std::max<int64_t>(nbases, 1));
        for (int64_t C = 16; C <= CPG_DECODE_CHUNK && C <= nbases; C += 16)
            gen = std::max(gen, vitg_ws_bytes(nbases / C, C));
        if ((rc = ws_get(ctx, WS_VGEN, gen, &p))) return rc;
    }
    return CPG_OK;
}

int cpg_reserve_ex(cpg_ctx* ctx, int64_t nbases, int flags) {
    if (!ctx || nbases < 0 || (flags & ~CPG_RESERVE_GENERAL))
        return set_error(CPG_E_INVALID, "bad argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    CPG_HIP(hipSetDevice(ctx->device));
    // every slot at its largest over ALL the chunk lengths the decode entry points take in
    // whole 256-base blocks (every multiple of 256 up to the reference's 1 Mi — a
    // non-power-of-two length takes another carve): the per-chunk slots grow with the chunk
    // count, so a reserve for 1 Mi chunks alone would still let a later call with shorter
    // chunks grow a slot (a device-wide synchronisation, ws_get)
    return reserve_lengths(ctx, nbases, flags, 256, CPG_DECODE_CHUNK, 256);
}

int cpg_reserve_chunk(cpg_ctx* ctx, int64_t nbases, int64_t chunk_len, int flags) {
    if (!ctx || nbases < 0 || chunk_len <= 0 || chunk_len % 32 || (flags & ~CPG_RESERVE_GENERAL))
        return set_error(CPG_E_INVALID, "bad argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    CPG_HIP(hipSetDevice(ctx->device));
    return reserve_lengths(ctx, nbases, flags, chunk_len, chunk_len, 1);
}

int cpg_workspace_bytes(cpg_ctx* ctx, int64_t* bytes) {
    if (!ctx || !bytes) return set_error(CPG_E_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    int64_t t = 0;
    for (const auto& b : ctx->ws) t += (int64_t)b.bytes;
    *bytes = t;
    return CPG_OK;
}

int cpg_stream_create_cu(int device, const uint32_t* cu_mask, int mask_words, void** out) {
    if (!out || !cu_mask || mask_words <= 0) return set_error(CPG_E_INVALID, "null argument");
    *out = nullptr;
    CPG_HIP(hipSetDevice(device));
    hipStream_t s;
    CPG_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask_words, cu_mask));
    *out = s;
    return CPG_OK;
}

int cpg_stream_destroy(void* stream) {
    if (!stream) return set_error(CPG_E_INVALID, "null stream");
    CPG_HIP(hipStreamDestroy(static_cast<hipStream_t>(stream)));
    return CPG_OK;
}

int cpg_sync(cpg_ctx* ctx, void* stream) {
    if (!ctx) return set_error(CPG_E_INVALID, "null ctx");
    CPG_HIP(hipSetDevice(ctx->device));
    hipStream_t s = pick(ctx, stream);
    uint32_t st = 0;
    CPG_HIP(hipMemcpyAsync(&st, ctx->d_status, 4, hipMemcpyDeviceToHost, s));
    CPG_HIP(hipStreamSynchronize(s));
    if (st) {
        CPG_HIP(hipMemsetAsync(ctx->d_status, 0, 4, s));
        CPG_HIP(hipStreamSynchronize(s));
        if (st & ST_GEN_NOT_SIGN)
            return set_error(CPG_E_UNSUPPORTED,
                             "viterbi (general model): the decoded path visits states that are "
                             "not their position's base (a dead end of zero transitions); sign "
                             "bits cannot carry it: use cpg_viterbi_states_d (status 0x%x)", st);
        if (st == ST_CONTIG_LAYOUT)
            return set_error(CPG_E_INVALID,
                             "contig batch: a contig breaks the layout contract (offset %% 64, "
                             "length >= 1 (<= 2^20 for the E-step), inside nbases); skipped");
        return set_error(CPG_E_VERIFY,
                         "kernel self-check failed (status 0x%x: %s%s%s%s)", st,
                         (st & ST_VERIFY_ENTRY) ? "viterbi block exit != next entry; " : "",
                         (st & ST_VERIFY_MAG) ? "composite out of exact range; " : "",
                         (st & ST_VERIFY_CHAIN) ? "traceback chain mismatch; " : "",
                         (st & ST_CONTIG_LAYOUT) ? "contig layout contract broken" : "");
    }
    return CPG_OK;
}

// ---- device entry points ----------------------------------------------------------
int cpg_count_labelled_d(cpg_ctx* ctx, const uint32_t* d_packed, const uint32_t* d_sign,
                         int64_t nbases, int64_t chunk_len, int64_t* d_counts, void* stream) {
    if (!ctx || !d_counts || (!d_sign && nbases > 0))
        return set_error(CPG_E_INVALID, "null argument");
    int rc = check_layout(d_packed, nbases, chunk_len);
    if (rc) return rc;
    if (chunk_len % 256) return set_error(CPG_E_INVALID, "chunk_len must be a multiple of 256");
    if (!aligned16(d_sign)) return set_error(CPG_E_INVALID, "sign buffer not 16-byte aligned");
    std::lock_guard<std::mutex> lk(ctx->mu);
    CPG_HIP(hipSetDevice(ctx->device));
    const int64_t nch = nbases / chunk_len;
    void* ws;
    if ((rc = ws_get(ctx, WS_COUNT, count_ws_bytes(nch), &ws))) return rc;
    CPG_HIP(launch_count(d_packed, d_sign, nch, chunk_len, (uint64_t*)ws, d_counts,
                         pick(ctx, stream)));
    return CPG_OK;
}

int cpg_viterbi_d(cpg_ctx* ctx, const cpg_model* model, const uint32_t* d_packed,
                  int64_t nbases, int64_t chunk_len, uint32_t* d_sign_out, double* d_score,
                  void* stream) {
    if (!ctx || !model || !d_sign_out) return set_error(CPG_E_INVALID, "null argument");
    int rc = check_layout(d_packed, nbases, chunk_len);
    if (rc) return rc;
    const int64_t nch = nbases / chunk_len;
    if (nch > 1 && chunk_len % 256)
        return set_error(CPG_E_INVALID, "chunk_len must be a multiple of 256 for >1 chunk");
    if (!aligned16(d_sign_out)) return set_error(CPG_E_INVALID, "sign_out not 16-byte aligned");
    std::lock_guard<std::mutex> lk(ctx->mu);
    CPG_HIP(hipSetDevice(ctx->device));
    hipStream_t s = pick(ctx, stream);
    // undecoded tail -> '-' bits (whole words past the last chunk): zeroed by the traceback
    // launch, or here when there is no chunk to decode
    const int64_t w_done = (nch * chunk_len + 31) / 32, w_all = (nbases + 31) / 32;
    const int64_t ntail = w_all > w_done ? w_all - w_done : 0;
    if (nch == 0) {
        if (ntail) CPG_HIP(hipMemsetAsync(d_sign_out + w_done, 0, (size_t)ntail * 4, s));
        return CPG_OK;
    }
    if (!vit_fast_ok(model)) {
        // outside the exact scan's contract: Mahout's 8-state loop itself (k_vit_general.hip)
        if (model_check_deterministic(model))
            return set_error(CPG_E_UNSUPPORTED,
                             "emission matrix not deterministic: the path's states are not "
                             "base + (sign ? 0 : 4), so sign bits cannot carry it; use "
                             "cpg_viterbi_states_d or cpg_decode_d");
        if ((rc = vit_general(ctx, model, d_packed, nch, chunk_len, nullptr, d_score, d_sign_out,
                              nullptr, true, s)))
            return rc;
        if (ntail) CPG_HIP(hipMemsetAsync(d_sign_out + w_done, 0, (size_t)ntail * 4, s));
        return CPG_OK;
    }
    VitConsts vc;
    static thread_local VitTables vt;
    if ((rc = vit_prepare(model, chunk_len, &vc, &vt))) return rc;
    const VitTables* d_vt;
    if ((rc = vit_tables(ctx, model, vc, vt, &d_vt))) return rc;
    void* ws;
    const size_t need = viterbi_ws_bytes(nch, chunk_len);
    if ((rc = ws_get(ctx, WS_VIT, need, &ws))) return rc;
    void* agg;
    if ((rc = ws_get(ctx, WS_VAGG, viterbi_agg_bytes(nch, chunk_len), &agg))) return rc;
    void* done;   // per-chunk counters: K5's workgroups, then (cpg_decode_d) K7's
    if ((rc = ws_get(ctx, WS_IDONE, (size_t)nch * 8, &done))) return rc;
    CPG_HIP(launch_viterbi(vc, d_vt, d_packed, nch, chunk_len, ws, ctx->ws[WS_VIT].bytes,
                           d_sign_out, d_score, nullptr, ctx->d_status, s,
                           static_cast<unsigned long long*>(agg), d_sign_out + w_done, ntail,
                           nullptr, static_cast<unsigned int*>(done)));
    return CPG_OK;
}

int cpg_islands_d(cpg_ctx* ctx, const uint32_t* d_packed, const uint32_t* d_sign,
                  int64_t nbases, int64_t chunk_len, cpg_island* d_out, int64_t cap,
                  int64_t* d_count, void* stream) {
    if (!ctx || !d_count || (cap > 0 && !d_out)) return set_error(CPG_E_INVALID, "null argument");
    int rc = check_layout(d_packed, nbases, chunk_len);
    if (rc) return rc;
    if (chunk_len % 32) return set_error(CPG_E_INVALID, "chunk_len must be a multiple of 32");
    std::lock_guard<std::mutex> lk(ctx->mu);
    CPG_HIP(hipSetDevice(ctx->device));
    const int64_t nch = nbases / chunk_len;
    void* ws;
    if ((rc = ws_get(ctx, WS_ISL, islands_ws_bytes(nch, chunk_len), &ws))) return rc;
    CPG_HIP(launch_islands(d_packed, d_sign, nch, chunk_len, 0, ws, ctx->ws[WS_ISL].bytes, d_out,
                           cap, d_count, pick(ctx, stream)));
    return CPG_OK;
}

int cpg_islands_at_d(cpg_ctx* ctx, const uint32_t* d_packed, const uint32_t* d_sign,
                     int64_t nbases, int64_t chunk_len, int64_t first_chunk, cpg_island* d_out,
                     int64_t cap, int64_t* d_count, void* stream) {
    if (!ctx || !d_count || (cap > 0 && !d_out)) return set_error(CPG_E_INVALID, "null argument");
    int rc = check_layout(d_packed, nbases, chunk_len);
    if (rc) return rc;
    if (chunk_len % 32) return set_error(CPG_E_INVALID, "chunk_len must be a multiple of 32");
    std::lock_guard<std::mutex> lk(ctx->mu);
    CPG_HIP(hipSetDevice(ctx->device));
    const int64_t nch = nbases / chunk_len;
    void* ws;
    if ((rc = ws_get(ctx, WS_ISL, islands_ws_bytes(nch, chunk_len), &ws))) return rc;
    CPG_HIP(launch_islands(d_packed, d_sign, nch, chunk_len, first_chunk, ws,
                           ctx->ws[WS_ISL].bytes, d_out, cap, d_count, pick(ctx, stream)));
    return CPG_OK;
}

int cpg_decode_d(cpg_ctx* ctx, const cpg_model* model, const uint32_t* d_packed,
                 int64_t nbases, int64_t chunk_len, int64_t first_chunk, uint32_t* d_sign_out,
                 double* d_score, cpg_island* d_out, int64_t cap, int64_t* d_count,
                 void* stream) {
    if (!ctx || !model || !d_sign_out || !d_count || (cap > 0 && !d_out))
        return set_error(CPG_E_INVALID, "null argument");
    int rc = check_layout(d_packed, nbases, chunk_len);
    if (rc) return rc;
    const int64_t nch = nbases / chunk_len;
    if (nch > 1 && chunk_len % 256)
        return set_error(CPG_E_INVALID, "chunk_len must be a multiple of 256 for >1 chunk");
    if (chunk_len % 32) return set_error(CPG_E_INVALID, "chunk_len must be a multiple of 32");
    if (!aligned16(d_sign_out)) return set_error(CPG_E_INVALID, "sign_out not 16-byte aligned");
    std::lock_guard<std::mutex> lk(ctx->mu);
    CPG_HIP(hipSetDevice(ctx->device));
    hipStream_t s = pick(ctx, stream);
    const int64_t w_done = (nch * chunk_len + 31) / 32, w_all = (nbases + 31) / 32;
    const int64_t ntail = w_all > w_done ? w_all - w_done : 0;
    void* wsi;
    if ((rc = ws_get(ctx, WS_ISL, islands_ws_bytes(nch, chunk_len), &wsi))) return rc;
    if (nch == 0) {
        if (ntail) CPG_HIP(hipMemsetAsync(d_sign_out + w_done, 0, (size_t)ntail * 4, s));
        CPG_HIP(hipMemsetAsync(d_count, 0, sizeof(int64_t), s));
        return CPG_OK;
    }
    if (!vit_fast_ok(model)) {
        // any model (k_vit_general.hip): the states as sign bits (state < 4) and state-packed
        // words (state & 3), over which the island kernels run the :262-339 loop on the
        // states themselves
        uint32_t* spk = nullptr;
        if ((rc = vit_general(ctx, model, d_packed, nch, chunk_len, nullptr, d_score, d_sign_out,
                              &spk, false, s)))
            return rc;
        if (ntail) CPG_HIP(hipMemsetAsync(d_sign_out + w_done, 0, (size_t)ntail * 4, s));
        CPG_HIP(launch_islands(spk, d_sign_out, nch, chunk_len, first_chunk, wsi,
                               ctx->ws[WS_ISL].bytes, d_out, cap, d_count, s));
        return CPG_OK;
    }
    VitConsts vc;
    static thread_local VitTables vt;
    if ((rc = vit_prepare(model, chunk_len, &vc, &vt))) return rc;
    const VitTables* d_vt;
    if ((rc = vit_tables(ctx, model, vc, vt, &d_vt))) return rc;
    void* ws;
    if ((rc = ws_get(ctx, WS_VIT, viterbi_ws_bytes(nch, chunk_len), &ws))) return rc;
    void* agg;
    if ((rc = ws_get(ctx, WS_VAGG, viterbi_agg_bytes(nch, chunk_len), &agg))) return rc;
    void* dn;   // per-chunk counters: K5's workgroups [0, nch), K7's [nch, 2 nch)
    if ((rc = ws_get(ctx, WS_IDONE, (size_t)nch * 8, &dn))) return rc;
    unsigned int* done = static_cast<unsigned int*>(dn);
    // fused: the traceback writes the island run records and a chunk's last traceback
    // workgroup runs its first resolve pass; the write pass places the records after it
    if (islands_fusable(nch, chunk_len) && tail_fusion_pays(nch)) {
        IslFuse fz;
        CPG_HIP(islands_fuse(&fz, wsi, ctx->ws[WS_ISL].bytes, nch, chunk_len, first_chunk, d_out,
                             cap, d_count, done + nch));
        CPG_HIP(launch_viterbi(vc, d_vt, d_packed, nch, chunk_len, ws, ctx->ws[WS_VIT].bytes,
                               d_sign_out, d_score, nullptr, ctx->d_status, s,
                               static_cast<unsigned long long*>(agg), d_sign_out + w_done, ntail,
                               &fz, done));
        CPG_HIP(islands_write(d_packed, fz, chunk_len, s));
        return CPG_OK;
    }
    if (islands_fusable(nch, chunk_len)) {
        // past the tail fusion: the traceback still writes the island tiles (the bases and
        // signs are not read again), the two resolve passes run after it
        IslFuse fz;
        CPG_HIP(islands_tiles(&fz, wsi, ctx->ws[WS_ISL].bytes, nch, chunk_len, first_chunk, d_out,
                              cap, d_count));
        CPG_HIP(launch_viterbi(vc, d_vt, d_packed, nch, chunk_len, ws, ctx->ws[WS_VIT].bytes,
                               d_sign_out, d_score, nullptr, ctx->d_status, s,
                               static_cast<unsigned long long*>(agg), d_sign_out + w_done, ntail,
                               &fz, done));
        CPG_HIP(islands_resolve(d_packed, fz, chunk_len, s));
        return CPG_OK;
    }
    CPG_HIP(launch_viterbi(vc, d_vt, d_packed, nch, chunk_len, ws, ctx->ws[WS_VIT].bytes,
                           d_sign_out, d_score, nullptr, ctx->d_status, s,
                           static_cast<unsigned long long*>(agg), d_sign_out + w_done, ntail,
                           nullptr, done));
    CPG_HIP(launch_islands(d_packed, d_sign_out, nch, chunk_len, first_chunk, wsi,
                           ctx->ws[WS_ISL].bytes, d_out, cap, d_count, s));
    return CPG_OK;
}

int cpg_viterbi_states_d(cpg_ctx* ctx, const cpg_model* model, const uint32_t* d_packed,
                         int64_t nbases, int64_t chunk_len, uint8_t* d_states_out,
                         double* d_score, void* stream) {
    if (!ctx || !model || (!d_states_out && nbases >= chunk_len))
        return set_error(CPG_E_INVALID, "null argument");
    int rc = check_layout(d_packed, nbases, chunk_len);
    if (rc) return rc;
    const int64_t nch = nbases / chunk_len;
    if (nch == 0) return CPG_OK;
    std::lock_guard<std::mutex> lk(ctx->mu);
    CPG_HIP(hipSetDevice(ctx->device));
    return vit_general(ctx, model, d_packed, nch, chunk_len, d_states_out, d_score, nullptr,
                       nullptr, false, pick(ctx, stream));
}

int cpg_bw_estep_d(cpg_ctx* ctx, const cpg_model* model, const uint32_t* d_packed,
                   int64_t nbases, int64_t chunk_len, double* d_counts, void* stream) {
    if (!ctx || !model || !d_counts) return set_error(CPG_E_INVALID, "null argument");
    int rc = check_layout(d_packed, nbases, chunk_len);
    if (rc) return rc;
    if (chunk_len % 256) return set_error(CPG_E_INVALID, "chunk_len must be a multiple of 256");
    if ((rc = model_check_deterministic(model))) return rc;
    if (chunk_len % 4096 || chunk_len > 65536)
        return set_error(CPG_E_INVALID, "E-step chunk_len must be a multiple of 4096, <= 65536");
    std::lock_guard<std::mutex> lk(ctx->mu);
    CPG_HIP(hipSetDevice(ctx->device));
    const int64_t nch = nbases / chunk_len;
    void* ws;
    if ((rc = ws_get(ctx, WS_EST, estep_ws_bytes(nch, chunk_len), &ws))) return rc;
    const double2* gtab = nullptr;
    if (nch > 0 && (rc = est_tables(ctx, model, &gtab))) return rc;
    CPG_HIP(launch_estep(*model, d_packed, nch, chunk_len, (unsigned long long*)ws, d_counts,
                         pick(ctx, stream), PART_ALL, gtab));
    return CPG_OK;
}

int cpg_train_pass_d(cpg_ctx* ctx, const cpg_model* model, const uint32_t* d_packed,
                     const uint32_t* d_sign, int64_t nbases, int64_t chunk_len,
                     double* d_estep_counts, int64_t* d_label_counts, void* stream) {
    if (!ctx || !model || !d_estep_counts || !d_label_counts || (!d_sign && nbases > 0))
        return set_error(CPG_E_INVALID, "null argument");
    int rc = check_layout(d_packed, nbases, chunk_len);
    if (rc) return rc;
    if (!aligned16(d_sign)) return set_error(CPG_E_INVALID, "sign buffer not 16-byte aligned");
    if ((rc = model_check_deterministic(model))) return rc;
    if (chunk_len % 4096 || chunk_len > 65536)
        return set_error(CPG_E_INVALID, "E-step chunk_len must be a multiple of 4096, <= 65536");
    std::lock_guard<std::mutex> lk(ctx->mu);
    CPG_HIP(hipSetDevice(ctx->device));
    const int64_t nch = nbases / chunk_len;
    void *wse, *wsc;
    if ((rc = ws_get(ctx, WS_EST, estep_ws_bytes(nch, chunk_len), &wse))) return rc;
    if ((rc = ws_get(ctx, WS_COUNT, count_ws_bytes(nch), &wsc))) return rc;
    const double2* gtab = nullptr;
    if (nch > 0 && (rc = est_tables(ctx, model, &gtab))) return rc;
    hipStream_t s = pick(ctx, stream);
    if (train_fusable(chunk_len)) {
        CPG_HIP(launch_train(*model, d_packed, d_sign, nch, chunk_len,
                             (unsigned long long*)wse, d_estep_counts,
                             (unsigned long long*)wsc, d_label_counts, s, gtab));
    } else {
        CPG_HIP(launch_estep(*model, d_packed, nch, chunk_len, (unsigned long long*)wse,
                             d_estep_counts, s, PART_ALL, gtab));
        CPG_HIP(launch_count(d_packed, d_sign, nch, chunk_len, (uint64_t*)wsc, d_label_counts, s));
    }
    return CPG_OK;
}

int cpg_merge_train_d(cpg_ctx* ctx, const void* d_gathered, int world, double* d_estep,
                      int64_t* d_counts, void* stream) {
    if (!ctx || !d_gathered || !d_estep || !d_counts || world < 1)
        return set_error(CPG_E_INVALID, "cpg_merge_train_d: bad argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    CPG_HIP(hipSetDevice(ctx->device));
    CPG_HIP(launch_merge_train(d_gathered, world, d_estep, d_counts, pick(ctx, stream)));
    return CPG_OK;
}

static int ingest_d(cpg_ctx* ctx, const char* d_txt, int64_t n, int mode, int compat_quirks,
             uint32_t* d_packed, int64_t cap_bases, cpg_ingest_result* d_result, void* stream,
             uint32_t count0) {
    if (!ctx || !d_result || (n > 0 && !d_txt) || (cap_bases > 0 && !d_packed))
        return set_error(CPG_E_INVALID, "cpg_ingest_d: null argument");
    if (n < 0 || cap_bases < 0 || (mode != 0 && mode != 1))
        return set_error(CPG_E_INVALID, "cpg_ingest_d: bad argument");
    const int64_t chunk = mode == 0 ? CPG_TRAIN_CHUNK : CPG_DECODE_CHUNK;
    if (count0 % chunk) return set_error(CPG_E_INVALID, "ingest: count0 not a chunk multiple");
    if (!aligned16(d_txt) || !aligned16(d_packed))
        return set_error(CPG_E_INVALID, "cpg_ingest_d: buffers must be 16-byte aligned");
    std::lock_guard<std::mutex> lk(ctx->mu);
    CPG_HIP(hipSetDevice(ctx->device));
    void* ws;
    int rc;
    if ((rc = ws_get(ctx, WS_ING, ingest_ws_bytes(n), &ws))) return rc;
    CPG_HIP(launch_ingest(reinterpret_cast<const uint8_t*>(d_txt), n, mode, compat_quirks, chunk,
                          d_packed, cap_bases, ws, ctx->ws[WS_ING].bytes,
                          reinterpret_cast<long long*>(d_result), pick(ctx, stream), count0));
    return CPG_OK;
}

int cpg_ingest_d(cpg_ctx* ctx, const char* d_txt, int64_t n, int mode, int compat_quirks,
                 uint32_t* d_packed, int64_t cap_bases, cpg_ingest_result* d_result,
                 void* stream) {
    return ingest_d(ctx, d_txt, n, mode, compat_quirks, d_packed, cap_bases, d_result, stream,
                    0u);
}

// ---- host-buffer entry points -------------------------------------------------------
#define CPG_TRY(x)              \
    do {                        \
        int rc_ = (x);          \
        if (rc_) return rc_;    \
    } while (0)

static int stage_in(cpg_ctx* ctx, int slot, const void* src, size_t bytes, void** dev) {
    CPG_TRY(ws_get(ctx, slot, bytes ? bytes : 16, dev));
    if (bytes) CPG_HIP(hipMemcpyAsync(*dev, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    return CPG_OK;
}

int cpg_count_labelled(cpg_ctx* ctx, const uint32_t* packed, const uint32_t* sign,
                       int64_t nbases, int64_t chunk_len, cpg_counts_i64* out) {
    if (!ctx || !packed || !sign || !out) return set_error(CPG_E_INVALID, "null argument");
    void *dp, *ds, *dc;
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        CPG_HIP(hipSetDevice(ctx->device));
        CPG_TRY(stage_in(ctx, WS_IN0, packed, (size_t)((nbases + 15) / 16) * 4, &dp));
        CPG_TRY(stage_in(ctx, WS_IN1, sign, (size_t)((nbases + 31) / 32) * 4, &ds));
        CPG_TRY(ws_get(ctx, WS_OUT0, sizeof(cpg_counts_i64), &dc));
    }
    CPG_TRY(cpg_count_labelled_d(ctx, (const uint32_t*)dp, (const uint32_t*)ds, nbases, chunk_len,
                                 (int64_t*)dc, ctx->stream));
    CPG_HIP(hipMemcpyAsync(out, dc, sizeof *out, hipMemcpyDeviceToHost, ctx->stream));
    return cpg_sync(ctx, ctx->stream);
}

int cpg_bw_estep(cpg_ctx* ctx, const cpg_model* model, const uint32_t* packed, int64_t nbases,
                 int64_t chunk_len, cpg_counts_f64* out) {
    if (!ctx || !packed || !out || !model) return set_error(CPG_E_INVALID, "null argument");
    void *dp, *dc;
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        CPG_HIP(hipSetDevice(ctx->device));
        CPG_TRY(stage_in(ctx, WS_IN0, packed, (size_t)((nbases + 15) / 16) * 4, &dp));
        CPG_TRY(ws_get(ctx, WS_OUT0, sizeof(cpg_counts_f64), &dc));
    }
    CPG_TRY(cpg_bw_estep_d(ctx, model, (const uint32_t*)dp, nbases, chunk_len, (double*)dc,
                           ctx->stream));
    CPG_HIP(hipMemcpyAsync(out, dc, sizeof *out, hipMemcpyDeviceToHost, ctx->stream));
    return cpg_sync(ctx, ctx->stream);
}

int cpg_viterbi(cpg_ctx* ctx, const cpg_model* model, const uint32_t* packed, int64_t nbases,
                int64_t chunk_len, uint32_t* sign_out, double* score) {
    if (!ctx || !packed || !sign_out || !model) return set_error(CPG_E_INVALID, "null argument");
    const int64_t nch = chunk_len > 0 ? nbases / chunk_len : 0;
    void *dp, *dsg, *dsc;
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        CPG_HIP(hipSetDevice(ctx->device));
        CPG_TRY(stage_in(ctx, WS_IN0, packed, (size_t)((nbases + 15) / 16) * 4, &dp));
        CPG_TRY(ws_get(ctx, WS_OUT0, (size_t)((nbases + 31) / 32) * 4 + 16, &dsg));
        CPG_TRY(ws_get(ctx, WS_OUT1, (size_t)(nch + 1) * 8, &dsc));
    }
    CPG_TRY(cpg_viterbi_d(ctx, model, (const uint32_t*)dp, nbases, chunk_len, (uint32_t*)dsg,
                          (double*)dsc, ctx->stream));
    CPG_HIP(hipMemcpyAsync(sign_out, dsg, (size_t)((nbases + 31) / 32) * 4, hipMemcpyDeviceToHost,
                           ctx->stream));
    if (score && nch > 0)
        CPG_HIP(hipMemcpyAsync(score, dsc, (size_t)nch * 8, hipMemcpyDeviceToHost, ctx->stream));
    return cpg_sync(ctx, ctx->stream);
}

// HmmEvaluator.decode(model, observations, true) (:260) for one array: obs in 0..3, n >= 1.
int cpg_decode_states(cpg_ctx* ctx, const cpg_model* model, const int32_t* obs, int64_t n,
                      int32_t* states_out) {
    if (!ctx || !model || !obs || !states_out) return set_error(CPG_E_INVALID, "null argument");
    if (n < 1)
        return set_error(CPG_E_INVALID,
                         "empty observation array (reference: NegativeArraySizeException)");
    std::vector<uint32_t> packed((size_t)(n + 15) / 16 + 4, 0u);
    for (int64_t i = 0; i < n; ++i) {
        if (obs[i] < 0 || obs[i] > 3)
            return set_error(CPG_E_INVALID,
                             "observation %lld = %d not in 0..3 (reference: "
                             "ArrayIndexOutOfBoundsException)", (long long)i, obs[i]);
        packed[i >> 4] |= (uint32_t)obs[i] << ((i & 15) * 2);
    }
    if (!vit_fast_ok(model)) {   // any model: Mahout's 8-state loop (k_vit_general.hip)
        void *dp, *dst;
        {
            std::lock_guard<std::mutex> lk(ctx->mu);
            CPG_HIP(hipSetDevice(ctx->device));
            CPG_TRY(stage_in(ctx, WS_IN0, packed.data(), packed.size() * 4, &dp));
            CPG_TRY(ws_get(ctx, WS_OUT0, (size_t)n + 64, &dst));
            CPG_TRY(vit_general(ctx, model, (const uint32_t*)dp, 1, n, (uint8_t*)dst, nullptr,
                                nullptr, nullptr, false, ctx->stream));
        }
        std::vector<uint8_t> st((size_t)n);
        CPG_HIP(hipMemcpyAsync(st.data(), dst, (size_t)n, hipMemcpyDeviceToHost, ctx->stream));
        CPG_TRY(cpg_sync(ctx, ctx->stream));
        for (int64_t i = 0; i < n; ++i) states_out[i] = st[i];
        return CPG_OK;
    }
    std::vector<uint32_t> sign((size_t)(n + 31) / 32 + 4, 0u);
    double score = 0.0;
    CPG_TRY(cpg_viterbi(ctx, model, packed.data(), n, n, sign.data(), &score));
    // pi = 0 for both live states at t=0: every candidate is -inf, Mahout's maxState stays 0
    // (state A+) at every step and the final argmax (strict '>' from -inf) leaves state 0
    // (SURVEY.md A.2); the '+' sign path is right, the indices are not the base's: patch them
    const bool degen = model->pi[obs[0]] == 0.0 && model->pi[obs[0] + 4] == 0.0;
    for (int64_t i = 0; i < n; ++i) {
        const bool plus = (sign[i >> 5] >> (i & 31)) & 1u;
        states_out[i] = degen ? 0 : obs[i] + (plus ? 0 : 4);
    }
    return CPG_OK;
}

static int ingest_gpu(cpg_ctx* ctx, const char* txt, size_t n, int mode, int compat_quirks,
                      uint32_t* packed, int64_t cap_bases, int64_t* nbases, uint32_t count0) {
    if (!ctx || !nbases || (n > 0 && !txt) || (cap_bases > 0 && !packed) || cap_bases < 0 ||
        (mode != 0 && mode != 1))
        return set_error(CPG_E_INVALID, "cpg_ingest_gpu: bad argument");
    *nbases = 0;
    void *dt, *dp, *dr;
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        CPG_HIP(hipSetDevice(ctx->device));
        CPG_TRY(stage_in(ctx, WS_IN0, txt, n, &dt));
        CPG_TRY(ws_get(ctx, WS_OUT0, (size_t)((cap_bases + 15) / 16) * 4 + 16, &dp));
        CPG_TRY(ws_get(ctx, WS_OUT1, sizeof(cpg_ingest_result), &dr));
    }
    CPG_TRY(ingest_d(ctx, (const char*)dt, (int64_t)n, mode, compat_quirks, (uint32_t*)dp,
                     cap_bases, (cpg_ingest_result*)dr, ctx->stream, count0));
    cpg_ingest_result r;
    CPG_HIP(hipMemcpyAsync(&r, dr, sizeof r, hipMemcpyDeviceToHost, ctx->stream));
    CPG_TRY(cpg_sync(ctx, ctx->stream));
    *nbases = r.nbases;
    // the committed chunks (and, as cpg_ingest, the pending tail bases that fit)
    const int64_t keep = r.status == CPG_OK ? cap_bases : r.nbases;
    if (keep > 0)
        CPG_HIP(hipMemcpy(packed, dp, (size_t)((keep + 15) / 16) * 4, hipMemcpyDeviceToHost));
    if (r.status == CPG_E_REF_CRASH)
        return set_error(CPG_E_REF_CRASH,
                         "reference throws at input byte %lld (decode reader on an empty list, "
                         "or the training reader's chunk vector past a 2^32 count wrap)", (long long)r.crash_byte);
    if (r.status == CPG_E_CAPACITY)
        return set_error(CPG_E_CAPACITY, "cpg_ingest_gpu: capacity %lld bases exceeded",
                         (long long)cap_bases);
    if (r.status != CPG_OK)
        return set_error((int)r.status, "cpg_ingest_gpu: device look-back timed out");
    return CPG_OK;
}

int cpg_ingest_gpu(cpg_ctx* ctx, const char* txt, size_t n, int mode, int compat_quirks,
                   uint32_t* packed, int64_t cap_bases, int64_t* nbases) {
    return ingest_gpu(ctx, txt, n, mode, compat_quirks, packed, cap_bases, nbases, 0u);
}

// test hook (cpg_internal.h): the device reader from Java count = count0
int cpgx_ingest_gpu_at(cpg_ctx* ctx, const char* txt, size_t n, int mode, int compat_quirks,
                       uint32_t* packed, int64_t cap_bases, int64_t* nbases, uint32_t count0) {
    return ingest_gpu(ctx, txt, n, mode, compat_quirks, packed, cap_bases, nbases, count0);
}

int cpg_islands(cpg_ctx* ctx, const uint32_t* packed, const uint32_t* sign, int64_t nbases,
                int64_t chunk_len, cpg_island* out, int64_t cap, int64_t* count) {
    if (!ctx || !packed || !sign || !count || (cap > 0 && !out))
        return set_error(CPG_E_INVALID, "null argument");
    void *dp, *ds, *dout, *dcnt;
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        CPG_HIP(hipSetDevice(ctx->device));
        CPG_TRY(stage_in(ctx, WS_IN0, packed, (size_t)((nbases + 15) / 16) * 4, &dp));
        CPG_TRY(stage_in(ctx, WS_IN1, sign, (size_t)((nbases + 31) / 32) * 4, &ds));
        CPG_TRY(ws_get(ctx, WS_OUT0, (size_t)(cap > 0 ? cap : 1) * sizeof(cpg_island), &dout));
        CPG_TRY(ws_get(ctx, WS_OUT1, 16, &dcnt));
    }
    CPG_TRY(cpg_islands_d(ctx, (const uint32_t*)dp, (const uint32_t*)ds, nbases, chunk_len,
                          (cpg_island*)dout, cap, (int64_t*)dcnt, ctx->stream));
    CPG_HIP(hipMemcpyAsync(count, dcnt, 8, hipMemcpyDeviceToHost, ctx->stream));
    CPG_TRY(cpg_sync(ctx, ctx->stream));
    const int64_t n = *count < cap ? *count : cap;
    if (n > 0)
        CPG_HIP(hipMemcpy(out, dout, (size_t)n * sizeof(cpg_island), hipMemcpyDeviceToHost));
    if (*count > cap) return set_error(CPG_E_CAPACITY, "need %lld island records", (long long)*count);
    return CPG_OK;
}

}  // extern "C"
