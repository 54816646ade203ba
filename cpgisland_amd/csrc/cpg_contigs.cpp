// cpg_contigs.cpp — C-ABI of the ragged contig batch (BASELINE config C4; include/cpg.h):
// validation, workspaces and the launches of k_contigs.hip.  Every contig is one observation
// sequence with the reference's per-chunk semantics (:130-141/:200 training, :256-260 decode,
// :262-339 islands).

#include "cpg_internal.h"

using namespace cpg;

namespace {

int check_batch(cpg_ctx* ctx, const uint32_t* packed, int64_t nbases, const int64_t* offs,
                const int32_t* lens, int64_t n) {
    if (!ctx) return set_error(CPG_E_INVALID, "null ctx");
    if (n < 0 || nbases < 0 || n >= (1ll << 31))
        return set_error(CPG_E_INVALID, "contig batch: n=%lld nbases=%lld", (long long)n,
                         (long long)nbases);
    if (n > 0 && (!packed || !offs || !lens))
        return set_error(CPG_E_INVALID, "contig batch: null buffer");
    if (!aligned16(packed)) return set_error(CPG_E_INVALID, "packed buffer not 16-byte aligned");
    return CPG_OK;
}

}  // namespace

extern "C" {

int cpg_contigs_order_d(cpg_ctx* ctx, const int32_t* d_lens, int64_t n, int32_t* d_order,
                        void* stream) {
    if (!ctx || (n > 0 && (!d_lens || !d_order)) || n < 0 || n >= (1ll << 31))
        return set_error(CPG_E_INVALID, "cpg_contigs_order_d: bad argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    CPG_HIP(hipSetDevice(ctx->device));
    void* ws;
    int rc;
    if ((rc = ws_get(ctx, WS_CSORT, contigs_sort_ws_bytes(n), &ws))) return rc;
    CPG_HIP(launch_contigs_order(d_lens, n, d_order, ws, ctx->ws[WS_CSORT].bytes,
                                 static_cast<hipStream_t>(stream)));
    return CPG_OK;
}

int cpg_contigs_count_labelled_d(cpg_ctx* ctx, const uint32_t* d_packed, const uint32_t* d_sign,
                                 int64_t nbases, const int64_t* d_offs, const int32_t* d_lens,
                                 const int32_t* d_order, int64_t n, int64_t* d_counts,
                                 void* stream) {
    int rc = check_batch(ctx, d_packed, nbases, d_offs, d_lens, n);
    if (rc) return rc;
    if (!d_counts || (n > 0 && !d_sign)) return set_error(CPG_E_INVALID, "null argument");
    if (!aligned16(d_sign)) return set_error(CPG_E_INVALID, "sign buffer not 16-byte aligned");
    std::lock_guard<std::mutex> lk(ctx->mu);
    CPG_HIP(hipSetDevice(ctx->device));
    void* ws;
    if ((rc = ws_get(ctx, WS_COUNT, count_ws_bytes(1), &ws))) return rc;
    CPG_HIP(launch_contigs_count(d_packed, d_sign, nbases, d_offs, d_lens, d_order, n,
                                 static_cast<uint64_t*>(ws), d_counts, ctx->d_status,
                                 static_cast<hipStream_t>(stream)));
    return CPG_OK;
}

int cpg_contigs_estep_d(cpg_ctx* ctx, const cpg_model* model, const uint32_t* d_packed,
                        int64_t nbases, const int64_t* d_offs, const int32_t* d_lens,
                        const int32_t* d_order, int64_t n, double* d_counts, void* stream) {
    int rc = check_batch(ctx, d_packed, nbases, d_offs, d_lens, n);
    if (rc) return rc;
    if (!model || !d_counts) return set_error(CPG_E_INVALID, "null argument");
    if ((rc = model_check_deterministic(model))) return rc;
    std::lock_guard<std::mutex> lk(ctx->mu);
    CPG_HIP(hipSetDevice(ctx->device));
    void *acc, *ck;
    if ((rc = ws_get(ctx, WS_EST, estep_ws_bytes(1, CPG_TRAIN_CHUNK), &acc))) return rc;
    // alpha checkpoints: 16 B per 64 bases of the packed span
    if ((rc = ws_get(ctx, WS_CCK, (size_t)((nbases + 63) / 64) * 16 + 64, &ck))) return rc;
    CPG_HIP(launch_contigs_estep(*model, d_packed, nbases, d_offs, d_lens, d_order, n, ck,
                                 static_cast<unsigned long long*>(acc), d_counts, ctx->d_status,
                                 static_cast<hipStream_t>(stream)));
    return CPG_OK;
}

int cpg_contigs_viterbi_d(cpg_ctx* ctx, const cpg_model* model, const uint32_t* d_packed,
                          int64_t nbases, const int64_t* d_offs, const int32_t* d_lens,
                          const int32_t* d_order, int64_t n, uint32_t* d_sign_out,
                          double* d_score, void* stream) {
    int rc = check_batch(ctx, d_packed, nbases, d_offs, d_lens, n);
    if (rc) return rc;
    if (!model || (n > 0 && !d_sign_out)) return set_error(CPG_E_INVALID, "null argument");
    if (!aligned16(d_sign_out)) return set_error(CPG_E_INVALID, "sign_out not 16-byte aligned");
    VitConsts vc;
    static thread_local VitTables vt;
    if ((rc = vit_prepare(model, CPG_DECODE_CHUNK, &vc, &vt))) return rc;
    std::lock_guard<std::mutex> lk(ctx->mu);
    CPG_HIP(hipSetDevice(ctx->device));
    void* bp;
    // 2-bit backpointers: 16 B per 64 bases of the packed span
    if ((rc = ws_get(ctx, WS_CBP, (size_t)((nbases + 63) / 64) * 16 + 64, &bp))) return rc;
    CPG_HIP(launch_contigs_viterbi(vc, d_packed, nbases, d_offs, d_lens, d_order, n,
                                   static_cast<uint32_t*>(bp), d_sign_out, d_score, ctx->d_status,
                                   static_cast<hipStream_t>(stream)));
    return CPG_OK;
}

int cpg_contigs_islands_d(cpg_ctx* ctx, const uint32_t* d_packed, const uint32_t* d_sign,
                          int64_t nbases, const int64_t* d_offs, const int32_t* d_lens,
                          const int32_t* d_order, int64_t n, cpg_island* d_out, int64_t cap,
                          int64_t* d_count, void* stream) {
    int rc = check_batch(ctx, d_packed, nbases, d_offs, d_lens, n);
    if (rc) return rc;
    if (!d_count || (cap > 0 && !d_out) || cap < 0 || (n > 0 && !d_sign))
        return set_error(CPG_E_INVALID, "null argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    CPG_HIP(hipSetDevice(ctx->device));
    void* ws;
    if ((rc = ws_get(ctx, WS_CISL, contigs_sort_ws_bytes(n), &ws))) return rc;
    CPG_HIP(launch_contigs_islands(d_packed, d_sign, nbases, d_offs, d_lens, d_order, n, ws,
                                   ctx->ws[WS_CISL].bytes, d_out, cap, d_count, ctx->d_status,
                                   static_cast<hipStream_t>(stream)));
    return CPG_OK;
}

}  // extern "C"
