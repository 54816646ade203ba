// cpg_pipeline.cpp — the whole-genome training + decode pass streamed from host memory
// (BASELINE config C5: genomes larger than one would stage at once, pinned host DRAM ->
// HBM overlapped with compute).  One call covers what the reference's driver does per genome:
// trainModel's mapper pass (CpGIslandFinder.java:130-141, :200) and testModel's decode +
// island scan (:256-339), on windows of whole 1 Mi decode chunks:
//
//   copy-in stream : H2D window k (packed bases, optional truth sign bits) into buffer k % nbuf
//   train stream   : E-step + labelled counts of the window's 64 Ki chunks, ACCUMULATED in the
//                    context's fixed-point accumulators (finalized once at the end: the result
//                    is bit-identical to one call over the whole genome)
//   decode stream  : exact Viterbi of the window's 1 Mi chunks + island scan appended after the
//                    earlier windows' records (device-side running count: no host round trip)
//   copy-out stream: D2H of the decoded sign bits of window k
// Events order buffer reuse (a window is overwritten only after both consumers and the
// copy-out of its decode are done).  The window boundaries are multiples of 1 Mi, so every
// training and decode chunk lies inside one window, exactly as in the unstreamed calls.

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "cpg_internal.h"
#include "isl_dev.h"

namespace cpg {
namespace {

struct HostPin {
    void* p = nullptr;
    bool registered = false;
    ~HostPin() {
        if (registered) (void)hipHostUnregister(p);
    }
};

// page-lock a caller buffer for the call's duration (DMA straight from it) unless it already
// is pinned; a failed registration leaves pageable copies (HIP stages them, slower).  Buffers
// under kPinMin stay pageable: staging costs little at that size, and a small caller
// buffer registered and unregistered here is soon handed out again by the caller's allocator
// for other (pageable) transfers.  (The one GPU fault seen in the streamed-genome tests,
// round 6: an illegal address reported in a torch H2D copy right after a 700,000-base call
// whose 175 KB and 88 KB inputs had been registered here; not reproduced, cause unproven.)
constexpr size_t kPinMin = 8u << 20;
void pin_host(HostPin& h, const void* p, size_t bytes) {
    if (!p || bytes < kPinMin) return;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeHost) return;
    (void)hipGetLastError();
    if (hipHostRegister(const_cast<void*>(p), bytes, hipHostRegisterDefault) == hipSuccess) {
        h.p = const_cast<void*>(p);
        h.registered = true;
    } else {
        (void)hipGetLastError();
    }
}

int ensure_streams(cpg_ctx* ctx) {
    if (ctx->ps[0]) return CPG_OK;
    int lo = 0, hi = 0;
    CPG_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CPG_HIP(hipStreamCreateWithFlags(&ctx->ps[0], hipStreamNonBlocking));
    CPG_HIP(hipStreamCreateWithFlags(&ctx->ps[1], hipStreamNonBlocking));
    // the decode kernels are latency-bound: high priority, the E-step fills the rest
    CPG_HIP(hipStreamCreateWithPriority(&ctx->ps[2], hipStreamNonBlocking, hi));
    CPG_HIP(hipStreamCreateWithFlags(&ctx->ps[3], hipStreamNonBlocking));
    for (auto& ev : ctx->pev) CPG_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    return CPG_OK;
}

size_t up256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace
}  // namespace cpg

using namespace cpg;

extern "C" int cpg_genome_run(cpg_ctx* ctx, const cpg_model* train_model,
                              const cpg_model* decode_model, const uint32_t* packed,
                              const uint32_t* sign, int64_t nbases, const cpg_genome_opts* opts,
                              cpg_counts_f64* estep_out, cpg_counts_i64* counts_out,
                              uint32_t* sign_out, double* score_out, cpg_island* islands_out,
                              int64_t island_cap, int64_t* island_count) {
    if (!ctx || (nbases > 0 && !packed) || nbases < 0)
        return set_error(CPG_E_INVALID, "cpg_genome_run: bad argument");
    if (estep_out && !train_model)
        return set_error(CPG_E_INVALID, "cpg_genome_run: estep_out needs train_model");
    if (counts_out && !sign)
        return set_error(CPG_E_INVALID, "cpg_genome_run: counts_out needs the truth sign bits");
    const bool decode = decode_model != nullptr;
    if (decode && (!island_count || (island_cap > 0 && !islands_out) || island_cap < 0))
        return set_error(CPG_E_INVALID, "cpg_genome_run: decoding needs island_count/islands_out");
    const int64_t D = CPG_DECODE_CHUNK, T = CPG_TRAIN_CHUNK;
    int64_t W = opts && opts->window_bases > 0 ? opts->window_bases : 64 * D;
    int nbuf = opts && opts->nbuf > 0 ? opts->nbuf : 3;
    const int64_t chunk0 = opts ? opts->first_chunk : 0;
    if (chunk0 < 0) return set_error(CPG_E_INVALID, "first_chunk < 0");
    if (W % D) return set_error(CPG_E_INVALID, "window_bases must be a multiple of 1,048,576");
    if (nbuf < 2 || nbuf > cpg_ctx::kMaxBuf)
        return set_error(CPG_E_INVALID, "nbuf must be in 2..%d", cpg_ctx::kMaxBuf);
    if (estep_out) {
        const int mrc = model_check_deterministic(train_model);
        if (mrc) return mrc;
    }
    if (island_count) *island_count = 0;
    const int64_t nwin = (nbases + W - 1) / W;
    const int64_t ndec = nbases / D;
    W = std::min<int64_t>(W, std::max<int64_t>(D, (nbases + D - 1) / D * D));
    nbuf = (int)std::min<int64_t>(nbuf, std::max<int64_t>(nwin, 1));

    std::lock_guard<std::mutex> lk(ctx->mu);
    CPG_HIP(hipSetDevice(ctx->device));
    int rc;
    if ((rc = ensure_streams(ctx))) return rc;
    hipStream_t sin = ctx->ps[0], str = ctx->ps[1], sdec = ctx->ps[2], sout = ctx->ps[3];

    // Viterbi constants/tables of the decode model (host), before any device work
    VitConsts vc;
    static thread_local VitTables vt;
    const VitTables* d_vt = nullptr;
    if (decode) {
        if ((rc = vit_prepare(decode_model, D, &vc, &vt))) return rc;
        if ((rc = vit_tables(ctx, decode_model, vc, vt, &d_vt))) return rc;
    }
    // workspaces sized for the largest window up front (ws_get may reallocate)
    void *ws_cnt = nullptr, *ws_vit = nullptr, *ws_isl = nullptr, *ws_est = nullptr;
    const int64_t wdec = W / D, wtr = W / T;
    if (counts_out && (rc = ws_get(ctx, WS_COUNT, count_ws_bytes(wtr), &ws_cnt))) return rc;
    if (estep_out && (rc = ws_get(ctx, WS_EST, estep_ws_bytes(wtr, T), &ws_est))) return rc;
    const double2* est_gtab = nullptr;
    if (estep_out && (rc = est_tables(ctx, train_model, &est_gtab))) return rc;
    if (decode && (rc = ws_get(ctx, WS_VIT, viterbi_ws_bytes(wdec, D), &ws_vit))) return rc;
    if (decode && (rc = ws_get(ctx, WS_ISL, islands_ws_bytes(wdec, D), &ws_isl))) return rc;
    void *ws_agg = nullptr, *ws_done = nullptr;
    if (decode && (rc = ws_get(ctx, WS_VAGG, viterbi_agg_bytes(wdec, D), &ws_agg))) return rc;
    if (decode && (rc = ws_get(ctx, WS_IDONE, (size_t)(wdec + 1) * 8, &ws_done))) return rc;
    // window buffers + results, one allocation
    const size_t bp = up256((size_t)(W / 16) * 4 + 64), bs = up256((size_t)(W / 32) * 4 + 64);
    const size_t per = bp + (sign ? bs : 0) + (decode ? bs : 0);
    const size_t o_score = per * nbuf, o_cnt = o_score + up256((size_t)(ndec + 1) * 8),
                 o_est = o_cnt + up256((size_t)(nwin + 1) * 8), o_lab = o_est + up256(105 * 8),
                 o_end = o_lab + up256(124 * 8);
    void* g;
    if ((rc = ws_get(ctx, WS_GEN, o_end, &g))) return rc;
    char* gb = static_cast<char*>(g);
    void* gi = nullptr;
    const int64_t icap = decode ? std::max<int64_t>(island_cap, 1) : 0;
    if (decode && (rc = ws_get(ctx, WS_GISL, (size_t)icap * sizeof(cpg_island), &gi))) return rc;
    auto buf_packed = [&](int b) { return reinterpret_cast<uint32_t*>(gb + per * b); };
    auto buf_sign = [&](int b) { return reinterpret_cast<uint32_t*>(gb + per * b + bp); };
    auto buf_out = [&](int b) {
        return reinterpret_cast<uint32_t*>(gb + per * b + bp + (sign ? bs : 0));
    };
    double* d_score = reinterpret_cast<double*>(gb + o_score);
    int64_t* d_icnt = reinterpret_cast<int64_t*>(gb + o_cnt);
    double* d_est = reinterpret_cast<double*>(gb + o_est);
    int64_t* d_lab = reinterpret_cast<int64_t*>(gb + o_lab);
    cpg_island* d_isl = static_cast<cpg_island*>(gi);

    // every earlier call's work (other streams included) done before this call's streams,
    // which are non-blocking, touch the workspaces
    CPG_HIP(hipDeviceSynchronize());
    // host buffers: DMA straight from/to them (page-locked for the call)
    HostPin pin_pk, pin_sg, pin_out;
    pin_host(pin_pk, packed, (size_t)((nbases + 15) / 16) * 4);
    pin_host(pin_sg, sign, (size_t)((nbases + 31) / 32) * 4);
    if (decode && sign_out) pin_host(pin_out, sign_out, (size_t)((nbases + 31) / 32) * 4);

    hipEvent_t* ev_in = ctx->pev;                          // window landed in buffer b
    hipEvent_t* ev_tr = ctx->pev + cpg_ctx::kMaxBuf;       // train done with buffer b
    hipEvent_t* ev_dec = ctx->pev + 2 * cpg_ctx::kMaxBuf;  // decode done with buffer b
    hipEvent_t* ev_out = ctx->pev + 3 * cpg_ctx::kMaxBuf;  // sign bits of buffer b copied out
    if (decode) CPG_HIP(hipMemsetAsync(d_icnt, 0, 8, sdec));
    for (int64_t k = 0; k < nwin; ++k) {
        const int b = (int)(k % nbuf);
        const int64_t start = k * W, nb = std::min(W, nbases - start);
        const int64_t ntr = nb / T, nd = nb / D;
        if (k >= nbuf) {   // buffer b free: both consumers of window k - nbuf are done
            CPG_HIP(hipStreamWaitEvent(sin, ev_tr[b], 0));
            CPG_HIP(hipStreamWaitEvent(sin, ev_dec[b], 0));
        }
        CPG_HIP(hipMemcpyAsync(buf_packed(b), packed + start / 16, (size_t)((nb + 15) / 16) * 4,
                               hipMemcpyHostToDevice, sin));
        if (sign)
            CPG_HIP(hipMemcpyAsync(buf_sign(b), sign + start / 32, (size_t)((nb + 31) / 32) * 4,
                                   hipMemcpyHostToDevice, sin));
        CPG_HIP(hipEventRecord(ev_in[b], sin));
        // train: accumulate only
        CPG_HIP(hipStreamWaitEvent(str, ev_in[b], 0));
        if (estep_out && ntr > 0)
            CPG_HIP(launch_estep(*train_model, buf_packed(b), ntr, T,
                                 static_cast<unsigned long long*>(ws_est), nullptr, str,
                                 PART_ACC, est_gtab));
        if (counts_out && ntr > 0)
            CPG_HIP(launch_count(buf_packed(b), buf_sign(b), ntr, T, static_cast<uint64_t*>(ws_cnt),
                                 nullptr, str, PART_ACC));
        CPG_HIP(hipEventRecord(ev_tr[b], str));
        // decode
        CPG_HIP(hipStreamWaitEvent(sdec, ev_in[b], 0));
        if (decode) {
            if (k >= nbuf) CPG_HIP(hipStreamWaitEvent(sdec, ev_out[b], 0));
            if (nd > 0) {
                if (islands_fusable(nd, D) && tail_fusion_pays(nd)) {   // fused decode (as cpg_decode_d)
                    IslFuse fz;
                    CPG_HIP(islands_fuse(&fz, ws_isl, ctx->ws[WS_ISL].bytes, nd, D,
                                         chunk0 + start / D, d_isl, island_cap, d_icnt + k + 1,
                                         static_cast<unsigned int*>(ws_done) + nd, d_icnt + k));
                    CPG_HIP(launch_viterbi(vc, d_vt, buf_packed(b), nd, D, ws_vit,
                                           ctx->ws[WS_VIT].bytes, buf_out(b), d_score + start / D,
                                           nullptr, ctx->d_status, sdec,
                                           static_cast<unsigned long long*>(ws_agg), nullptr, 0,
                                           &fz, static_cast<unsigned int*>(ws_done)));
                    CPG_HIP(islands_write(buf_packed(b), fz, D, sdec));
                } else {
                    CPG_HIP(launch_viterbi(vc, d_vt, buf_packed(b), nd, D, ws_vit,
                                           ctx->ws[WS_VIT].bytes, buf_out(b), d_score + start / D,
                                           nullptr, ctx->d_status, sdec,
                                           static_cast<unsigned long long*>(ws_agg), nullptr, 0,
                                           nullptr, static_cast<unsigned int*>(ws_done)));
                    CPG_HIP(launch_islands(buf_packed(b), buf_out(b), nd, D, chunk0 + start / D,
                                           ws_isl, ctx->ws[WS_ISL].bytes, d_isl, island_cap,
                                           d_icnt + k + 1, sdec, d_icnt + k));
                }
            } else {
                CPG_HIP(hipMemcpyAsync(d_icnt + k + 1, d_icnt + k, 8, hipMemcpyDeviceToDevice, sdec));
            }
        }
        CPG_HIP(hipEventRecord(ev_dec[b], sdec));
        if (decode && sign_out && nd > 0) {
            CPG_HIP(hipStreamWaitEvent(sout, ev_dec[b], 0));
            CPG_HIP(hipMemcpyAsync(sign_out + start / 32, buf_out(b), (size_t)(nd * D / 32) * 4,
                                   hipMemcpyDeviceToHost, sout));
        }
        CPG_HIP(hipEventRecord(ev_out[b], sout));
    }
    // finalize: the accumulators of the whole genome -> the result structs
    if (estep_out) {
        CPG_HIP(launch_estep(*train_model, nullptr, 0, T, static_cast<unsigned long long*>(ws_est),
                             d_est, str, PART_FINAL));
        CPG_HIP(hipMemcpyAsync(estep_out, d_est, sizeof *estep_out, hipMemcpyDeviceToHost, str));
    }
    if (counts_out) {
        CPG_HIP(launch_count(nullptr, nullptr, 0, T, static_cast<uint64_t*>(ws_cnt), d_lab, str,
                             PART_FINAL));
        CPG_HIP(hipMemcpyAsync(counts_out, d_lab, sizeof *counts_out, hipMemcpyDeviceToHost, str));
    }
    int64_t total = 0;
    if (decode) {
        if (score_out && ndec > 0)
            CPG_HIP(hipMemcpyAsync(score_out, d_score, (size_t)ndec * 8, hipMemcpyDeviceToHost, sdec));
        CPG_HIP(hipMemcpyAsync(&total, d_icnt + nwin, 8, hipMemcpyDeviceToHost, sdec));
    }
    CPG_HIP(hipStreamSynchronize(sin));
    CPG_HIP(hipStreamSynchronize(str));
    CPG_HIP(hipStreamSynchronize(sdec));
    CPG_HIP(hipStreamSynchronize(sout));
    if (decode) {
        const int64_t n = std::min(total, island_cap);
        if (n > 0)
            CPG_HIP(hipMemcpy(islands_out, d_isl, (size_t)n * sizeof(cpg_island),
                              hipMemcpyDeviceToHost));
        *island_count = total;
        if (sign_out) {   // the undecoded tail reads '-' (as cpg_viterbi_d)
            const int64_t w0 = ndec * D / 32, w1 = (nbases + 31) / 32;
            if (w1 > w0) std::memset(sign_out + w0, 0, (size_t)(w1 - w0) * 4);
        }
    }
    if ((rc = cpg_sync(ctx, nullptr))) return rc;   // kernel self-checks (status word)
    if (decode && total > island_cap)
        return set_error(CPG_E_CAPACITY, "need %lld island records", (long long)total);
    return CPG_OK;
}
