/*
 * cpg.h — C-ABI of libcpg.so, the MI355X-native hot path of CpGIslandFinder.
 *
 * Reference: /root/reference/CpGIslandFinder.java (ErangaD/CpGIsland).  Every entry
 * point below names the reference interface it replaces (file:line).  The reference
 * host is Java; its drop-in binding (Panama FFM downcalls, JNI fallback) is shown in
 * INTEGRATION.md.  No torch / HIP types appear in these signatures: plain pointers,
 * sizes and an opaque context.  Streams are passed as `void*`: a hipStream_t, NULL
 * meaning the HIP null stream (as in the HIP API itself).
 *
 * Conventions
 *   - return 0 (CPG_OK) or a negative CPG_E_* code; no exceptions cross the ABI.
 *     cpg_last_error() returns a thread-local message for the last failure.
 *   - every output buffer is caller-owned.  The context owns device workspace,
 *     pinned staging buffers and its stream.
 *   - one call at a time per context (contexts are internally serialised); separate
 *     contexts (one per device / process) run concurrently.  Each kind of "_d" entry
 *     point owns its own workspace in the context, so launches of DIFFERENT kinds (e.g.
 *     the E-step and the Viterbi) may execute concurrently on different streams; two
 *     launches of the same kind must be ordered by the caller (same stream or events).
 *   - "_d" entry points take DEVICE pointers (HBM-resident inputs, the bench path)
 *     and are asynchronous on `stream`; call cpg_sync() to wait and collect the
 *     context's device-side status word (set by the kernels' self checks).
 *     Entry points without "_d" take HOST pointers, stage through pinned memory and
 *     return after the results are in the caller's buffers.
 *
 * Data layout (HBM and host alike)
 *   packed bases : uint32 words, 16 bases per word, base k at bits 2*(k%16),
 *                  A=0 C=1 G=2 T=3 (the reference's symbol map, :114-123 / :240-249)
 *   sign bits    : uint32 words, 32 bases per word, bit k%32; 1 = '+' (island state
 *                  0..3), 0 = '-' (state 4..7)
 *   model        : state order A+ C+ G+ T+ A- C- G- T- (:182-189), row-major
 */
#ifndef CPG_H_
#define CPG_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CPG_ABI_VERSION 1

/* status codes */
#define CPG_OK              0
#define CPG_E_INVALID     (-1)  /* bad argument: null pointer, size, symbol not in 0..3
                                   (reference: ArrayIndexOutOfBounds / NegativeArraySize) */
#define CPG_E_DEVICE      (-2)  /* HIP runtime error / no device */
#define CPG_E_UNSUPPORTED (-3)  /* model outside the GPU path's contract (see cpg_viterbi_d) */
#define CPG_E_CAPACITY    (-4)  /* caller's output buffer too small (*count holds the need) */
#define CPG_E_REF_CRASH   (-5)  /* reference would throw at this input (decode ingest) */
#define CPG_E_VERIFY      (-6)  /* a kernel's exactness self-check failed */

#define CPG_TRAIN_CHUNK   65536    /* 0x10000  — CpGIslandFinder.java:130 */
#define CPG_DECODE_CHUNK  1048576  /* 0x100000 — CpGIslandFinder.java:256 */

/* HMM over the 8 hidden states x 4 symbols.  CpGIslandFinder.java:155-173 */
typedef struct cpg_model {
    double pi[8];
    double a[8][8];
    double b[8][4];
} cpg_model;

/* Baum-Welch sufficient statistics (expected counts, fp64) summed over chunks:
 * the mapper's stripes (initial, transition row i, emission row i) behind
 * BaumWelchDriver.runBaumWelchMR (called at CpGIslandFinder.java:200). */
typedef struct cpg_counts_f64 {
    double init[8];
    double trans[8][8];
    double emit[8][4];
    double loglik;          /* sum over chunks of log P(chunk | model) */
} cpg_counts_f64;

/* Hard-label ("labelled") integer counts, same stripe layout + dinucleotide and
 * mononucleotide histograms.  Build-defined. */
typedef struct cpg_counts_i64 {
    int64_t init[8];
    int64_t trans[8][8];
    int64_t emit[8][4];
    int64_t dinuc[4][4];
    int64_t mono[4];
} cpg_counts_i64;

#define CPG_COUNTS_I64_N 124   /* int64 fields in cpg_counts_i64 */
#define CPG_COUNTS_F64_N 105   /* doubles in cpg_counts_f64 */

/* One island record, exactly the values the reference formats at :287-288:
 *   "%d %d %d %f %f\n", beg+chunk*0x100000+1, end+chunk*0x100000+1, islandLen,
 *   cgcontent, oeratio   (Java int arithmetic: coordinates wrap at 2^31). */
typedef struct cpg_island {
    int32_t beg1;      /* 1-based start, int32-wrapped as in Java */
    int32_t end1;      /* 1-based end (inclusive), int32-wrapped */
    int32_t len;       /* islandLen */
    int32_t chunk;     /* decode chunk index (0-based) */
    double  cg;        /* (C+G)/len                         (:280) */
    double  oe;        /* (int32)(CpG*len) / (C*G) or 0.0    (:281-283) */
} cpg_island;

typedef struct cpg_ctx cpg_ctx;

/* ---- context ---------------------------------------------------------------- */
int         cpg_open(int device, cpg_ctx** out);
void        cpg_close(cpg_ctx* ctx);
const char* cpg_last_error(void);
int         cpg_abi_version(void);
/* Pre-size the context's workspace for inputs of up to nbases bases, for every decode chunk
 * length that is a multiple of 256 up to 1 Mi (the per-chunk slots at their largest: 256-base
 * chunks), so that the _d entry points never allocate for those lengths (required before
 * hipGraph capture).  Shorter island chunk lengths (cpg_islands_d / cpg_islands_at_d take
 * any multiple of 32) and lengths past 1 Mi are outside this promise: such a call may grow a
 * slot.  A slot that has to grow (a larger input, another chunk length) synchronises the
 * whole device first: the old buffer may still be read by a kernel on another stream.
 * cpg_reserve_chunk sizes for ONE decode chunk length instead (a caller on the reference's
 * 1 Mi chunks does not pay for 256-base ones).
 * The general-model Viterbi (cpg_viterbi_states_d, and cpg_viterbi_d / cpg_decode_d /
 * cpg_decode_states for models outside the exact scan's contract) needs up to ~26 B of
 * workspace per base (its backpointer ballots); cpg_reserve does NOT size it: that path
 * allocates at its first use and is outside this contract unless the workspace was reserved
 * with cpg_reserve_ex(ctx, nbases, CPG_RESERVE_GENERAL). */
int         cpg_reserve(cpg_ctx* ctx, int64_t nbases);
#define CPG_RESERVE_GENERAL 1   /* also size the general-model Viterbi's workspace */
int         cpg_reserve_ex(cpg_ctx* ctx, int64_t nbases, int flags);
/* As cpg_reserve_ex, for decode / island calls with this one chunk_len (a multiple of 32;
 * > 1 chunk per call needs a multiple of 256 for the Viterbi) and the training chunk
 * CPG_TRAIN_CHUNK; the _d entry points then never allocate for calls of at most nbases bases
 * with that chunk length. */
int         cpg_reserve_chunk(cpg_ctx* ctx, int64_t nbases, int64_t chunk_len, int flags);
/* Device workspace currently held by the context, in bytes (all slots). */
int         cpg_workspace_bytes(cpg_ctx* ctx, int64_t* bytes);
/* Wait for `stream` and return the first kernel-reported status since the last
 * cpg_sync: CPG_OK; CPG_E_VERIFY (a Viterbi exactness self-check failed); CPG_E_INVALID
 * (a broken contig layout); CPG_E_UNSUPPORTED (a general-model path not representable as
 * sign bits); CPG_E_DEVICE (the device reader, cpg_ingest_d).  No kernel of the decode /
 * island entry points waits for another workgroup.  The outputs of cpg_viterbi_d /
 * cpg_decode_d / cpg_islands_d are valid only once cpg_sync has returned CPG_OK for them. */
int         cpg_sync(cpg_ctx* ctx, void* stream);
/* A HIP stream whose kernels run only on the compute units set in cu_mask (mask_words
 * 32-bit words, bit i = compute unit i in the runtime's order): partitions the GPU between
 * concurrently running stages, e.g. the training pass and the latency-bound decode.
 * Pass it as `stream` to the _d entry points; destroy with cpg_stream_destroy. */
int         cpg_stream_create_cu(int device, const uint32_t* cu_mask, int mask_words,
                                 void** out);
int         cpg_stream_destroy(void* stream);

/* ---- host utilities (no device) ---------------------------------------------- */
/* The reference's initial model, CpGIslandFinder.java:155-173. */
int cpg_initial_model(cpg_model* out);

/* ASCII ingest, CpGIslandFinder.java:112-145 (mode 0 = training) and :238-259
 * (mode 1 = decode).  Maps A/a C/c G/g T/t to 0..3 and skips every other byte.
 *   mode 0: emits whole 65,536-base chunks (tail dropped); with compat_quirks != 0 an
 *           extra all-A chunk is emitted for every non-ACGT byte read while the base
 *           count sits on a chunk multiple (:130-141 runs per character).
 *   mode 1: emits whole 1,048,576-base chunks (tail never decoded, :256); with
 *           compat_quirks != 0 returns CPG_E_REF_CRASH when the reference would call
 *           observedSequence.get(i) on an empty list (:257-258); *nbases then holds
 *           the bases decoded before the crash.
 * The base count is a Java int (:107, :236): at 2^32 bases it wraps to 0 and the chunk test
 * is skipped.  Mode 1 then decodes the held chunk at the next multiple and drops the 2^20
 * bases read after the wrap (no error: the reference's clear()); mode 0 returns
 * CPG_E_REF_CRASH at the byte that brings the count to 2^32 + 65,536 (DenseVector.set past
 * its size, :133-134) — whatever compat_quirks says.
 * packed: caller buffer of cap_bases/16 words; *nbases = bases written. */
int cpg_ingest(const char* txt, size_t n, int mode, int compat_quirks,
               uint32_t* packed, int64_t cap_bases, int64_t* nbases);

/* Deterministic counter-based synthetic genome: bases
 * [start, start+n) of the genome for `seed`, '-' background from the '-' block of the
 * initial model, planted '+' islands (U[300,3000] long, mean gap 100 kbp).  start must
 * be a multiple of 32.  sign_bits may be NULL.  Multithreaded (nthreads<=0: all). */
int cpg_synth(uint64_t seed, int64_t start, int64_t n, uint32_t* packed,
              uint32_t* sign_bits, int nthreads);

/* The reducer: row-normalise init, transition rows and emission rows into a model.
 * Replaces the MAHOUT-627 reducer + BaumWelchUtils.createHmmModel (:203). */
int cpg_bw_normalize(const cpg_counts_f64* counts, cpg_model* out);
/* Labelled-count M-step (same normalisation over the integer counts). */
int cpg_counts_normalize(const cpg_counts_i64* counts, cpg_model* out);

/* The reference's text outputs, byte-exact (Java rendering of doubles: shortest
 * round-trip digits; root locale).  Both return CPG_E_CAPACITY with *nbytes = the size
 * needed when cap is too small.  No terminating NUL is written.
 *   cpg_format_islands: one line per record, String.format("%d %d %d %f %f\n", beg1, end1,
 *                       len, cg, oe) as at CpGIslandFinder.java:287-288 (%f: HALF_UP on
 *                       the shortest digits);
 *   cpg_format_model  : the trained-model file of :207-224: per state i, Double.toString
 *                       of pi[i], newline, a[i][0..7] each followed by " ", newline,
 *                       b[i][0..3] each followed by " ", newline. */
int cpg_format_islands(const cpg_island* recs, int64_t n, char* buf, int64_t cap,
                       int64_t* nbytes);
int cpg_format_model(const cpg_model* model, char* buf, int64_t cap, int64_t* nbytes);

/* ---- device path: HBM-resident inputs (device pointers), async on `stream` ----- */

/* Labelled counts over whole chunk_len chunks (tail dropped).  d_counts: device
 * buffer of CPG_COUNTS_I64_N int64 (cpg_counts_i64 layout), OVERWRITTEN. */
int cpg_count_labelled_d(cpg_ctx* ctx, const uint32_t* d_packed, const uint32_t* d_sign,
                         int64_t nbases, int64_t chunk_len, int64_t* d_counts,
                         void* stream);

/* Baum-Welch E-step (mapper) over whole chunk_len chunks; every chunk is an
 * independent observation sequence (:130-141).  d_counts: CPG_COUNTS_F64_N doubles
 * (cpg_counts_f64 layout), OVERWRITTEN.  Deterministic (fixed reduction order).
 * chunk_len: a multiple of 4096, at most 65536 (the reference's 0x10000). */
int cpg_bw_estep_d(cpg_ctx* ctx, const cpg_model* model, const uint32_t* d_packed,
                   int64_t nbases, int64_t chunk_len, double* d_counts, void* stream);

/* The training pass in one call: cpg_bw_estep_d (model, d_packed -> d_estep_counts) and
 * cpg_count_labelled_d (d_packed, d_sign -> d_label_counts) over the same whole chunk_len
 * chunks (the mapper pass of :200 over the chunks of :130-141, with the labelled counts of
 * the same chunks).  Results identical to the two calls; with chunk_len >= 16384 both run
 * in ONE launch (each E-step lane also counts its 64 bases; one finalize), otherwise as
 * the two launches.  chunk_len: a multiple of 4096, at most 65536. */
int cpg_train_pass_d(cpg_ctx* ctx, const cpg_model* model, const uint32_t* d_packed,
                     const uint32_t* d_sign, int64_t nbases, int64_t chunk_len,
                     double* d_estep_counts, int64_t* d_label_counts, void* stream);

/* The reducer over ranks (:200-203, multi-GPU): d_gathered holds `world` rank records, each
 * CPG_COUNTS_F64_N doubles (the rank's cpg_counts_f64) followed by CPG_COUNTS_I64_N int64
 * (its cpg_counts_i64) — CPG_TRAIN_RECORD_BYTES bytes, e.g. the output of one all-gather of
 * every rank's record.  d_estep (CPG_COUNTS_F64_N doubles) = the fp64 records summed in rank
 * order (bitwise identical on every rank), d_counts (CPG_COUNTS_I64_N int64) = the exact
 * integer sums.  One launch. */
#define CPG_TRAIN_RECORD_BYTES ((CPG_COUNTS_F64_N + CPG_COUNTS_I64_N) * 8)
int cpg_merge_train_d(cpg_ctx* ctx, const void* d_gathered, int world, double* d_estep,
                      int64_t* d_counts, void* stream);

/* Viterbi decode, HmmEvaluator.decode(trainedModel, chunk, true) (:260), of every
 * whole chunk_len chunk (tail not decoded, :256).  Output: the state path as sign bits
 * (state = base + (sign ? 0 : 4)), identical to Mahout's sequential fp64 Viterbi, and
 * the final best log-probability per chunk (d_score, may be NULL).  Asynchronous: the
 * outputs are valid once cpg_sync has returned CPG_OK (the kernels' self-checks report
 * through it).
 * Models: the exact parallel scan takes deterministic emission rows (b[i][i%4] == 1),
 * 0 < a[i][j] <= 1 and 0 <= pi[i] <= 1; other models with deterministic emission rows (zero
 * transitions, pi outside) run Mahout's 8-state loop (cpg_viterbi_states_d's path), and
 * cpg_sync reports CPG_E_UNSUPPORTED if their path leaves the bases' states (a dead end of
 * zero transitions: sign bits cannot carry it); non-deterministic emission rows:
 * CPG_E_UNSUPPORTED at once (use cpg_viterbi_states_d or cpg_decode_d).  chunk_len: a
 * multiple of 256 when there is more than one chunk.
 * A chunk with pi = 0 for both live states of its first base ("degenerate") decodes, as in
 * Mahout's loop, to the all-state-0 path with score -inf: its sign bits (all
 * '+') do not represent that path — a -inf d_score marks such chunks (cpg_viterbi_states_d
 * returns the states themselves). */
int cpg_viterbi_d(cpg_ctx* ctx, const cpg_model* model, const uint32_t* d_packed,
                  int64_t nbases, int64_t chunk_len, uint32_t* d_sign_out,
                  double* d_score, void* stream);

/* HmmEvaluator.decode(model, chunk, true) (:260) for ANY model the reference accepts (zero
 * transition probabilities, emission rows that are not deterministic, pi with zeros):
 * Mahout's 8-state recurrence itself, bit-identical, chunks in parallel.
 * d_states_out: one byte per position of the whole chunks (states 0..7; bytes past the last
 * whole chunk are not written); d_score: best log-probability per chunk (may be NULL).
 * chunk_len: a multiple of 16 when there is more than one chunk.  A correctness path
 * (~1 Gbase/s): cpg_viterbi_d / cpg_decode_d take it themselves for models outside the
 * exact scan's contract. */
int cpg_viterbi_states_d(cpg_ctx* ctx, const cpg_model* model, const uint32_t* d_packed,
                         int64_t nbases, int64_t chunk_len, uint8_t* d_states_out,
                         double* d_score, void* stream);

/* Island scan + filter, CpGIslandFinder.java:262-339, over every whole chunk.
 * d_out: capacity `cap` records; *d_count (device int64) receives the number of
 * kept islands (written even when > cap; records beyond cap are dropped). */
int cpg_islands_d(cpg_ctx* ctx, const uint32_t* d_packed, const uint32_t* d_sign,
                  int64_t nbases, int64_t chunk_len, cpg_island* d_out, int64_t cap,
                  int64_t* d_count, void* stream);

/* As cpg_islands_d with the chunk numbering starting at first_chunk: a shard of the
 * genome (multi-GPU) reports the same coordinates/chunk indices as the unsharded run. */
int cpg_islands_at_d(cpg_ctx* ctx, const uint32_t* d_packed, const uint32_t* d_sign,
                     int64_t nbases, int64_t chunk_len, int64_t first_chunk,
                     cpg_island* d_out, int64_t cap, int64_t* d_count, void* stream);

/* The reference's decode loop body in one call: HmmEvaluator.decode (:260) then the island
 * scan + filter (:262-339) of every whole chunk — cpg_viterbi_d followed by
 * cpg_islands_at_d(first_chunk) on the same buffers, with identical outputs (d_sign_out,
 * d_score, d_out, *d_count).  When chunk_len is a multiple of 65,536 (the reference's
 * 1 Mi decode chunk) the traceback kernel also writes the island scan's run records from
 * the sign words it produces, so the sign bits are not read back.  Any model: outside the
 * exact scan's contract the decode runs Mahout's 8-state loop (cpg_viterbi_states_d's path),
 * d_sign_out then holding state < 4 and the island scan running on the states themselves
 * (the :262-339 loop reads only them).  The outputs are valid once cpg_sync has returned
 * CPG_OK. */
int cpg_decode_d(cpg_ctx* ctx, const cpg_model* model, const uint32_t* d_packed,
                 int64_t nbases, int64_t chunk_len, int64_t first_chunk, uint32_t* d_sign_out,
                 double* d_score, cpg_island* d_out, int64_t cap, int64_t* d_count,
                 void* stream);

/* Device-side ASCII ingest: the reference's readers (CpGIslandFinder.java:112-145, mode 0 =
 * training; :238-259, mode 1 = decode) over raw text already in HBM, with exactly the
 * semantics of cpg_ingest (same quirks, same committed prefix, same error rules).  d_txt:
 * 16-byte aligned.  d_packed: capacity cap_bases bases (zeroed, then written; bases past the
 * last committed chunk may be written too, as by cpg_ingest).  *d_result (device memory)
 * receives the outcome: asynchronous on `stream`, like every "_d" entry point. */
typedef struct cpg_ingest_result {
    int64_t nbases;        /* committed bases (whole chunks), cpg_ingest's *nbases */
    int64_t status;        /* CPG_OK, CPG_E_REF_CRASH, CPG_E_CAPACITY or CPG_E_DEVICE */
    int64_t crash_byte;    /* input byte at which the reference throws, else -1 */
    int64_t valid_bases;   /* ACGT bytes in the text */
    int64_t extra_chunks;  /* all-A chunks the training reader inserts (:130-141 quirk) */
    int64_t reserved[3];
} cpg_ingest_result;
int cpg_ingest_d(cpg_ctx* ctx, const char* d_txt, int64_t n, int mode, int compat_quirks,
                 uint32_t* d_packed, int64_t cap_bases, cpg_ingest_result* d_result,
                 void* stream);

/* ---- ragged contig batches (BASELINE config C4) ------------------------------------ */
/* A batch of independent sequences in ONE packed buffer of nbases bases: contig c occupies
 * bases [offs[c], offs[c] + lens[c]), offs[c] % 64 == 0 (each contig starts a 64-base block:
 * aligned 16-B loads, whole sign words of its own), lens[c] >= 1, contigs not overlapping.
 * Build-defined batch semantics: every contig is one observation sequence exactly as one
 * whole chunk is in the reference (training :130-141 -> BW mapper :200; decode :256-260 ->
 * HmmEvaluator.decode; islands :262-339 with the contig as the chunk).  d_offs int64[n],
 * d_lens int32[n], device.  A contig breaking the contract is skipped and cpg_sync reports
 * CPG_E_INVALID.
 * d_order (may be NULL = batch order): the wavefront schedule from cpg_contigs_order_d —
 * contig indices by decreasing length, so the 64 lanes of a wave (one contig each) have
 * nearly equal work.  Results never depend on the order. */
int cpg_contigs_order_d(cpg_ctx* ctx, const int32_t* d_lens, int64_t n, int32_t* d_order,
                        void* stream);
/* labelled counts over all contigs (init = each contig's first base); as cpg_count_labelled_d */
int cpg_contigs_count_labelled_d(cpg_ctx* ctx, const uint32_t* d_packed, const uint32_t* d_sign,
                                 int64_t nbases, const int64_t* d_offs, const int32_t* d_lens,
                                 const int32_t* d_order, int64_t n, int64_t* d_counts,
                                 void* stream);
/* Baum-Welch E-step summed over contigs (each contig <= 1,048,576 bases); as cpg_bw_estep_d */
int cpg_contigs_estep_d(cpg_ctx* ctx, const cpg_model* model, const uint32_t* d_packed,
                        int64_t nbases, const int64_t* d_offs, const int32_t* d_lens,
                        const int32_t* d_order, int64_t n, double* d_counts, void* stream);
/* exact Viterbi per contig: sign bits at the contig's own bit positions of d_sign_out (a
 * buffer shaped like the packed span, 32 bases per word; bits past a contig's end are '-'),
 * best log-probability per contig in d_score[c] (may be NULL).  Model contract as
 * cpg_viterbi_d. */
int cpg_contigs_viterbi_d(cpg_ctx* ctx, const cpg_model* model, const uint32_t* d_packed,
                          int64_t nbases, const int64_t* d_offs, const int32_t* d_lens,
                          const int32_t* d_order, int64_t n, uint32_t* d_sign_out,
                          double* d_score, void* stream);
/* island scan per contig: records in contig order, beg1/end1 1-based within the contig,
 * `chunk` = contig index; an island open at a contig's end is dropped (as at a chunk end). */
int cpg_contigs_islands_d(cpg_ctx* ctx, const uint32_t* d_packed, const uint32_t* d_sign,
                          int64_t nbases, const int64_t* d_offs, const int32_t* d_lens,
                          const int32_t* d_order, int64_t n, cpg_island* d_out, int64_t cap,
                          int64_t* d_count, void* stream);

/* ---- streamed whole-genome pass (host memory -> HBM, overlapped) ---------------- */
/* One training + decode pass over a genome in HOST memory, streamed to the device in windows
 * of whole 1 Mi chunks (BASELINE config C5): H2D copies of window k+1 overlap the E-step /
 * labelled counts (train stream) and the Viterbi / island scan (decode stream) of window k,
 * and the D2H of the decoded path.  It is the reference's trainModel mapper pass (:130-141,
 * :200) and testModel (:256-339) for one genome in one call, with results identical to the
 * "_d" entry points over the whole genome at once (the E-step and count accumulators are
 * fixed point and finalized once; island records are appended in chunk order).
 *   train_model  : E-step model (NULL: no E-step; estep_out must then be NULL)
 *   decode_model : Viterbi model (NULL: no decode)
 *   sign         : truth labels for the labelled counts (NULL: none; counts_out NULL)
 *   sign_out     : decoded path as sign bits (NULL: not returned); the tail reads '-'
 *   score_out    : best log-probability per decode chunk (NULL: not returned)
 *   islands_out / island_cap / island_count : as cpg_islands (CPG_E_CAPACITY if exceeded)
 * Host buffers that are not pinned are page-locked for the duration of the call. */
typedef struct cpg_genome_opts {
    int64_t window_bases;   /* multiple of CPG_DECODE_CHUNK; 0: 64 Mi */
    int     nbuf;           /* device window buffers, 2..8; 0: 3 */
    int     reserved;
    int64_t first_chunk;    /* decode-chunk index of base 0 (a shard of a larger genome):
                               island coordinates / chunk numbers as in the unsharded run */
} cpg_genome_opts;
int cpg_genome_run(cpg_ctx* ctx, const cpg_model* train_model, const cpg_model* decode_model,
                   const uint32_t* packed, const uint32_t* sign, int64_t nbases,
                   const cpg_genome_opts* opts, cpg_counts_f64* estep_out,
                   cpg_counts_i64* counts_out, uint32_t* sign_out, double* score_out,
                   cpg_island* islands_out, int64_t island_cap, int64_t* island_count);

/* ---- host-buffer entry points (stage through pinned memory, synchronous) ------- */
int cpg_count_labelled(cpg_ctx* ctx, const uint32_t* packed, const uint32_t* sign,
                       int64_t nbases, int64_t chunk_len, cpg_counts_i64* out);
int cpg_bw_estep(cpg_ctx* ctx, const cpg_model* model, const uint32_t* packed,
                 int64_t nbases, int64_t chunk_len, cpg_counts_f64* out);
int cpg_viterbi(cpg_ctx* ctx, const cpg_model* model, const uint32_t* packed,
                int64_t nbases, int64_t chunk_len, uint32_t* sign_out, double* score);
/* Exact HmmEvaluator.decode(model, obs, true) (:260) for one observation array:
 * obs[i] in 0..3 (else CPG_E_INVALID, the reference's ArrayIndexOutOfBounds), n >= 1.
 * states_out[i] in 0..7. */
int cpg_decode_states(cpg_ctx* ctx, const cpg_model* model, const int32_t* obs,
                      int64_t n, int32_t* states_out);
/* cpg_ingest computed on the GPU: host text staged through pinned memory, the packed
 * chunks copied back.  Same arguments, results and return codes as cpg_ingest. */
int cpg_ingest_gpu(cpg_ctx* ctx, const char* txt, size_t n, int mode, int compat_quirks,
                   uint32_t* packed, int64_t cap_bases, int64_t* nbases);
int cpg_islands(cpg_ctx* ctx, const uint32_t* packed, const uint32_t* sign,
                int64_t nbases, int64_t chunk_len, cpg_island* out, int64_t cap,
                int64_t* count);

#ifdef __cplusplus
}
#endif
#endif /* CPG_H_ */
