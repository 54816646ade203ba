/*
 * cpg_oracle.h — CPU restatement of CpGIslandFinder's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker (or as the timed
 * CPU baseline).  The product (libcpg.so) never links or calls it.
 *
 * PARITY UNPINNED: the reference (Java + unvendored Mahout / MAHOUT-627 / Hadoop) cannot
 * be compiled or run in this container (no JDK, no jars, no network; SURVEY.md §0.2-0.3,
 * §8c) and ships no tests or golden vectors.  This restatement follows
 * /root/reference/CpGIslandFinder.java line by line where the logic is in that file, and
 * Apache Mahout's HmmAlgorithms.viterbiAlgorithm (scaled=true, public source, version
 * unpinned) for the decode; the Baum-Welch E-step follows Rabiner's rescaled
 * forward-backward (MAHOUT-627's exact convention is not available).  It is cross-checked
 * against an independent Python restatement (oracle/pyref.py) and hand-derived
 * known-answer tests (tests/test_oracle.py).
 */
#ifndef CPG_ORACLE_H_
#define CPG_ORACLE_H_
#include <stdint.h>
#include "../include/cpg.h"

#ifdef __cplusplus
extern "C" {
#endif

void    orc_initial_model(cpg_model* m);

/* CpGIslandFinder.java:112-145: symbols (0..3, one byte each) of the training chunk
 * stream, including the all-A quirk chunks; returns the number of symbols written
 * (a multiple of 65536) or -1 if cap would be exceeded. */
int64_t orc_ingest_train(const uint8_t* txt, int64_t n, uint8_t* syms, int64_t cap);
/* CpGIslandFinder.java:238-259: symbols of the decoded chunks; *crash = 1 when the
 * reference throws (get(i) on an empty list), the return value then counts the symbols
 * of the chunks decoded before it. */
int64_t orc_ingest_decode(const uint8_t* txt, int64_t n, uint8_t* syms, int64_t cap,
                          int* crash);
/* The same readers starting from Java `count` = count0 with an empty list (a test hook for
 * the 2^32 wrap of the int counter: count0 a multiple of the chunk below 2^32).  The
 * training reader's crash at the wrap (DenseVector.set(65536), :133-134) and the decode
 * reader's (get(i) on an empty list) report the input byte in *crash_byte (-1: none). */
int64_t orc_ingest_train_at(const uint8_t* txt, int64_t n, uint8_t* syms, int64_t cap,
                            uint32_t count0, int64_t* crash_byte);
int64_t orc_ingest_decode_at(const uint8_t* txt, int64_t n, uint8_t* syms, int64_t cap,
                             uint32_t count0, int* crash, int64_t* crash_byte);

/* Mahout HmmAlgorithms.viterbiAlgorithm(model, obs, scaled=true), 8 states, Math.log in
 * the inner loop exactly as Mahout does.  states_out[T]; returns max final delta. */
double  orc_viterbi8(const cpg_model* m, const uint8_t* obs, int64_t T, int32_t* states_out);
/* Same recurrence collapsed to the two live states, logs
 * precomputed.  sign_out[t] = 1 for '+'.  Returns max final delta. */
double  orc_viterbi2(const cpg_model* m, const uint8_t* obs, int64_t T, uint8_t* sign_out);

/* Rabiner-rescaled forward-backward over one observation sequence, 8 states;
 * ACCUMULATES into acc (init += gamma_0, trans += sum xi, emit += sum gamma,
 * loglik += log P). */
void    orc_estep8(const cpg_model* m, const uint8_t* obs, int64_t T, cpg_counts_f64* acc);
/* Reducer: row-normalise. */
void    orc_normalize(const cpg_counts_f64* c, cpg_model* out);

/* Labelled integer counts over whole chunks of chunk_len (tail dropped); ACCUMULATES. */
void    orc_count_labelled(const uint8_t* obs, const uint8_t* sign, int64_t n,
                           int64_t chunk_len, cpg_counts_i64* acc);

/* Island scan + filter, CpGIslandFinder.java:262-339, of ONE decoded chunk:
 * states[T] (0..7), chunk index for the coordinates.  Returns the number of records
 * kept (records beyond cap are counted but not written). */
int64_t orc_islands(const int32_t* states, int64_t T, int32_t chunk, cpg_island* out,
                    int64_t cap);

/* Java String.format("%d %d %d %f %f\n", ...) of one record (Formatter HALF_UP on the
 * shortest repr digits).  Returns bytes written (excluding NUL). */
int     orc_format_island(const cpg_island* r, char* buf, int cap);

#ifdef __cplusplus
}
#endif
#endif
