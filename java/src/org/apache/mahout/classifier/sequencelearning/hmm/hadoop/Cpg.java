package org.apache.mahout.classifier.sequencelearning.hmm.hadoop;

import java.lang.foreign.Arena;
import java.lang.foreign.FunctionDescriptor;
import java.lang.foreign.Linker;
import java.lang.foreign.MemoryLayout;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.StructLayout;
import java.lang.foreign.SymbolLookup;
import java.lang.invoke.MethodHandle;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_DOUBLE;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

import org.apache.mahout.classifier.sequencelearning.hmm.HmmModel;

/**
 * Panama FFM (JDK 22+) downcalls into libcpg.so, the MI355X hot path of CpGIslandFinder
 * (include/cpg.h).  Same package as the reference (CpGIslandFinder.java:1), so the adapters sit
 * beside the MAHOUT-627 classes they replace.
 *
 * NOT COMPILED OR RUN in this build's container: the image has no JDK.  The struct layouts
 * below are checked against the C header's sizeof / offsetof by tests/test_java_layout.py
 * (a C probe compiled with gcc); the downcalls themselves are unverified.
 *
 * One context per device; the context serialises its calls (cpg.h: one call at a time per
 * context, separate contexts run concurrently).  Errors: a negative status is mapped to the
 * exception the reference would have thrown (check()).
 */
public final class Cpg {
  private Cpg() {}

  // ---- struct layouts of include/cpg.h (state order A+ C+ G+ T+ A- C- G- T-, :182-189) -----
  /** cpg_model: pi[8] | a[8][8] | b[8][4], row-major (:155-173). */
  public static final StructLayout CPG_MODEL = MemoryLayout.structLayout(
      MemoryLayout.sequenceLayout(8, JAVA_DOUBLE).withName("pi"),
      MemoryLayout.sequenceLayout(64, JAVA_DOUBLE).withName("a"),
      MemoryLayout.sequenceLayout(32, JAVA_DOUBLE).withName("b")).withName("cpg_model");

  /** cpg_counts_f64: the mapper's stripes (initial, transition rows, emission rows) + loglik. */
  public static final StructLayout CPG_COUNTS_F64 = MemoryLayout.structLayout(
      MemoryLayout.sequenceLayout(8, JAVA_DOUBLE).withName("init"),
      MemoryLayout.sequenceLayout(64, JAVA_DOUBLE).withName("trans"),
      MemoryLayout.sequenceLayout(32, JAVA_DOUBLE).withName("emit"),
      JAVA_DOUBLE.withName("loglik")).withName("cpg_counts_f64");

  /** cpg_counts_i64: labelled int64 counts, same stripes + dinucleotide / mononucleotide. */
  public static final StructLayout CPG_COUNTS_I64 = MemoryLayout.structLayout(
      MemoryLayout.sequenceLayout(8, JAVA_LONG).withName("init"),
      MemoryLayout.sequenceLayout(64, JAVA_LONG).withName("trans"),
      MemoryLayout.sequenceLayout(32, JAVA_LONG).withName("emit"),
      MemoryLayout.sequenceLayout(16, JAVA_LONG).withName("dinuc"),
      MemoryLayout.sequenceLayout(4, JAVA_LONG).withName("mono")).withName("cpg_counts_i64");

  /** cpg_island: one line of the island file, "%d %d %d %f %f\n" (:287-288). */
  public static final StructLayout CPG_ISLAND = MemoryLayout.structLayout(
      JAVA_INT.withName("beg1"),
      JAVA_INT.withName("end1"),
      JAVA_INT.withName("len"),
      JAVA_INT.withName("chunk"),
      JAVA_DOUBLE.withName("cg"),
      JAVA_DOUBLE.withName("oe")).withName("cpg_island");

  public static final int CPG_OK = 0;
  public static final int CPG_E_INVALID = -1;
  public static final long TRAIN_CHUNK = 65536L;     // :130-131
  public static final long DECODE_CHUNK = 1048576L;  // :230, :256-257

  // ---- downcalls -------------------------------------------------------------------------
  private static final Linker L = Linker.nativeLinker();
  private static final SymbolLookup LIB =
      SymbolLookup.libraryLookup(System.getProperty("cpg.lib", "libcpg.so"), Arena.global());

  private static MethodHandle h(String name, FunctionDescriptor d) {
    return L.downcallHandle(LIB.find(name).orElseThrow(), d);
  }

  static final MethodHandle OPEN = h("cpg_open", FunctionDescriptor.of(JAVA_INT, JAVA_INT, ADDRESS));
  static final MethodHandle ERR = h("cpg_last_error", FunctionDescriptor.of(ADDRESS));
  /** int cpg_decode_states(ctx, model, const int32_t* obs, int64_t n, int32_t* states) */
  static final MethodHandle DECODE_STATES = h("cpg_decode_states",
      FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS));
  /** int cpg_bw_estep(ctx, model, const uint32_t* packed, nbases, chunk_len, cpg_counts_f64*) */
  static final MethodHandle BW_ESTEP = h("cpg_bw_estep",
      FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, JAVA_LONG, JAVA_LONG, ADDRESS));
  /** int cpg_bw_normalize(const cpg_counts_f64*, cpg_model*) */
  static final MethodHandle BW_NORMALIZE = h("cpg_bw_normalize",
      FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS));
  /** int cpg_viterbi(ctx, model, packed, nbases, chunk_len, sign_out, score) */
  static final MethodHandle VITERBI = h("cpg_viterbi",
      FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, JAVA_LONG, JAVA_LONG, ADDRESS, ADDRESS));
  /** int cpg_islands(ctx, packed, sign, nbases, chunk_len, out, cap, count) */
  static final MethodHandle ISLANDS = h("cpg_islands",
      FunctionDescriptor.of(JAVA_INT, ADDRESS, ADDRESS, ADDRESS, JAVA_LONG, JAVA_LONG, ADDRESS,
                            JAVA_LONG, ADDRESS));

  /** The cpg_ctx* of device 0 (property cpg.device), opened once. */
  public static final MemorySegment CTX;
  static {
    try (Arena a = Arena.ofConfined()) {
      MemorySegment out = a.allocate(ADDRESS);
      check((int) OPEN.invokeExact(Integer.getInteger("cpg.device", 0), out));
      CTX = out.get(ADDRESS, 0);
    } catch (Throwable t) {
      throw new ExceptionInInitializerError(t);
    }
  }

  /** Negative status -> the reference's exception family (cpg.h conventions). */
  public static void check(int rc) {
    if (rc >= 0) return;
    String msg;
    try {
      msg = ((MemorySegment) ERR.invokeExact()).reinterpret(4096).getString(0);
    } catch (Throwable t) {
      msg = "?";
    }
    if (rc == CPG_E_INVALID) throw new ArrayIndexOutOfBoundsException(msg);
    throw new IllegalStateException("libcpg " + rc + ": " + msg);
  }

  /** A Mahout HmmModel as a cpg_model segment (the getters of :204-206 / :208-222). */
  public static MemorySegment model(Arena a, HmmModel m) {
    MemorySegment s = a.allocate(CPG_MODEL);
    for (int i = 0; i < 8; i++) s.setAtIndex(JAVA_DOUBLE, i, m.getInitialProbabilities().get(i));
    for (int i = 0; i < 8; i++)
      for (int j = 0; j < 8; j++)
        s.setAtIndex(JAVA_DOUBLE, 8 + 8 * i + j, m.getTransitionMatrix().get(i, j));
    for (int i = 0; i < 8; i++)
      for (int k = 0; k < 4; k++)
        s.setAtIndex(JAVA_DOUBLE, 72 + 4 * i + k, m.getEmissionMatrix().get(i, k));
    return s;
  }

  /** Symbols 0..3 (the reference's A/C/G/T, :114-123) -> packed words, 16 per int, base k at
   *  bits 2(k mod 16) (include/cpg.h layout). */
  public static MemorySegment pack(Arena a, double[] symbols, int n) {
    MemorySegment s = a.allocate(JAVA_INT, (n + 15) / 16);
    for (int k = 0; k < n; k++) {
      int v = (int) symbols[k];
      if (v < 0 || v > 3) throw new ArrayIndexOutOfBoundsException(v);
      long idx = k >>> 4;
      int w = s.getAtIndex(JAVA_INT, idx);
      s.setAtIndex(JAVA_INT, idx, w | (v << (2 * (k & 15))));
    }
    return s;
  }
}
