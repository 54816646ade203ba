package org.apache.mahout.classifier.sequencelearning.hmm.hadoop;

import java.io.IOException;
import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;

import static java.lang.foreign.ValueLayout.JAVA_DOUBLE;
import static java.lang.foreign.ValueLayout.JAVA_INT;

import org.apache.hadoop.io.DoubleWritable;
import org.apache.hadoop.io.IntWritable;
import org.apache.hadoop.io.LongWritable;
import org.apache.hadoop.io.MapWritable;
import org.apache.hadoop.io.Text;
import org.apache.hadoop.mapreduce.Mapper;
import org.apache.mahout.classifier.sequencelearning.hmm.HmmModel;
import org.apache.mahout.math.Vector;
import org.apache.mahout.math.VectorWritable;

/**
 * The Baum-Welch mapper (MAHOUT-627, called through BaumWelchDriver.runBaumWelchMR at
 * CpGIslandFinder.java:200-201) on the GPU: the chunks of an input split — the 65,536-symbol
 * VectorWritables trainModel writes (:130-141) — are packed 16 symbols per int and their
 * rescaled forward-backward expected counts summed by ONE cpg_bw_estep call per batch (the
 * GPU pays off on many chunks per call, not one), emitted in cleanup() as the stripes the
 * reducer sums: "INITIAL" (8), "TRANSIT_i" (row i of 8), "EMIT_i" (row i of 4).
 *
 * The stripe key names follow the MAHOUT-627 patch's description; that patch was never released
 * or vendored (SURVEY.md §0.2), so its exact naming is UNPINNED.  The model is loaded by
 * loadModel(), which the deployment wires to its BaumWelchUtils model path.
 *
 * NOT COMPILED OR RUN here (no JDK, no Hadoop / Mahout jars in the image).
 */
public class GpuBaumWelchMapper extends Mapper<LongWritable, VectorWritable, Text, MapWritable> {
  static final int CHUNK = (int) Cpg.TRAIN_CHUNK;
  static final int BATCH_CHUNKS = 1024;   // 64 Mi symbols per downcall

  private HmmModel model;
  private Arena arena;
  private MemorySegment packed;      // BATCH_CHUNKS chunks of CHUNK / 16 ints
  private int nbatched;
  private final double[] sum = new double[105];   // cpg_counts_f64, summed over batches

  /** The current iteration's model (BaumWelchConfigKeys model path); deployment-specific. */
  protected HmmModel loadModel(Context context) throws IOException {
    throw new UnsupportedOperationException("wire to BaumWelchUtils.createHmmModel");
  }

  @Override
  protected void setup(Context context) throws IOException {
    model = loadModel(context);
    arena = Arena.ofShared();
    packed = arena.allocate(JAVA_INT, (long) BATCH_CHUNKS * (CHUNK / 16));
  }

  @Override
  protected void map(LongWritable key, VectorWritable value, Context context) {
    Vector v = value.get();
    if (v.size() != CHUNK) return;   // trainModel writes whole chunks only (:130-141)
    long base = (long) nbatched * (CHUNK / 16);
    for (int w = 0; w < CHUNK / 16; w++) {
      int word = 0;
      for (int k = 0; k < 16; k++) word |= ((int) v.getQuick(16 * w + k) & 3) << (2 * k);
      packed.setAtIndex(JAVA_INT, base + w, word);
    }
    if (++nbatched == BATCH_CHUNKS) flush();
  }

  private void flush() {
    if (nbatched == 0) return;
    try (Arena a = Arena.ofConfined()) {
      MemorySegment out = a.allocate(Cpg.CPG_COUNTS_F64);
      Cpg.check((int) Cpg.BW_ESTEP.invokeExact(Cpg.CTX, Cpg.model(a, model), packed,
                                               (long) nbatched * CHUNK, (long) CHUNK, out));
      for (int i = 0; i < 105; i++) sum[i] += out.getAtIndex(JAVA_DOUBLE, i);
    } catch (RuntimeException e) {
      throw e;
    } catch (Throwable t) {
      throw new IllegalStateException(t);
    }
    nbatched = 0;
  }

  private static MapWritable stripe(double[] s, int off, int n) {
    MapWritable m = new MapWritable();
    for (int j = 0; j < n; j++) m.put(new IntWritable(j), new DoubleWritable(s[off + j]));
    return m;
  }

  @Override
  protected void cleanup(Context context) throws IOException, InterruptedException {
    flush();
    context.write(new Text("INITIAL"), stripe(sum, 0, 8));
    for (int i = 0; i < 8; i++) context.write(new Text("TRANSIT_" + i), stripe(sum, 8 + 8 * i, 8));
    for (int i = 0; i < 8; i++) context.write(new Text("EMIT_" + i), stripe(sum, 72 + 4 * i, 4));
    arena.close();
  }
}
