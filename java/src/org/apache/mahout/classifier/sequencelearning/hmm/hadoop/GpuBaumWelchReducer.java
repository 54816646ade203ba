package org.apache.mahout.classifier.sequencelearning.hmm.hadoop;

import java.io.IOException;
import java.util.Map;

import org.apache.hadoop.io.DoubleWritable;
import org.apache.hadoop.io.IntWritable;
import org.apache.hadoop.io.MapWritable;
import org.apache.hadoop.io.Text;
import org.apache.hadoop.io.Writable;
import org.apache.hadoop.mapreduce.Reducer;

/**
 * The Baum-Welch reducer (MAHOUT-627, behind runBaumWelchMR at CpGIslandFinder.java:200-203) for
 * GpuBaumWelchMapper's stripes: the stripes of one key summed in arrival order, then the row
 * normalised as cpg_bw_normalize does it (sum left to right, each entry / the sum) — so a
 * model rebuilt from these rows equals cpg_bw_normalize of the summed cpg_counts_f64 when the
 * stripes arrive in chunk order.  Stripe key names: UNPINNED (see GpuBaumWelchMapper).
 *
 * NOT COMPILED OR RUN here (no JDK, no Hadoop jars in the image).
 */
public class GpuBaumWelchReducer extends Reducer<Text, MapWritable, Text, MapWritable> {
  @Override
  protected void reduce(Text key, Iterable<MapWritable> stripes, Context context)
      throws IOException, InterruptedException {
    int n = key.toString().startsWith("EMIT_") ? 4 : 8;
    double[] row = new double[n];
    for (MapWritable s : stripes)
      for (Map.Entry<Writable, Writable> e : s.entrySet())
        row[((IntWritable) e.getKey()).get()] += ((DoubleWritable) e.getValue()).get();
    double total = 0.0;
    for (int j = 0; j < n; j++) total += row[j];
    MapWritable out = new MapWritable();
    for (int j = 0; j < n; j++) out.put(new IntWritable(j), new DoubleWritable(row[j] / total));
    context.write(key, out);
  }
}
