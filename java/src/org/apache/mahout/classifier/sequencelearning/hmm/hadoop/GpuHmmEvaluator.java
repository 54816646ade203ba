package org.apache.mahout.classifier.sequencelearning.hmm.hadoop;

import java.lang.foreign.Arena;
import java.lang.foreign.MemorySegment;

import static java.lang.foreign.ValueLayout.JAVA_INT;

import org.apache.mahout.classifier.sequencelearning.hmm.HmmEvaluator;
import org.apache.mahout.classifier.sequencelearning.hmm.HmmModel;

/**
 * Drop-in for {@code HmmEvaluator.decode(trainedModel, testSequence, true)} at
 * CpGIslandFinder.java:260: the state path of Mahout's scaled Viterbi, exact (cpg_decode_states:
 * the same fp64 recurrence and '>' tie-break, any model).  In testModel the line becomes
 * {@code int[] hiddenStates = GpuHmmEvaluator.decode(trainedModel, testSequence, true);}
 *
 * NOT COMPILED OR RUN here (no JDK in the image); its C side is what tests/ exercise.
 */
public final class GpuHmmEvaluator {
  private GpuHmmEvaluator() {}

  public static int[] decode(HmmModel model, int[] observations, boolean scaled) {
    if (!scaled) return HmmEvaluator.decode(model, observations, false);   // not the hot path
    if (observations.length == 0) throw new NegativeArraySizeException();  // as Mahout's does
    try (Arena a = Arena.ofConfined()) {
      MemorySegment obs = a.allocateFrom(JAVA_INT, observations);
      MemorySegment out = a.allocate(JAVA_INT, observations.length);
      Cpg.check((int) Cpg.DECODE_STATES.invokeExact(Cpg.CTX, Cpg.model(a, model), obs,
                                                     (long) observations.length, out));
      return out.toArray(JAVA_INT);
    } catch (RuntimeException e) {
      throw e;
    } catch (Throwable t) {
      throw new IllegalStateException(t);
    }
  }
}
