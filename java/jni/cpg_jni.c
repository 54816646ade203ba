/* cpg_jni.c — JNI fallback (JDK < 22) for GpuHmmEvaluator.decode (CpGIslandFinder.java:260)
 * over libcpg.so.  NOT BUILT here (no JDK, so no jni.h in the image):
 *   gcc -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *       java/jni/cpg_jni.c -Lcpgisland_amd -lcpg -o libcpg_jni.so
 * Java side:  static native int decodeStates(double[] model104, int[] obs, int[] states);
 * a negative return is a CPG_E_* code, mapped to exceptions as Cpg.check does. */
#include <jni.h>

#include "cpg.h"

static cpg_ctx* ctx;

JNIEXPORT jint JNICALL Java_org_apache_mahout_classifier_sequencelearning_hmm_hadoop_GpuHmmEvaluator_decodeStates(
    JNIEnv* env, jclass cls, jdoubleArray model, jintArray obs, jintArray out) {
    (void)cls;
    if (!ctx && cpg_open(0, &ctx) != CPG_OK) return CPG_E_DEVICE;
    if ((*env)->GetArrayLength(env, model) != 104) return CPG_E_INVALID;
    const jsize n = (*env)->GetArrayLength(env, obs);
    if ((*env)->GetArrayLength(env, out) < n) return CPG_E_INVALID;
    double* m = (*env)->GetPrimitiveArrayCritical(env, model, 0);
    jint* o = (*env)->GetPrimitiveArrayCritical(env, obs, 0);
    jint* s = (*env)->GetPrimitiveArrayCritical(env, out, 0);
    const int rc = cpg_decode_states(ctx, (const cpg_model*)m, o, n, s);
    (*env)->ReleasePrimitiveArrayCritical(env, out, s, 0);
    (*env)->ReleasePrimitiveArrayCritical(env, obs, o, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, model, m, JNI_ABORT);
    return rc;
}
