// k_reduce.hip — the training pass's reducer over ranks.
//
// Replaces the reducer's sum of the mapper outputs (CpGIslandFinder.java:200-203, Mahout
// BaumWelchReducer) across ranks: every rank contributes one record — its E-step counts
// (cpg_counts_f64, 105 doubles) followed by its labelled counts (cpg_counts_i64, 124 int64) —
// and after ONE all-gather of the records every rank sums them itself: the doubles in rank
// order (bitwise identical on every rank and across runs, whatever the collective's
// algorithm), the integers exactly.  One launch of one workgroup, instead of a collective per
// output plus a chain of small element-wise kernels.

#include "cpg_internal.h"

namespace cpg {
namespace {

constexpr int kF = CPG_COUNTS_F64_N, kI = CPG_COUNTS_I64_N, kRec = kF + kI;

__global__ __launch_bounds__(256) void k_merge_train(const unsigned long long* __restrict__ g,
                                                     int world, double* __restrict__ estep,
                                                     int64_t* __restrict__ counts) {
    const int t = threadIdx.x;
    if (t < kF) {
        double s = 0.0;
        for (int r = 0; r < world; ++r) s += __longlong_as_double((long long)g[r * kRec + t]);
        estep[t] = s;
    } else if (t < kRec) {
        int64_t s = 0;
        for (int r = 0; r < world; ++r) s += (int64_t)g[r * kRec + t];
        counts[t - kF] = s;
    }
}

}  // namespace

hipError_t launch_merge_train(const void* gathered, int world, double* estep, int64_t* counts,
                              hipStream_t s) {
    hipLaunchKernelGGL(k_merge_train, dim3(1), dim3(256), 0, s,
                       static_cast<const unsigned long long*>(gathered), world, estep, counts);
    return hipGetLastError();
}

}  // namespace cpg
