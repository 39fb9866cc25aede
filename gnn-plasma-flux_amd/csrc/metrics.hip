// Rollout scoring over the per-step metrics the rollout kernels write
// (SURVEY.md 8f rank 1): the per-IC numbers the reference's evaluation
// scripts compute on host trajectories, here from the device-resident
// [B][T+1][HF_NUM_METRICS] series (and the [B][T+1][3] MSE series of
// hf_run_compare), one thread per IC.
//
//  - explosion tracking: the first step whose state is not finite, and the
//    steps completed before it (scripts/evaluation/evaluate_long_rollout.py:53-66);
//  - energy / charge drift |x_t - x_0| (evaluate_all.py:135-143,
//    evaluate_long_rollout.py:38-45,72), final values at the last finite
//    step (evaluate_long_rollout.py:72-74; = evaluate_all.py:157-158 when
//    nothing exploded);
//  - MSE totals: mse_n + mse_u + mse_E per step, its final value and its mean
//    over t = 0..T (evaluate_all.py:129-132,155-156; evaluate_multi_ic.py:88-94).
//
// HBM-bound and tiny (K floats per IC-step read once); it runs after the
// rollout on the same stream, so a multi-GPU job gathers its summaries with the
// metric series.
#include "hf_internal.h"

namespace hf {
namespace {

constexpr int kSumThreads = 256;

__global__ __launch_bounds__(kSumThreads) void rollout_summary_kernel(const float *__restrict__ met,
                                                                     const float *__restrict__ mse,
                                                                     const float *__restrict__ met_ref, int B,
                                                                     int T, float *__restrict__ summary,
                                                                     float *__restrict__ drift) {
  const int64_t b = (int64_t)blockIdx.x * kSumThreads + threadIdx.x;
  if (b >= B) return;
  const int K = HF_NUM_METRICS, T1 = T + 1;
  const float *m = met + b * T1 * K;
  const float nanf_ = __int_as_float(0x7fc00000);
  // evaluate_long_rollout.py:53-66: stepping stops at the first non-finite state
  int exploded = -1;
  for (int t = 1; t <= T; ++t)
    if (m[t * K + 2] == 0.f) {
      exploded = t;
      break;
    }
  const int actual = exploded < 0 ? T : exploded - 1;
  const float e0 = m[0], q0 = m[1];
  float *sm = summary + b * HF_NUM_SUMMARY;
  sm[0] = (float)exploded;
  sm[1] = (float)actual;
  sm[2] = fabsf(m[actual * K + 0] - e0);
  sm[3] = fabsf(m[actual * K + 1] - q0);
  if (mse) {
    const float *ms = mse + b * T1 * 3;
    double acc = 0.0;
    float last = 0.f;
    for (int t = 0; t <= T; ++t) {
      // float32 (n + u) + E, as numpy adds the three float32 series
      last = __fadd_rn(__fadd_rn(ms[t * 3 + 0], ms[t * 3 + 1]), ms[t * 3 + 2]);
      acc += (double)last;
    }
    sm[4] = last;
    sm[5] = (float)(acc / T1);
  } else {
    sm[4] = sm[5] = nanf_;
  }
  const float *r = met_ref ? met_ref + b * T1 * K : nullptr;
  sm[6] = r ? fabsf(r[T * K + 0] - r[0]) : nanf_;
  sm[7] = r ? fabsf(r[T * K + 1] - r[1]) : nanf_;
  if (drift) {
    float *d = drift + b * T1 * 4;
    for (int t = 0; t <= T; ++t) {
      d[t * 4 + 0] = fabsf(m[t * K + 0] - e0);
      d[t * 4 + 1] = fabsf(m[t * K + 1] - q0);
      d[t * 4 + 2] = r ? fabsf(r[t * K + 0] - r[0]) : nanf_;
      d[t * 4 + 3] = r ? fabsf(r[t * K + 1] - r[1]) : nanf_;
    }
  }
}

}  // namespace

hipError_t launch_rollout_summary(const float *met, const float *mse, const float *met_ref, int B, int T,
                                  float *summary, float *drift, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(rollout_summary_kernel, dim3((B + kSumThreads - 1) / kSumThreads), dim3(kSumThreads), 0, s,
                     met, mse, met_ref, B, T, summary, drift);
  return hipGetLastError();
}

}  // namespace hf
