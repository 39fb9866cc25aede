// Finite-volume update + spectral (circulant) Poisson solve for any nx.
//
// One 256-thread workgroup per IC; the IC's chain lives in LDS for the
// update and the O(nx^2) float64 circulant product (src/baseline_solver.py:
// 59-101, src/hybrid_solver.py:45-63).  HBM traffic per cell-step is the
// 12 B state read + 12 B state write (+4 B face flux in hybrid mode).
#include "hf_device.h"
#include "hf_internal.h"

namespace hf {
namespace {

constexpr int kFvThreads = 256;

__device__ __forceinline__ void block_metrics(MetricAcc &m, float *dst, int nx) {
  __shared__ double s_e[kFvThreads / 64], s_q[kFvThreads / 64];
  __shared__ float s_m[kFvThreads / 64];
  __shared__ int s_f[kFvThreads / 64];
  m.wave_reduce();
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s_e[w] = m.energy;
    s_q[w] = m.charge;
    s_m[w] = m.maxdev;
    s_f[w] = m.finite;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    MetricAcc t;
    t.init();
    for (int i = 0; i < kFvThreads / 64; ++i) {
      t.energy += s_e[i];
      t.charge += s_q[i];
      t.maxdev = s_m[i] > t.maxdev ? s_m[i] : t.maxdev;
      t.finite &= s_f[i];
    }
    t.store(dst, nx);
  }
}

// LDS: c[nx] (double) | u, F, rho, E (float) | FFT buffers 2 x nx double2 (FFT nx only)
inline size_t fv_lds_bytes(int nx) {
  size_t b = (size_t)nx * (sizeof(double) + 4 * sizeof(float));
  if (poisson_uses_fft(nx)) b = ((b + 15) & ~size_t(15)) + 2 * sizeof(double2) * nx;
  return b;
}

template <bool HYBRID>
__global__ __launch_bounds__(kFvThreads) void fv_step_kernel(
    const float *__restrict__ in, int64_t ld_in, float *__restrict__ out, int64_t ld_out,
    const float *__restrict__ face_flux, const double *__restrict__ pc, int nx, float c, float dt,
    float nu, float dx2, float *__restrict__ flux_out, int64_t ld_flux, float *__restrict__ metrics,
    int64_t ld_metrics) {
  extern __shared__ double s_dyn[];
  double *s_c = s_dyn;
  float *s_u = reinterpret_cast<float *>(s_c + nx);
  float *s_F = s_u + nx;
  float *s_rho = s_F + nx;
  float *s_E = s_rho + nx;
  const bool fft = poisson_uses_fft(nx);
  double2 *fa = reinterpret_cast<double2 *>(reinterpret_cast<char *>(s_dyn) +
                                            (((size_t)nx * (sizeof(double) + 4 * sizeof(float)) + 15) & ~size_t(15)));
  const int64_t b = blockIdx.x;
  const float *st = in + b * ld_in;
  float *so = out + b * ld_out;
  for (int i = threadIdx.x; i < nx; i += kFvThreads) {
    const float u = st[nx + i];
    s_u[i] = u;
    s_F[i] = HYBRID ? face_flux[b * nx + i] : __fmul_rn(st[i], u);  // F_n = n*u (:70-71)
    if (!fft) s_c[i] = pc[i];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nx; i += kFvThreads) {
    const int im = i == 0 ? nx - 1 : i - 1;
    const int ip = i == nx - 1 ? 0 : i + 1;
    const float F = s_F[i];
    const float n_new = continuity(st[i], F, s_F[im], c);
    const float E = st[2 * nx + i];
    const float u_new = HYBRID ? velocity_hybrid(s_u[i], s_u[im], E, c, dt)
                               : velocity_classical(s_u[i], s_u[im], s_u[ip], E, c, dt, nu, dx2);
    s_rho[i] = __fsub_rn(n_new, 1.0f);
    so[i] = n_new;
    so[nx + i] = u_new;
    if (flux_out) flux_out[b * ld_flux + i] = F;
  }
  __syncthreads();
  if (fft) poisson_fft(s_rho, fa, fa + nx, pc, nx, s_E);
  MetricAcc m;
  m.init();
  for (int i = threadIdx.x; i < nx; i += kFvThreads) {
    const float E_new = fft ? s_E[i] : poisson_cell(s_rho, s_c, i, nx);
    so[2 * nx + i] = E_new;
    if (metrics) m.add(so[i], so[nx + i], E_new);
  }
  if (metrics) block_metrics(m, metrics + b * ld_metrics, nx);
}

__global__ __launch_bounds__(kFvThreads) void state_metrics_kernel(const float *__restrict__ st,
                                                                   int64_t ld, int nx,
                                                                   float *__restrict__ metrics,
                                                                   int64_t ld_metrics) {
  const int64_t b = blockIdx.x;
  const float *s = st + b * ld;
  MetricAcc m;
  m.init();
  for (int i = threadIdx.x; i < nx; i += kFvThreads) m.add(s[i], s[nx + i], s[2 * nx + i]);
  block_metrics(m, metrics + b * ld_metrics, nx);
}

__global__ __launch_bounds__(kFvThreads) void poisson_kernel(const float *__restrict__ n, int ld_n,
                                                             float *__restrict__ E, int ld_E,
                                                             const double *__restrict__ pc,
                                                             int nx) {
  extern __shared__ double s_dyn[];
  double *s_c = s_dyn;
  float *s_u = reinterpret_cast<float *>(s_c + nx);  // unused: keeps the fv LDS layout
  float *s_rho = s_u + 2 * nx;
  float *s_E = s_rho + nx;
  const bool fft = poisson_uses_fft(nx);
  double2 *fa = reinterpret_cast<double2 *>(reinterpret_cast<char *>(s_dyn) +
                                            (((size_t)nx * (sizeof(double) + 4 * sizeof(float)) + 15) & ~size_t(15)));
  const int64_t b = blockIdx.x;
  for (int i = threadIdx.x; i < nx; i += kFvThreads) {
    if (!fft) s_c[i] = pc[i];
    s_rho[i] = __fsub_rn(n[b * ld_n + i], 1.0f);  // rho = n - n0 (:60)
  }
  __syncthreads();
  if (fft) poisson_fft(s_rho, fa, fa + nx, pc, nx, s_E);
  for (int i = threadIdx.x; i < nx; i += kFvThreads)
    E[b * ld_E + i] = fft ? s_E[i] : poisson_cell(s_rho, s_c, i, nx);
}

// Per-step channel MSE of two trajectories (scripts/evaluation/evaluate_multi_ic.py:88-90).
__global__ __launch_bounds__(kFvThreads) void traj_mse_kernel(const float *__restrict__ a,
                                                              const float *__restrict__ b, int nx,
                                                              float *__restrict__ mse) {
  __shared__ double s_part[kFvThreads / 64];
  const int64_t row = blockIdx.x;  // (ic, t)
  const float *pa = a + row * 3 * nx, *pb = b + row * 3 * nx;
  for (int ch = 0; ch < 3; ++ch) {
    double acc = 0.0;
    for (int i = threadIdx.x; i < nx; i += kFvThreads) {
      const double d = (double)pa[ch * nx + i] - (double)pb[ch * nx + i];
      acc += d * d;
    }
    for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      double t = 0.0;
      for (int w = 0; w < kFvThreads / 64; ++w) t += s_part[w];
      mse[row * 3 + ch] = (float)(t / nx);
    }
    __syncthreads();
  }
}

}  // namespace

hipError_t launch_traj_mse(const float *a, const float *b, int B, int T1, int nx, float *mse, hipStream_t s) {
  const int64_t rows = (int64_t)B * T1;
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(traj_mse_kernel, dim3((unsigned)rows), dim3(kFvThreads), 0, s, a, b, nx, mse);
  return hipGetLastError();
}

hipError_t launch_fv_step(const float *in, int64_t ld_in, float *out, int64_t ld_out,
                          const float *face_flux, const double *pc, int B, int nx, float c,
                          float dt, float nu, float dx2, float *flux_out, int64_t ld_flux,
                          float *metrics, int64_t ld_metrics, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  const size_t lds = fv_lds_bytes(nx);
  if (face_flux)
    hipLaunchKernelGGL(fv_step_kernel<true>, dim3(B), dim3(kFvThreads), lds, s, in, ld_in, out,
                       ld_out, face_flux, pc, nx, c, dt, nu, dx2, flux_out, ld_flux, metrics,
                       ld_metrics);
  else
    hipLaunchKernelGGL(fv_step_kernel<false>, dim3(B), dim3(kFvThreads), lds, s, in, ld_in, out,
                       ld_out, face_flux, pc, nx, c, dt, nu, dx2, flux_out, ld_flux, metrics,
                       ld_metrics);
  return hipGetLastError();
}

hipError_t launch_state_metrics(const float *st, int64_t ld, int B, int nx, float *metrics,
                                int64_t ld_metrics, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(state_metrics_kernel, dim3(B), dim3(kFvThreads), 0, s, st, ld, nx, metrics,
                     ld_metrics);
  return hipGetLastError();
}

hipError_t launch_poisson(const float *n, int ld_n, float *E, int ld_E, const double *pc, int B,
                          int nx, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  const size_t lds = fv_lds_bytes(nx);
  hipLaunchKernelGGL(poisson_kernel, dim3(B), dim3(kFvThreads), lds, s, n, ld_n, E, ld_E, pc, nx);
  return hipGetLastError();
}

}  // namespace hf
