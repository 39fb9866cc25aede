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

// LDS, circulant nx: c[nx] (double) | u, F, rho, E (float).
// LDS, FFT nx: u, F (float) | FFT buffers 2 x nx double2 | twiddles nx/4 double2.
__host__ __device__ inline size_t fv_fft_offset(int nx) { return ((size_t)nx * 2 * sizeof(float) + 15) & ~size_t(15); }
inline size_t fv_lds_bytes(int nx) {
  return poisson_uses_fft(nx) ? fv_fft_offset(nx) + (2 * (size_t)nx + nx / 4) * sizeof(double2)
                              : (size_t)nx * (sizeof(double) + 4 * sizeof(float));
}

// Carve of the dynamic LDS (see fv_lds_bytes).
struct FvLds {
  double *c;
  float *u, *F, *rho, *E;
  double2 *fa, *fb, *tw;
  __device__ FvLds(double *s_dyn, int nx) {
    if (poisson_uses_fft(nx)) {
      c = nullptr;
      u = reinterpret_cast<float *>(s_dyn);
      F = u + nx;
      rho = E = nullptr;
      fa = reinterpret_cast<double2 *>(reinterpret_cast<char *>(s_dyn) + fv_fft_offset(nx));
      fb = fa + nx;
      tw = fb + nx;
    } else {
      c = s_dyn;
      u = reinterpret_cast<float *>(c + nx);
      F = u + nx;
      rho = F + nx;
      E = rho + nx;
      fa = fb = tw = nullptr;
    }
  }
};

// Stage the first quarter of the plan's twiddles (after the circulant column c[nx]) into LDS.
__device__ __forceinline__ void stage_twiddles(const double *pc, double2 *s_tw, int nx) {
  const double2 *tw = reinterpret_cast<const double2 *>(pc + nx);
  for (int q = threadIdx.x; q < nx / 4; q += blockDim.x) s_tw[q] = tw[q];
}

template <bool HYBRID>
__global__ __launch_bounds__(kFvThreads) void fv_step_kernel(
    const float *__restrict__ in, int64_t ld_in, float *__restrict__ out, int64_t ld_out,
    const float *__restrict__ face_flux, const double *__restrict__ pc, int nx, float c, float dt,
    float nu, float dx2, float *__restrict__ flux_out, int64_t ld_flux, float *__restrict__ metrics,
    int64_t ld_metrics) {
  extern __shared__ double s_dyn[];
  const FvLds L(s_dyn, nx);
  const bool fft = poisson_uses_fft(nx);
  const int64_t b = blockIdx.x;
  const float *st = in + b * ld_in;
  float *so = out + b * ld_out;
  for (int i = threadIdx.x; i < nx; i += kFvThreads) {
    const float u = st[nx + i];
    L.u[i] = u;
    L.F[i] = HYBRID ? face_flux[b * nx + i] : __fmul_rn(st[i], u);  // F_n = n*u (:70-71)
    if (!fft) L.c[i] = pc[i];
  }
  if (fft) stage_twiddles(pc, L.tw, nx);
  __syncthreads();
  for (int i = threadIdx.x; i < nx; i += kFvThreads) {
    const int im = i == 0 ? nx - 1 : i - 1;
    const int ip = i == nx - 1 ? 0 : i + 1;
    const float F = L.F[i];
    const float n_new = continuity(st[i], F, L.F[im], c);
    const float E = st[2 * nx + i];
    const float u_new = HYBRID ? velocity_hybrid(L.u[i], L.u[im], E, c, dt)
                               : velocity_classical(L.u[i], L.u[im], L.u[ip], E, c, dt, nu, dx2);
    const float rho = __fsub_rn(n_new, 1.0f);
    if (fft) L.fa[i] = make_double2((double)rho, 0.0);
    else L.rho[i] = rho;
    so[i] = n_new;
    so[nx + i] = u_new;
    if (flux_out) flux_out[b * ld_flux + i] = F;
  }
  const double2 *X = nullptr;
  if (fft) X = poisson_fft(L.fa, L.fb, L.tw, pc + 2 * nx, nx);
  else __syncthreads();
  MetricAcc m;
  m.init();
  for (int i = threadIdx.x; i < nx; i += kFvThreads) {
    const float E_new = fft ? (float)(X[i].x / nx) : poisson_cell(L.rho, L.c, i, nx);
    so[2 * nx + i] = E_new;
    if (metrics) m.add(so[i], so[nx + i], E_new);
  }
  if (metrics) block_metrics(m, metrics + b * ld_metrics, nx);
}

// FFT sizes: two ICs per workgroup share one complex transform pair.  The
// spectral operator T = i/k (k = 0 zeroed) maps the FFT of a real signal to
// the FFT of a real signal, so with z = rho_a + i rho_b,
//   ifft(T fft(z)) = ifft(T fft(rho_a)) + i ifft(T fft(rho_b)) = E_a + i E_b:
// the real part is IC a's field and the imaginary part IC b's, for half the
// transform work per IC (src/baseline_solver.py:59-68 evaluates each
// separately; the two agree to float64 rounding, far below the float32 result).
// Every global read is issued up front (one HBM round trip): n and E into
// registers, u and F (read at i-1, i+1) into LDS, where they share the second
// FFT buffer (first written by the transform, after its opening barrier).
// LDS: FFT buffer a [nx] double2 | buffer b [nx] double2 = u, F [2][nx] float |
// twiddles nx/4 double2: 36 KiB at nx = 1024, four workgroups per CU.
constexpr int kFvPer = kFftMaxNx / kFvThreads;  // cells per thread, at most
inline size_t fv_pair_lds_bytes(int nx) { return (2 * (size_t)nx + nx / 4) * sizeof(double2); }

template <bool HYBRID>
__global__ __launch_bounds__(kFvThreads) void fv_step_pair_kernel(
    const float *__restrict__ in, int64_t ld_in, float *__restrict__ out, int64_t ld_out,
    const float *__restrict__ face_flux, const double *__restrict__ pc, int nx, float c, float dt,
    float nu, float dx2, float *__restrict__ flux_out, int64_t ld_flux, float *__restrict__ metrics,
    int64_t ld_metrics, int B) {
  extern __shared__ double s_dyn[];
  double2 *fa = reinterpret_cast<double2 *>(s_dyn);
  double2 *fb = fa + nx, *tw = fb + nx;
  float *s_u = reinterpret_cast<float *>(fb);  // [2][nx], then [2][nx] F: the 16*nx bytes of fb
  float *s_F = s_u + 2 * nx;
  const int64_t b0 = 2 * (int64_t)blockIdx.x;
  const int nic = b0 + 1 < B ? 2 : 1;
  float n_r[2][kFvPer], E_r[2][kFvPer];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    if (q < nic) {
      const float *st = in + (b0 + q) * ld_in;
#pragma unroll
      for (int k = 0; k < kFvPer; ++k) {
        const int i = threadIdx.x + k * kFvThreads;
        if (i < nx) {
          const float n = st[i], u = st[nx + i];
          n_r[q][k] = n;
          E_r[q][k] = st[2 * nx + i];
          s_u[q * nx + i] = u;
          s_F[q * nx + i] = HYBRID ? face_flux[(b0 + q) * nx + i] : __fmul_rn(n, u);  // F_n = n*u (:70-71)
        }
      }
    }
  }
  stage_twiddles(pc, tw, nx);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kFvPer; ++k) {
    const int i = threadIdx.x + k * kFvThreads;
    if (i >= nx) break;
    const int im = i == 0 ? nx - 1 : i - 1;
    const int ip = i == nx - 1 ? 0 : i + 1;
    double rho[2] = {0.0, 0.0};
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (q >= nic) break;
      float *so = out + (b0 + q) * ld_out;
      const float *u = s_u + q * nx, *Fq = s_F + q * nx;
      const float F = Fq[i];
      const float n_new = continuity(n_r[q][k], F, Fq[im], c);
      const float E = E_r[q][k];
      const float u_new = HYBRID ? velocity_hybrid(u[i], u[im], E, c, dt)
                                 : velocity_classical(u[i], u[im], u[ip], E, c, dt, nu, dx2);
      rho[q] = (double)__fsub_rn(n_new, 1.0f);
      so[i] = n_new;
      so[nx + i] = u_new;
      if (flux_out) flux_out[(b0 + q) * ld_flux + i] = F;
    }
    fa[i] = make_double2(rho[0], rho[1]);
  }
  const double2 *X = poisson_fft(fa, fb, tw, pc + 2 * nx, nx);
  MetricAcc m[2];
  m[0].init();
  m[1].init();
  for (int i = threadIdx.x; i < nx; i += kFvThreads) {
    for (int q = 0; q < nic; ++q) {
      float *so = out + (b0 + q) * ld_out;
      const float E_new = (float)((q == 0 ? X[i].x : X[i].y) / nx);
      so[2 * nx + i] = E_new;
      if (metrics) m[q].add(so[i], so[nx + i], E_new);
    }
  }
  if (metrics) {
    block_metrics(m[0], metrics + b0 * ld_metrics, nx);
    if (nic == 2) {
      __syncthreads();  // block_metrics' shared partials are reused
      block_metrics(m[1], metrics + (b0 + 1) * ld_metrics, nx);
    }
  }
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
  const FvLds L(s_dyn, nx);
  const bool fft = poisson_uses_fft(nx);
  const int64_t b = blockIdx.x;
  for (int i = threadIdx.x; i < nx; i += kFvThreads) {
    const float rho = __fsub_rn(n[b * ld_n + i], 1.0f);  // rho = n - n0 (:60)
    if (fft) {
      L.fa[i] = make_double2((double)rho, 0.0);
    } else {
      L.c[i] = pc[i];
      L.rho[i] = rho;
    }
  }
  const double2 *X = nullptr;
  if (fft) {
    stage_twiddles(pc, L.tw, nx);
    X = poisson_fft(L.fa, L.fb, L.tw, pc + 2 * nx, nx);
  } else {
    __syncthreads();
  }
  for (int i = threadIdx.x; i < nx; i += kFvThreads)
    E[b * ld_E + i] = fft ? (float)(X[i].x / nx) : poisson_cell(L.rho, L.c, i, nx);
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
  if (poisson_uses_fft(nx)) {  // two ICs per workgroup, one transform pair
    const size_t lds = fv_pair_lds_bytes(nx);
    const unsigned grid = (unsigned)((B + 1) / 2);
    if (face_flux)
      hipLaunchKernelGGL(fv_step_pair_kernel<true>, dim3(grid), dim3(kFvThreads), lds, s, in, ld_in, out, ld_out,
                         face_flux, pc, nx, c, dt, nu, dx2, flux_out, ld_flux, metrics, ld_metrics, B);
    else
      hipLaunchKernelGGL(fv_step_pair_kernel<false>, dim3(grid), dim3(kFvThreads), lds, s, in, ld_in, out, ld_out,
                         face_flux, pc, nx, c, dt, nu, dx2, flux_out, ld_flux, metrics, ld_metrics, B);
    return hipGetLastError();
  }
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
