// Device helpers shared by the chain and finite-volume kernels.
//
// The elementwise finite-volume arithmetic reproduces the reference's numpy
// float32 expressions operation by operation; every op is an explicitly
// rounded __f*_rn intrinsic so no FMA contraction can change a result
// (src/hybrid_solver.py:45-58, src/baseline_solver.py:70-94).
#pragma once

// HIP's __f*_rn helpers are plain operators unless OCML_BASIC_ROUNDED_OPERATIONS
// is set, and hipcc contracts a*b+c into FMA by default: turn contraction off
// for every TU that includes this header (explicit fmaf / MFMA are unaffected).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace hf {

// torch.relu semantics: NaN propagates (v_max_f32 would turn NaN into 0 and
// hide a blow-up from the finiteness metric).  IEEE-754-2019 maximum lowers to
// one gfx950 v_maximum3_f32, which propagates NaN.
__device__ __forceinline__ float relu(float x) { return __builtin_elementwise_maximum(x, 0.0f); }

// F = f32(0.5 * f32(F_fwd + F_bwd))                 src/hybrid_solver.py:45-48
__device__ __forceinline__ float face_flux(float ffwd, float fbwd) {
  return __fmul_rn(0.5f, __fadd_rn(ffwd, fbwd));
}

// n' = n - c*(F - F_left)                           src/hybrid_solver.py:51-52
__device__ __forceinline__ float continuity(float n, float F, float Fl, float c) {
  return __fsub_rn(n, __fmul_rn(c, __fsub_rn(F, Fl)));
}

// 0.5*u*u evaluated left to right in float32        src/hybrid_solver.py:55
__device__ __forceinline__ float burgers_flux(float u) { return __fmul_rn(__fmul_rn(0.5f, u), u); }

// u' = (u - c*(Fu - Fu_left)) + dt*E                src/hybrid_solver.py:55-58
__device__ __forceinline__ float velocity_hybrid(float u, float ul, float E, float c, float dt) {
  float adv = __fsub_rn(u, __fmul_rn(c, __fsub_rn(burgers_flux(u), burgers_flux(ul))));
  return __fadd_rn(adv, __fmul_rn(dt, E));
}

// u' = (u - c*(Fu-Fu_l)) + dt*(E + nu*((u_r - 2u) + u_l)/dx2)   src/baseline_solver.py:89-94
__device__ __forceinline__ float velocity_classical(float u, float ul, float ur, float E, float c,
                                                   float dt, float nu, float dx2) {
  float adv = __fsub_rn(u, __fmul_rn(c, __fsub_rn(burgers_flux(u), burgers_flux(ul))));
  float lap = __fdiv_rn(__fadd_rn(__fsub_rn(ur, __fmul_rn(2.f, u)), ul), dx2);
  return __fadd_rn(adv, __fmul_rn(dt, __fadd_rn(E, __fmul_rn(nu, lap))));
}

// Circulant spectral Poisson for one cell: E[i] = f32(sum_j c[(i-j) mod nx] * rho[j]),
// accumulated in float64 (src/baseline_solver.py:59-68; see hf_poisson_coeffs).
__device__ __forceinline__ float poisson_cell(const float *s_rho, const double *s_c, int i, int nx) {
  double a0 = 0.0, a1 = 0.0;
  int d = i;  // (i - j) mod nx, walking j upward
  int j = 0;
  for (; j + 1 < nx; j += 2) {
    a0 = fma(s_c[d], (double)s_rho[j], a0);
    d = d == 0 ? nx - 1 : d - 1;
    a1 = fma(s_c[d], (double)s_rho[j + 1], a1);
    d = d == 0 ? nx - 1 : d - 1;
  }
  if (j < nx) a0 = fma(s_c[d], (double)s_rho[j], a0);
  return (float)(a0 + a1);
}

// ---------------------------------------------------------------- FFT Poisson
// For power-of-two nx >= kFftMinNx the spectral operator is applied as the
// reference writes it (src/baseline_solver.py:59-68), E = Re(ifft(1j*fft(rho)/k)),
// with a float64 Stockham radix-2 FFT in LDS instead of the O(nx^2) circulant.
// The plan buffer (hf_poisson_coeffs) then holds, after the circulant column
// c[nx]: twiddles exp(-2 pi i m / nx) for m < nx/2 as (re, im), and 1/k_q (0 at q = 0).
// In-place-style block FFT: returns the buffer holding the result (a or b).
__device__ __forceinline__ double2 *fft_block(double2 *a, double2 *b, const double2 *__restrict__ tw, int n,
                                              bool inverse) {
  for (int ns = 1; ns < n; ns <<= 1) {
    __syncthreads();
    for (int jj = threadIdx.x; jj < n / 2; jj += blockDim.x) {
      const double2 a0 = a[jj], a1 = a[jj + n / 2];
      const int k = jj & (ns - 1);
      double2 w = tw[k * (n / (2 * ns))];
      if (inverse) w.y = -w.y;
      const double2 t = make_double2(a1.x * w.x - a1.y * w.y, a1.x * w.y + a1.y * w.x);
      const int d = ((jj - k) << 1) + k;
      b[d] = make_double2(a0.x + t.x, a0.y + t.y);
      b[d + ns] = make_double2(a0.x - t.x, a0.y - t.y);
    }
    double2 *s = a;
    a = b;
    b = s;
  }
  __syncthreads();
  return a;
}

// E[q] for the whole IC (block-wide): rho (LDS floats) -> out (LDS floats).
__device__ __forceinline__ void poisson_fft(const float *s_rho, double2 *a, double2 *b, const double *plan, int nx,
                                           float *out) {
  const double2 *tw = reinterpret_cast<const double2 *>(plan + nx);
  const double *inv_k = plan + 2 * nx;
  for (int q = threadIdx.x; q < nx; q += blockDim.x) a[q] = make_double2((double)s_rho[q], 0.0);
  double2 *X = fft_block(a, b, tw, nx, false);
  double2 *Y = X == a ? b : a;
  for (int q = threadIdx.x; q < nx; q += blockDim.x) {
    const double ik = inv_k[q];                       // 1j * X / k, k = 0 mode zeroed
    X[q] = make_double2(-X[q].y * ik, X[q].x * ik);
  }
  X = fft_block(X, Y, tw, nx, true);
  for (int q = threadIdx.x; q < nx; q += blockDim.x) out[q] = (float)(X[q].x / nx);
  __syncthreads();
}

// Per-state rollout metrics, partial sums for one cell.
struct MetricAcc {
  double energy;  // sum u^2 + E^2
  double charge;  // sum n
  float maxdev;   // max |n - 1|
  int finite;     // 1 while every value is finite
  __device__ void init() { energy = 0; charge = 0; maxdev = 0.f; finite = 1; }
  __device__ void add(float n, float u, float E) {
    energy += (double)u * u + (double)E * E;
    charge += n;
    float dv = fabsf(n - 1.0f);
    maxdev = dv > maxdev ? dv : maxdev;
    finite &= (isfinite(n) && isfinite(u) && isfinite(E)) ? 1 : 0;
  }
  __device__ void wave_reduce() {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      energy += __shfl_xor(energy, o, 64);
      charge += __shfl_xor(charge, o, 64);
      float m = __shfl_xor(maxdev, o, 64);
      maxdev = m > maxdev ? m : maxdev;
      finite &= __shfl_xor(finite, o, 64);
    }
  }
  __device__ void store(float *dst, int nx) const {
    dst[0] = (float)(0.5 * energy / nx);
    dst[1] = (float)(charge / nx);
    dst[2] = finite ? 1.f : 0.f;
    dst[3] = finite ? maxdev : __int_as_float(0x7fc00000);
  }
};

}  // namespace hf
