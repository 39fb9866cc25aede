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
#ifdef HF_DIAG_NOPOISSON  // timing diagnostic only: results are wrong
  return s_rho[i] * (float)s_c[i];
#endif
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
__device__ __forceinline__ double2 cmul(double2 a, double2 w) {
  return make_double2(a.x * w.x - a.y * w.y, a.x * w.y + a.y * w.x);
}
// exp(-+2 pi i m / n) for 0 <= m < n from the quarter table tw[m < n/4] (the
// plan holds m < n/2; only the first quarter is staged): quadrant q multiplies
// by (-i)^q, a swap and sign flips, so every twiddle is exactly the table's.
__device__ __forceinline__ double2 twiddle(const double2 *__restrict__ tw, int m, int n, bool inverse) {
  const int n4 = n / 4, q = m / n4;
  const double2 t = tw[m - q * n4];
  double2 w = q == 0 ? t : q == 1 ? make_double2(t.y, -t.x) : q == 2 ? make_double2(-t.x, -t.y)
                                                                    : make_double2(-t.y, t.x);
  if (inverse) w.y = -w.y;
  return w;
}

// Block FFT, Stockham autosort: radix-4 passes (one radix-2 pass first when
// log2 n is odd), one barrier per pass.  Returns the buffer holding the
// result (a or b).  tests/test_abi_cpu.py::_stockham models the same passes.
__device__ __forceinline__ double2 *fft_block(double2 *a, double2 *b, const double2 *__restrict__ tw, int n,
                                              bool inverse) {
  int ns = 1;
  if ((__builtin_ctz(n) & 1) != 0) {  // radix-2 pass, ns = 1: twiddle 1
    __syncthreads();
    for (int jj = threadIdx.x; jj < n / 2; jj += blockDim.x) {
      const double2 a0 = a[jj], a1 = a[jj + n / 2];
      b[2 * jj] = make_double2(a0.x + a1.x, a0.y + a1.y);
      b[2 * jj + 1] = make_double2(a0.x - a1.x, a0.y - a1.y);
    }
    double2 *s = a;
    a = b;
    b = s;
    ns = 2;
  }
  for (; ns < n; ns <<= 2) {
    __syncthreads();
    for (int jj = threadIdx.x; jj < n / 4; jj += blockDim.x) {
      const int k = jj & (ns - 1);
      const int m = k * (n / (4 * ns));
      const double2 a0 = a[jj];
      const double2 a1 = cmul(a[jj + n / 4], twiddle(tw, m, n, inverse));
      const double2 a2 = cmul(a[jj + n / 2], twiddle(tw, 2 * m, n, inverse));
      const double2 a3 = cmul(a[jj + 3 * n / 4], twiddle(tw, 3 * m, n, inverse));
      const double2 b0 = make_double2(a0.x + a2.x, a0.y + a2.y), b1 = make_double2(a0.x - a2.x, a0.y - a2.y);
      const double2 b2 = make_double2(a1.x + a3.x, a1.y + a3.y);
      const double2 t = make_double2(a1.x - a3.x, a1.y - a3.y);
      const double2 b3 = inverse ? make_double2(-t.y, t.x) : make_double2(t.y, -t.x);  // (a1 - a3) * (+-i)
      const int d = (jj - k) * 4 + k;
      b[d] = make_double2(b0.x + b2.x, b0.y + b2.y);
      b[d + ns] = make_double2(b1.x + b3.x, b1.y + b3.y);
      b[d + 2 * ns] = make_double2(b0.x - b2.x, b0.y - b2.y);
      b[d + 3 * ns] = make_double2(b1.x - b3.x, b1.y - b3.y);
    }
    double2 *s = a;
    a = b;
    b = s;
  }
  __syncthreads();
  return a;
}

// Spectral Poisson for the whole IC (block-wide).  On entry a[q] = (rho_q, 0),
// written before the call by any thread (fft_block opens with a barrier);
// s_tw holds the plan's twiddles (staged in LDS).  Returns the buffer X with
// E_q = X[q].x / nx (the caller rounds to float32).
__device__ __forceinline__ double2 *poisson_fft(double2 *a, double2 *b, const double2 *s_tw, const double *inv_k,
                                               int nx) {
  double2 *X = fft_block(a, b, s_tw, nx, false);
  double2 *Y = X == a ? b : a;
  for (int q = threadIdx.x; q < nx; q += blockDim.x) {
    const double ik = inv_k[q];                       // 1j * X / k, k = 0 mode zeroed
    X[q] = make_double2(-X[q].y * ik, X[q].x * ik);
  }
  return fft_block(X, Y, s_tw, nx, true);
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
