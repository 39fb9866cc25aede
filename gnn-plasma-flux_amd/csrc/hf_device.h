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

// tanh in f32 for the comparison models' one-launch rollouts (PureGNN, PINN):
// |x| < 0.55: x + x^3 P(x^2), a degree-4 fit of (tanh x - x) / x^3 (<= 0.8 ulp
// evaluated in f32); otherwise 1 - 2 / (1 + 2^(2|x|/ln 2)) on the hardware
// v_exp_f32 / v_rcp_f32 (<= 2 ulp with both correctly rounded, <= 4 with
// both one ulp off; tests/test_tanh_fast_cpu.py), sign restored.  About 15 VALU against the
// device libm tanhf's 22 (with its exact division); NaN propagates.
__device__ __forceinline__ float tanh_fast(float x) {
  const float ax = __builtin_fabsf(x);
  const float e = __builtin_amdgcn_exp2f(ax * 2.88539008177792681f);
  const float big = __builtin_fmaf(-2.0f, __builtin_amdgcn_rcpf(1.0f + e), 1.0f);
  const float x2 = x * x;
  float p = -0.006287517491728067f;
  p = __builtin_fmaf(p, x2, 0.02108195051550865f);
  p = __builtin_fmaf(p, x2, -0.05385509133338928f);
  p = __builtin_fmaf(p, x2, 0.13332617282867432f);
  p = __builtin_fmaf(p, x2, -0.33333319425582886f);
  const float small = __builtin_fmaf(x * x2, p, x);
  return ax < 0.55f ? small : __builtin_copysignf(big, x);
}
// tanh_fast of two values, bit-identical to two tanh_fast calls: the same f32
// operations in the same order, the multiplies / adds / fmas as packed f32
// (v_pk_mul_f32, v_pk_add_f32, v_pk_fma_f32), exp and rcp per element.
typedef float hf_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ hf_f2 tanh_fast2(hf_f2 x) {
  const hf_f2 ax = __builtin_elementwise_abs(x);
  const hf_f2 t = ax * 2.88539008177792681f;
  const hf_f2 e = hf_f2{__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y)};
  const hf_f2 d = 1.0f + e;
  const hf_f2 r = hf_f2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  const hf_f2 big = __builtin_elementwise_fma(hf_f2(-2.0f), r, hf_f2(1.0f));
  const hf_f2 x2 = x * x;
  hf_f2 p = hf_f2(-0.006287517491728067f);
  p = __builtin_elementwise_fma(p, x2, hf_f2(0.02108195051550865f));
  p = __builtin_elementwise_fma(p, x2, hf_f2(-0.05385509133338928f));
  p = __builtin_elementwise_fma(p, x2, hf_f2(0.13332617282867432f));
  p = __builtin_elementwise_fma(p, x2, hf_f2(-0.33333319425582886f));
  const hf_f2 small = __builtin_elementwise_fma(x * x2, p, x);
  return hf_f2{ax.x < 0.55f ? small.x : __builtin_copysignf(big.x, x.x),
               ax.y < 0.55f ? small.y : __builtin_copysignf(big.y, x.y)};
}

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

// poisson_cell for a compile-time even NX (the fused rollouts), term for term
// and chain for chain the same sums: rho is held as double (the same value as
// the (double) conversion above) and the column twice, s_c2[m] = c[m mod NX]
// for m < 2 NX, so term j reads s_c2[i + NX - j] at a constant offset from one
// per-lane base and every LDS read is an immediate-offset ds_read with no index
// arithmetic; unrolled, the reads run ahead of the two fp64 FMA chains instead
// of one wrap-around index update and two dependent reads per term.
template <int NX>
__device__ __forceinline__ float poisson_cell_nx(const double *s_rho, const double *s_c2, int i) {
  static_assert(NX % 2 == 0, "even chain length");
#ifdef HF_DIAG_NOPOISSON  // timing diagnostic only: results are wrong
  return (float)(s_rho[i] * s_c2[i]);
#endif
  const double *cb = s_c2 + i + 1;  // term j at cb[NX - 1 - j]
  double a0 = 0.0, a1 = 0.0;
#pragma unroll
  for (int j = 0; j < NX; j += 2) {
    a0 = fma(cb[NX - 1 - j], s_rho[j], a0);
    a1 = fma(cb[NX - 2 - j], s_rho[j + 1], a1);
  }
  return (float)(a0 + a1);
}

// ------------------------------------------ tridiagonal Poisson (opt-in mode)
// HF_POISSON_TRIDIAG (include/hybridflux.h) is NOT the reference's operator:
// the reference solves spectrally (src/baseline_solver.py:59-68, the default
// here and the only parity mode).  It is the north star's cyclic-reduction
// tridiagonal solve of the same equation, dE/dx = -(rho - mean rho), in the
// second-order potential form on the periodic grid:
//   (phi[i-1] - 2 phi[i] + phi[i+1]) / dx^2 = rho[i] - mean(rho),
//   E[i] = -(phi[i+1] - phi[i-1]) / (2 dx).
// Its Fourier symbol E_k = i (dx/2) cot(k dx/2) rho_k tends to the spectral
// i rho_k / k as k dx -> 0 (0.02 relative at the k = 5 modes of the ICs at
// nx = 64, ~1e-3 absolute in E).  With the unit right-hand side
// d = rho - mean and phi = dx^2 psi:  E[i] = h (psi[i-1] - psi[i+1]), h = dx/2
// (the whole plan of this mode, hf_poisson_plan).  The periodic system is
// singular (constants) and E does not depend on the gauge, so psi[0] = 0 and
// equation 0 is dropped: a Dirichlet tridiagonal system for psi[1..n-1].
//
// Cyclic reduction by one wave on a wave-private LDS row (T = double, or
// double2 for a pair of ICs solved together): while the survivors (stride s)
// are even in number, eliminate every other one,
//   d[i] <- d[i-s] + 2 d[i] + d[i+s]          (i = 0 mod 2s; the coefficients
// of the reduced system stay (1, -2, 1) at stride 2s); the R = n/s survivors
// left (R odd, 1 for power-of-two n) are solved by lane 0 with psi[0] = 0 by
// the Thomas recurrence of (1, -2, 1), whose pivots are -(j+1)/j in closed
// form; then back-substitution level by level,
//   psi[i] = ((psi[i-s] + psi[i+s]) - d[i]) / 2   (i = s mod 2s).
// Float64 throughout.  Only the wave's own s_waitcnt orders the LDS levels (a
// wave's LDS operations complete in order): no workgroup barrier.
__device__ __forceinline__ void wave_lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ double tri_zero(double) { return 0.0; }
__device__ __forceinline__ double2 tri_zero(double2) { return make_double2(0.0, 0.0); }
__device__ __forceinline__ double tri_add(double a, double b) { return a + b; }
__device__ __forceinline__ double2 tri_add(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double tri_sub(double a, double b) { return a - b; }
__device__ __forceinline__ double2 tri_sub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double tri_scale(double a, double k) { return a * k; }
__device__ __forceinline__ double2 tri_scale(double2 a, double k) { return make_double2(a.x * k, a.y * k); }
__device__ __forceinline__ double tri_wave_sum(double a) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) a += __shfl_xor(a, o, 64);
  return a;
}
__device__ __forceinline__ double2 tri_wave_sum(double2 a) { return make_double2(tri_wave_sum(a.x), tri_wave_sum(a.y)); }

// On entry x[0..n) = rho (any offset: the mean is removed here); on exit
// x = psi with psi[0] = 0.  All 64 lanes of the wave call it (wave-uniform n).
template <class T>
__device__ void tridiag_psi_wave(T *x, int n, int lane) {
  T acc = tri_zero(T());
  for (int i = lane; i < n; i += 64) acc = tri_add(acc, x[i]);
  const T mean = tri_scale(tri_wave_sum(acc), 1.0 / (double)n);
  for (int i = lane; i < n; i += 64) x[i] = tri_sub(x[i], mean);
  wave_lds_fence();
  int s = 1;
  for (; n % (2 * s) == 0; s *= 2) {  // forward reduction: survivors i = 2 s k
    for (int k = lane; k < n / (2 * s); k += 64) {
      const int i = 2 * s * k;
      const T l = x[i == 0 ? n - s : i - s], r = x[i + s];
      x[i] = tri_add(tri_add(l, r), tri_scale(x[i], 2.0));
    }
    wave_lds_fence();
  }
  if (lane == 0) {  // the R = n / s (odd) survivors j s, psi[0] = psi[R s] = 0
    const int R = n / s;
    T dp = tri_zero(T());
    for (int j = 1; j < R; ++j) {
      dp = tri_scale(tri_sub(x[j * s], dp), -(double)j / (double)(j + 1));
      x[j * s] = dp;
    }
    T p = tri_zero(T());
    for (int j = R - 1; j >= 1; --j) {
      p = tri_add(x[j * s], tri_scale(p, (double)j / (double)(j + 1)));
      x[j * s] = p;
    }
    x[0] = tri_zero(T());
  }
  wave_lds_fence();
  for (s /= 2; s >= 1; s /= 2) {  // back-substitution: i = s + 2 s k
    for (int k = lane; k < n / (2 * s); k += 64) {
      const int i = s + 2 * s * k;
      const T l = x[i - s], r = x[i + s == n ? 0 : i + s];
      x[i] = tri_scale(tri_sub(tri_add(l, r), x[i]), 0.5);
    }
    wave_lds_fence();
  }
}

// E at cell i from psi (tridiag_psi_wave): h (psi[i-1] - psi[i+1]), h = dx/2
__device__ __forceinline__ double tri_E(const double *psi, int i, int n, double h) {
  return h * (psi[i == 0 ? n - 1 : i - 1] - psi[i == n - 1 ? 0 : i + 1]);
}
__device__ __forceinline__ double2 tri_E(const double2 *psi, int i, int n, double h) {
  const double2 l = psi[i == 0 ? n - 1 : i - 1], r = psi[i == n - 1 ? 0 : i + 1];
  return make_double2(h * (l.x - r.x), h * (l.y - r.y));
}

// ---------------------------------------------------------------- FFT Poisson
// For power-of-two nx in [kFftMinNx, kFftMaxNx] the spectral operator is
// applied as the reference writes it (src/baseline_solver.py:59-68),
// E = Re(ifft(1j*fft(rho)/k)), k=0 mode zeroed, by float64 FFTs run by ONE
// wave: lane l holds the N/64 values at indices l + 64v in registers, the
// transform is a mixed-radix Stockham sequence (radix R = min(N/64, 16,
// what is left): 256 = 4^4, 512 = 8^3, 1024 = 16*16*4, 2048 = 16*16*8) whose
// butterflies a lane evaluates in registers, and the passes exchange values
// through a wave-private LDS buffer (the wave's own s_waitcnt orders it: no
// workgroup barrier).  The first pass reads, and the last pass writes, the
// lane's own indices l + 64v, so the FV update feeds the transform and takes
// E back without LDS.  Twiddles exp(-+2 pi i e/N) come from the plan
// (hf_poisson_coeffs: e < N/2 as (re, im); e >= N/2 by negation), so each is
// exactly the plan's value.  tests/test_abi_cpu.py::_stockham models the same
// passes in numpy.
// float64 complex product as 2 multiplies + 2 FMAs (this header turns
// contraction off for the float32 FV expressions; the transforms round at
// 1e-16 and do not need it)
__device__ __forceinline__ double2 cmul(double2 a, double2 w) {
  return make_double2(fma(a.x, w.x, -(a.y * w.y)), fma(a.x, w.y, a.y * w.x));
}
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }

// exp(-+2 pi i e / N) for 0 <= e < N from the plan's half table
template <int N, bool INV>
__device__ __forceinline__ double2 plan_twiddle(const double2 *__restrict__ tw, int e) {
  const bool hi = e >= N / 2;
  double2 w = tw[hi ? e - N / 2 : e];
  if (hi) w = make_double2(-w.x, -w.y);
  if (INV) w.y = -w.y;
  return w;
}

// t * exp(-+2 pi i q / 16) with the constant's exact special cases (q % 4 == 0)
template <int Q, bool INV>
__device__ __forceinline__ double2 mul_w16(double2 t) {
  constexpr double kC[16] = {1.0, 0.92387953251128675613, 0.70710678118654752440, 0.38268343236508977173,
                             0.0, -0.38268343236508977173, -0.70710678118654752440, -0.92387953251128675613,
                             -1.0, -0.92387953251128675613, -0.70710678118654752440, -0.38268343236508977173,
                             0.0, 0.38268343236508977173, 0.70710678118654752440, 0.92387953251128675613};
  constexpr int q = Q & 15;
  if constexpr (q == 0) return t;
  else if constexpr (q == 8) return make_double2(-t.x, -t.y);
  else if constexpr (q == 4) return INV ? make_double2(-t.y, t.x) : make_double2(t.y, -t.x);   // * (+-i)
  else if constexpr (q == 12) return INV ? make_double2(t.y, -t.x) : make_double2(-t.y, t.x);
  else {
    constexpr double c = kC[q], sn = kC[(q + 12) & 15];  // sin(2 pi q/16) = cos(2 pi (q - 4)/16)
    const double si = INV ? sn : -sn;
    return make_double2(fma(t.x, c, -(t.y * si)), fma(t.x, si, t.y * c));
  }
}

// Butterfly combine of a radix-2 DIT step: y_s = e_s + W_R^s o_s,
// y_{s+R/2} = e_s - W_R^s o_s for s = S..R/2-1 (W_R^s as a constant).
template <int R, bool INV, int S = 0>
__device__ __forceinline__ void dit_combine(const double2 (&e)[R / 2], const double2 (&o)[R / 2], double2 (&y)[R]) {
  if constexpr (S < R / 2) {
    const double2 t = mul_w16<S * (16 / R), INV>(o[S]);
    y[S] = cadd(e[S], t);
    y[S + R / 2] = csub(e[S], t);
    dit_combine<R, INV, S + 1>(e, o, y);
  }
}

// In-register DFT of size R (1..16): y_s = sum_r y_r exp(-+2 pi i r s / R),
// radix-2 decimation in time.
template <int R, bool INV>
__device__ __forceinline__ void dft_reg(double2 (&y)[R]) {
  if constexpr (R > 1) {
    double2 e[R / 2], o[R / 2];
#pragma unroll
    for (int i = 0; i < R / 2; ++i) {
      e[i] = y[2 * i];
      o[i] = y[2 * i + 1];
    }
    dft_reg<R / 2, INV>(e);
    dft_reg<R / 2, INV>(o);
    dit_combine<R, INV>(e, o, y);
  }
}

// Padded wave-private LDS index: one double2 of padding per 16 keeps the
// strided butterfly writes off a single bank group.
__device__ __forceinline__ int fft_pad(int idx) { return idx + (idx >> 4); }
template <int N>
constexpr int fft_lds_elems() { return N + N / 16; }

// Stockham passes NS.. of an N-point transform.  v[t + r*(V/R)] holds index
// lane + 64t + r*N/R; the first pass (NS == 1) reads v, the last writes it.
#ifndef HF_FFT_MAX_RADIX
#define HF_FFT_MAX_RADIX 16
#endif
constexpr int kFftMaxRadix = HF_FFT_MAX_RADIX;
template <int N, int NS, bool INV>
__device__ __forceinline__ void fft_passes(double2 (&v)[N / 64], double2 *lds, const double2 *__restrict__ tw,
                                           int lane) {
  constexpr int V = N / 64;
  constexpr int RV = V < kFftMaxRadix ? V : kFftMaxRadix;
  constexpr int R = RV < N / NS ? RV : N / NS;
  constexpr int B = V / R;  // butterflies per lane
  constexpr bool kLast = NS * R == N;
  // the pass's inputs: the registers (first pass) or the previous pass's LDS output
  if constexpr (NS > 1) {
#pragma unroll
    for (int t = 0; t < B; ++t)
#pragma unroll
      for (int r = 0; r < R; ++r) v[t + r * B] = lds[fft_pad(lane + 64 * t + r * (N / R))];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every lane's reads before any write
  }
  double2 (&x)[V] = v;
#pragma unroll
  for (int t = 0; t < B; ++t) {
    const int j = lane + 64 * t;
    const int k = j & (NS - 1);
    const int m = k * (N / (R * NS));
    double2 y[R];
#pragma unroll
    for (int r = 0; r < R; ++r) y[r] = (NS == 1 || r == 0) ? x[t + r * B] : cmul(x[t + r * B], plan_twiddle<N, INV>(tw, r * m));
    dft_reg<R, INV>(y);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if constexpr (kLast) v[t + r * B] = y[r];                    // index j + r*NS = lane + 64(t + rB)
      else lds[fft_pad((j - k) * R + k + r * NS)] = y[r];
    }
  }
  if constexpr (!kLast) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    fft_passes<N, NS * R, INV>(v, lds, tw, lane);
  }
}

// Spectral Poisson of one wave's N-cell chain pair: on entry v[i] = (rho_a,
// rho_b) at cell lane + 64i; on exit v[i] = N * (E_a, E_b) there.  The operator
// i/k maps the FFT of a real signal to the FFT of a real signal, so the real
// and imaginary parts of the packed transform are the two fields.  plan =
// hf_poisson_coeffs (twiddles at plan + N, 1/k at plan + 2N).
// poisson_wave_tw takes the plan's twiddles and 1/k wherever they are staged
// (global memory, or an LDS copy in fv_run_fft_kernel).
template <int N>
__device__ __forceinline__ void poisson_wave_tw(double2 (&v)[N / 64], double2 *lds, const double2 *__restrict__ tw,
                                                const double *__restrict__ inv_k, int lane) {
#ifndef HF_DIAG_NOFFT  // timing diagnostic only: results are wrong (no transforms)
  fft_passes<N, 1, false>(v, lds, tw, lane);
#endif
#pragma unroll
  for (int i = 0; i < N / 64; ++i) {
    const double ik = inv_k[lane + 64 * i];  // 1j * X / k, k = 0 mode zeroed
    v[i] = make_double2(-v[i].y * ik, v[i].x * ik);
  }
#ifndef HF_DIAG_NOFFT
  fft_passes<N, 1, true>(v, lds, tw, lane);
#endif
}
template <int N>
__device__ __forceinline__ void poisson_wave(double2 (&v)[N / 64], double2 *lds, const double *__restrict__ plan,
                                             int lane) {
  poisson_wave_tw<N>(v, lds, reinterpret_cast<const double2 *>(plan + N), plan + 2 * N, lane);
}

// Per-state rollout metrics, partial sums for one cell.
// The finite flag is not tested per value: every value a lane adds is finite
// exactly when its double sums are (a finite float term is bounded, |n| <
// 2^128 and u^2 + E^2 < 2^257, so no nx overflows them; a NaN or +-Inf value
// makes its sum NaN or +-Inf, and +Inf + -Inf is NaN), so settle() derives it
// from the sums before they are combined.  Same flag, bit for bit, as a
// per-value isfinite test, without its compare and select per value.
struct MetricAcc {
  double energy;  // sum u^2 + E^2
  double charge;  // sum n
  float maxdev;   // max |n - 1|
  int finite;     // 1 while every value is finite (settled from the sums)
  __device__ void init() { energy = 0; charge = 0; maxdev = 0.f; finite = 1; }
  __device__ void add(float n, float u, float E) {
    energy += (double)u * u + (double)E * E;
    charge += n;
    float dv = fabsf(n - 1.0f);
    maxdev = dv > maxdev ? dv : maxdev;
  }
  // the same sums split in two: n, u when the update produces them, E after the solve
  __device__ void add_nu(float n, float u) {
    energy += (double)u * u;
    charge += n;
    float dv = fabsf(n - 1.0f);
    maxdev = dv > maxdev ? dv : maxdev;
  }
  __device__ void add_E(float E) { energy += (double)E * E; }
  __device__ void settle() { finite &= (isfinite(energy) && isfinite(charge)) ? 1 : 0; }
  __device__ void wave_reduce() {
    settle();
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
    const bool fin = finite && isfinite(energy) && isfinite(charge);
    dst[0] = (float)(0.5 * energy / nx);
    dst[1] = (float)(charge / nx);
    dst[2] = fin ? 1.f : 0.f;
    dst[3] = fin ? maxdev : __int_as_float(0x7fc00000);
  }
};

}  // namespace hf
