// Finite-volume update + spectral Poisson solve for any nx
// (src/baseline_solver.py:59-101, src/hybrid_solver.py:45-63).
//
// FFT sizes (power-of-two nx in 256..2048): one wave per pair of ICs, the
// transform in registers + a wave-private LDS buffer (hf_device.h
// poisson_wave).  Other nx: one 256-thread workgroup per IC, the chain in
// LDS and the exact O(nx^2) float64 circulant.  HBM traffic per cell-step is
// the 12 B state read + 12 B state write (+4 B face flux in hybrid mode).
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

// LDS of the circulant kernels (nx not an FFT size): c[nx] (double) | u, F, rho, E (float).
inline size_t fv_lds_bytes(int nx) { return (size_t)nx * (sizeof(double) + 4 * sizeof(float)); }

struct FvLds {
  double *c;
  float *u, *F, *rho, *E;
  __device__ FvLds(double *s_dyn, int nx) {
    c = s_dyn;
    u = reinterpret_cast<float *>(c + nx);
    F = u + nx;
    rho = F + nx;
    E = rho + nx;
  }
};

// Circulant nx (any nx that is not an FFT size): one 256-thread workgroup per IC.
// tri (HF_POISSON_TRIDIAG, wave-uniform): the c row holds rho, then psi, and
// wave 0 runs the cyclic reduction (hf_device.h tridiag_psi_wave); pc[0] = h.
template <bool HYBRID>
__global__ __launch_bounds__(kFvThreads) void fv_step_kernel(
    const float *__restrict__ in, int64_t ld_in, float *__restrict__ out, int64_t ld_out,
    const float *__restrict__ face_flux, const double *__restrict__ pc, int nx, float c, float dt,
    float nu, float dx2, float *__restrict__ flux_out, int64_t ld_flux, float *__restrict__ metrics,
    int64_t ld_metrics, int tri) {
  extern __shared__ double s_dyn[];
  const FvLds L(s_dyn, nx);
  const int64_t b = blockIdx.x;
  const float *st = in + b * ld_in;
  float *so = out + b * ld_out;
  for (int i = threadIdx.x; i < nx; i += kFvThreads) {
    const float u = st[nx + i];
    L.u[i] = u;
    L.F[i] = HYBRID ? face_flux[b * nx + i] : __fmul_rn(st[i], u);  // F_n = n*u (:70-71)
    if (!tri) L.c[i] = pc[i];
  }
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
    if (tri) L.c[i] = (double)rho;
    else L.rho[i] = rho;
    so[i] = n_new;
    so[nx + i] = u_new;
    if (flux_out) flux_out[b * ld_flux + i] = F;
  }
  __syncthreads();
  if (tri) {
    if (threadIdx.x < 64) tridiag_psi_wave<double>(L.c, nx, threadIdx.x);
    __syncthreads();
  }
  const double h = tri ? pc[0] : 0.0;
  MetricAcc m;
  m.init();
  for (int i = threadIdx.x; i < nx; i += kFvThreads) {
    const float E_new = tri ? (float)tri_E(L.c, i, nx, h) : poisson_cell(L.rho, L.c, i, nx);
    so[2 * nx + i] = E_new;
    if (metrics) m.add(so[i], so[nx + i], E_new);
  }
  if (metrics) block_metrics(m, metrics + b * ld_metrics, nx);
}

// ------------------------------------------------------------ large nx
// nx > kFvLdsMaxNx (the chain no longer fits the LDS plan above): the update
// and the Poisson solve run as separate launches over global memory, a
// 256-cell block per workgroup (grid: ICs x cell blocks).  The Poisson sum
// walks j in the order poisson_cell does, the even terms into a0 and the odd
// ones into a1, with rho and the window of c a tile needs staged in LDS, so
// E is the LDS kernels' value bit for bit; the metrics come from
// state_metrics_kernel, which sums in fv_step_kernel's order.
constexpr int kFvLdsMaxNx = 6144;  // fv_lds_bytes(6144) = 144 KiB of dynamic LDS
constexpr int kPoissonTileJ = 1024;

template <bool HYBRID>
__global__ __launch_bounds__(kFvThreads) void fv_update_kernel(const float *__restrict__ in, int64_t ld_in,
                                                               float *__restrict__ out, int64_t ld_out,
                                                               const float *__restrict__ face_flux, int nx, float c,
                                                               float dt, float nu, float dx2,
                                                               float *__restrict__ flux_out, int64_t ld_flux) {
  const int64_t b = blockIdx.x;
  const int i = blockIdx.y * kFvThreads + threadIdx.x;
  if (i >= nx) return;
  const float *st = in + b * ld_in;
  float *so = out + b * ld_out;
  const int im = i == 0 ? nx - 1 : i - 1;
  const int ip = i == nx - 1 ? 0 : i + 1;
  const float u = st[nx + i], um = st[nx + im];
  const float F = HYBRID ? face_flux[b * nx + i] : __fmul_rn(st[i], u);  // F_n = n*u (:70-71)
  const float Fm = HYBRID ? face_flux[b * nx + im] : __fmul_rn(st[im], um);
  const float E = st[2 * nx + i];
  so[i] = continuity(st[i], F, Fm, c);
  so[nx + i] = HYBRID ? velocity_hybrid(u, um, E, c, dt)
                      : velocity_classical(u, um, st[nx + ip], E, c, dt, nu, dx2);
  if (flux_out) flux_out[b * ld_flux + i] = F;
}

// E[i] = f32(sum_j c[(i-j) mod nx] (n_j - 1)) for the block's 256 cells.
__global__ __launch_bounds__(kFvThreads) void poisson_tiled_kernel(const float *__restrict__ n, int64_t ld_n,
                                                                   float *__restrict__ E, int64_t ld_E,
                                                                   const double *__restrict__ pc, int nx) {
  __shared__ float s_rho[kPoissonTileJ];
  __shared__ double s_c[kPoissonTileJ + kFvThreads];
  const int64_t b = blockIdx.x;
  const int i0 = blockIdx.y * kFvThreads, i = i0 + threadIdx.x;
  double a0 = 0.0, a1 = 0.0;
  for (int j0 = 0; j0 < nx; j0 += kPoissonTileJ) {
    const int T = nx - j0 < kPoissonTileJ ? nx - j0 : kPoissonTileJ;
    __syncthreads();  // the previous tile is consumed
    for (int k = threadIdx.x; k < T; k += kFvThreads) s_rho[k] = __fsub_rn(n[b * ld_n + j0 + k], 1.0f);
    // s_c[m] = c[(i0 - j0 - (T-1) + m) mod nx]: term (i, j0 + k) reads m = (i - i0) + T-1 - k
    const int base = i0 - j0 - (T - 1);
    for (int m = threadIdx.x; m < T + kFvThreads - 1; m += kFvThreads) {
      int d = (base + m) % nx;
      s_c[m] = pc[d < 0 ? d + nx : d];
    }
    __syncthreads();
    if (i < nx) {
      const double *cc = s_c + threadIdx.x + T - 1;  // cc[-k] = c[(i - j0 - k) mod nx]
      int k = 0;
      for (; k + 1 < T; k += 2) {  // j0 is even: k's parity is j's
        a0 = fma(cc[-k], (double)s_rho[k], a0);
        a1 = fma(cc[-k - 1], (double)s_rho[k + 1], a1);
      }
      if (k < T) a0 = fma(cc[-k], (double)s_rho[k], a0);  // odd nx: the last j is even
    }
  }
  if (i < nx) E[b * ld_E + i] = (float)(a0 + a1);
}

// Tridiagonal (HF_POISSON_TRIDIAG) E for one IC per 256-thread workgroup, any
// nx <= kTriMaxNx: rho staged as float64 in dynamic LDS, cyclic reduction by
// wave 0 (tridiag_psi_wave), E by every thread.  hf_poisson in this mode and the
// large-nx step (after fv_update_kernel).  pc[0] = h = dx/2.
__global__ __launch_bounds__(kFvThreads) void poisson_tri_kernel(const float *__restrict__ n, int64_t ld_n,
                                                                 float *__restrict__ E, int64_t ld_E,
                                                                 const double *__restrict__ pc, int nx) {
  extern __shared__ double s_dyn[];
  const int64_t b = blockIdx.x;
  for (int i = threadIdx.x; i < nx; i += kFvThreads) s_dyn[i] = (double)__fsub_rn(n[b * ld_n + i], 1.0f);
  __syncthreads();
  if (threadIdx.x < 64) tridiag_psi_wave<double>(s_dyn, nx, threadIdx.x);
  __syncthreads();
  const double h = pc[0];
  for (int i = threadIdx.x; i < nx; i += kFvThreads) E[b * ld_E + i] = (float)tri_E(s_dyn, i, nx, h);
}

// ------------------------------------------------------------ FFT sizes
// One WAVE per pair of ICs (4 waves per workgroup, no workgroup barrier):
// lane l owns cells l + 64v (v < N/64) of both ICs.  It reads n, u, E (and F
// in hybrid mode) once, coalesced; the chain neighbours u[i-1], F[i-1] (and
// u[i+1] for the viscous term) come from the adjacent lane by a wave rotation
// (DPP wave_ror / wave_rol: lane 0's left neighbour is lane 63 of the
// previous register, the periodic wrap included).  The update writes n', u'
// and packs rho = n' - 1 of the two ICs as one complex value, which
// poisson_wave<N> turns into N (E_a + i E_b) in the same registers.
// HBM: 12 B read + 12 B write per cell (+4 B F).  The transforms use a
// wave-private padded LDS buffer.
constexpr int kDppWaveShl1 = 0x130;  // lane l <- lane l+1 (lane 63: no source)
constexpr int kDppWaveRol1 = 0x134;  // lane l <- lane l+1 (lane 63 <- lane 0)
constexpr int kDppWaveShr1 = 0x138;  // lane l <- lane l-1 (lane 0: no source)
constexpr int kDppWaveRor1 = 0x13C;  // lane l <- lane l-1 (lane 0 <- lane 63)
// src moved by CTRL; lanes without a source keep `old`
template <int CTRL>
__device__ __forceinline__ float wave_dpp(float old, float src) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src), CTRL, 0xF, 0xF, false));
}
// value at cell i-1 (left) or i+1 (right) for every register of a lane's
// cells: a wave shift, and for the lane that shifts out of the wave (lane 0
// left, lane 63 right) the rotated neighbour register (periodic wrap included)
template <int V>
__device__ __forceinline__ void left_of(const float (&x)[V], float (&l)[V]) {
#pragma unroll
  for (int i = 0; i < V; ++i)
    l[i] = wave_dpp<kDppWaveShr1>(wave_dpp<kDppWaveRor1>(0.f, x[(i + V - 1) % V]), x[i]);
}
template <int V>
__device__ __forceinline__ void right_of(const float (&x)[V], float (&rt)[V]) {
#pragma unroll
  for (int i = 0; i < V; ++i) rt[i] = wave_dpp<kDppWaveShl1>(wave_dpp<kDppWaveRol1>(0.f, x[(i + 1) % V]), x[i]);
}

constexpr int kFftWaves = 4;

// One IC's step inputs, cells lane + 64v: n, u, E and the face flux F
// (hybrid: the GNN's; classical: n*u, src/baseline_solver.py:70-71).
template <int N>
struct FvIn {
  float n[N / 64], u[N / 64], E[N / 64], F[N / 64];
};
template <bool HYBRID, int N>
__device__ __forceinline__ void fv_load(const float *__restrict__ st, const float *__restrict__ Fb, int lane,
                                        FvIn<N> &x) {
#pragma unroll
  for (int i = 0; i < N / 64; ++i) {
    const int cell = lane + 64 * i;
    x.n[i] = st[cell];
    x.u[i] = st[N + cell];
    x.E[i] = st[2 * N + cell];
    if constexpr (HYBRID) x.F[i] = Fb[cell];
  }
  if constexpr (!HYBRID) {
#pragma unroll
    for (int i = 0; i < N / 64; ++i) x.F[i] = __fmul_rn(x.n[i], x.u[i]);
  }
}

// The update of one IC's cells (lane + 64v) held by this lane: writes n', u'
// (and F), accumulates the n, u part of the metrics, returns rho = n' - 1.
template <bool HYBRID, int N>
__device__ __forceinline__ void fv_update_in(const FvIn<N> &x, float *__restrict__ so, float c, float dt, float nu,
                                             float dx2, float *__restrict__ fo, bool want_m, MetricAcc &m, int lane,
                                             double (&rho)[N / 64]) {
  constexpr int V = N / 64;
  float ul[V], Fl[V], ur[V];
  left_of<V>(x.u, ul);
  left_of<V>(x.F, Fl);
  if constexpr (!HYBRID) right_of<V>(x.u, ur);
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int cell = lane + 64 * i;
    const float n_new = continuity(x.n[i], x.F[i], Fl[i], c);
    float u_new;
    if constexpr (HYBRID) u_new = velocity_hybrid(x.u[i], ul[i], x.E[i], c, dt);
    else u_new = velocity_classical(x.u[i], ul[i], ur[i], x.E[i], c, dt, nu, dx2);
    so[cell] = n_new;
    so[N + cell] = u_new;
    if (fo) fo[cell] = x.F[i];
    if (want_m) m.add_nu(n_new, u_new);
    rho[i] = (double)__fsub_rn(n_new, 1.0f);
  }
}

// The Poisson stage of the FFT-size kernels on one wave's IC pair: on entry
// v[i] = (rho_a, rho_b) at cell lane + 64 i, on exit (E_a, E_b) there before
// the float32 rounding.  Spectral (the reference's operator): the packed
// transform pair (poisson_wave_tw), then / N.  TRI (HF_POISSON_TRIDIAG): the
// pair's rows through the wave-private LDS buffer, cyclic reduction on both
// at once (tridiag_psi_wave<double2>), E = h (psi[i-1] - psi[i+1]).
template <int N, bool TRI>
__device__ __forceinline__ void poisson_pair(double2 (&v)[N / 64], double2 *lds, const double2 *__restrict__ tw,
                                             const double *__restrict__ inv_k, double h, int lane) {
  if constexpr (TRI) {
    wave_lds_fence();  // earlier reads of the buffer (the parked rho of IC a) are done
#pragma unroll
    for (int i = 0; i < N / 64; ++i) lds[lane + 64 * i] = v[i];
    wave_lds_fence();
    tridiag_psi_wave<double2>(lds, N, lane);
#pragma unroll
    for (int i = 0; i < N / 64; ++i) v[i] = tri_E(lds, lane + 64 * i, N, h);
    wave_lds_fence();  // every lane's psi reads before the buffer is written again
  } else {
    poisson_wave_tw<N>(v, lds, tw, inv_k, lane);
#pragma unroll
    for (int i = 0; i < N / 64; ++i) v[i] = make_double2(v[i].x / N, v[i].y / N);
  }
}

template <int N, bool IMAG>
__device__ __forceinline__ void fv_finish_lane(float *__restrict__ so, const double2 (&v)[N / 64], MetricAcc &m,
                                               float *__restrict__ mo, int lane) {
#pragma unroll
  for (int i = 0; i < N / 64; ++i) {
    const float E_new = (float)(IMAG ? v[i].y : v[i].x);
    so[2 * N + lane + 64 * i] = E_new;
    if (mo) m.add_E(E_new);
  }
  if (mo) {
    m.wave_reduce();
    if (lane == 0) m.store(mo, N);
  }
}

// N = 2048: the wave-private LDS (4 x 2176 double2, ~139 KB) admits one
// workgroup per CU, so a min-blocks hint of 2 would only cap the VGPRs.
template <bool HYBRID, int N, bool TRI>
__global__ __launch_bounds__(64 * kFftWaves, N >= 2048 ? 1 : 2) void fv_step_fft_kernel(
    const float *__restrict__ in, int64_t ld_in, float *__restrict__ out, int64_t ld_out,
    const float *__restrict__ face_flux, const double *__restrict__ pc, float c, float dt, float nu, float dx2,
    float *__restrict__ flux_out, int64_t ld_flux, float *__restrict__ metrics, int64_t ld_metrics, int B) {
  constexpr int V = N / 64;
  __shared__ double2 s_fft[kFftWaves][fft_lds_elems<N>()];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;  // wave-uniform: scalar IC indices and bases
  const int64_t a = 2 * ((int64_t)blockIdx.x * kFftWaves + wave), b = a + 1;
  if (a >= B) return;  // a whole wave; nothing below synchronises the workgroup
  const bool two = b < B;
  double *rho_a = reinterpret_cast<double *>(s_fft[wave]);  // the transform's buffer, free until it starts
  MetricAcc ma, mb;
  ma.init();
  mb.init();
  double2 v[V];
  // IC b's inputs are loaded before IC a's stores: loads and stores share
  // vmcnt, so a load issued after them would wait until they had drained
  // (HF_FV_NO_PREFETCH: the old order, A/B builds only)
  FvIn<N> xb;
#ifndef HF_FV_NO_PREFETCH
  if (two) fv_load<HYBRID, N>(in + b * ld_in, HYBRID ? face_flux + b * N : nullptr, lane, xb);
#endif
  {
    FvIn<N> xa;
    fv_load<HYBRID, N>(in + a * ld_in, HYBRID ? face_flux + a * N : nullptr, lane, xa);
    double r[V];
    fv_update_in<HYBRID, N>(xa, out + a * ld_out, c, dt, nu, dx2, flux_out ? flux_out + a * ld_flux : nullptr,
                            metrics != nullptr, ma, lane, r);
#pragma unroll
    for (int i = 0; i < V; ++i) rho_a[lane + 64 * i] = r[i];  // parked while IC b's update holds the registers
  }
  {
    double r[V];
#ifdef HF_FV_NO_PREFETCH
    if (two) fv_load<HYBRID, N>(in + b * ld_in, HYBRID ? face_flux + b * N : nullptr, lane, xb);
#endif
    if (two)
      fv_update_in<HYBRID, N>(xb, out + b * ld_out, c, dt, nu, dx2, flux_out ? flux_out + b * ld_flux : nullptr,
                              metrics != nullptr, mb, lane, r);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < V; ++i) v[i] = make_double2(rho_a[lane + 64 * i], two ? r[i] : 0.0);
  }
  poisson_pair<N, TRI>(v, s_fft[wave], reinterpret_cast<const double2 *>(pc + N), pc + 2 * N, TRI ? pc[0] : 0.0,
                       lane);
  fv_finish_lane<N, false>(out + a * ld_out, v, ma, metrics ? metrics + a * ld_metrics : nullptr, lane);
  if (two) fv_finish_lane<N, true>(out + b * ld_out, v, mb, metrics ? metrics + b * ld_metrics : nullptr, lane);
}

// ---------------------------------------------- classical rollout, FFT sizes
// BaselineSolver.run over T steps in ONE launch (src/baseline_solver.py:80-118):
// the wave of an IC pair keeps both states in registers for the whole
// rollout, so HBM sees state0 once, the trajectory rows it is asked for
// (12 B/cell-step) and the final state; no state is re-read.  Every step is
// the arithmetic of fv_step_fft_kernel<false, N> in the same order (update of
// IC a, of IC b, the packed transform, E of a, of b; the metrics' partial sums
// the same), so the rollout equals T launches of it bit for bit.  Registers:
// n, u, E of two ICs (6 N/64) + the packed rho/E (4 N/64): N <= kFvRunMaxNx.
constexpr int kFvRunMaxNx = 1024;

// classical update of one IC held in registers (fv_update_in<false, N>'s
// expressions); n, u become n', u'; rho = n' - 1.  ro: trajectory row or null.
template <int N>
__device__ __forceinline__ void fv_update_regs(float (&n)[N / 64], float (&u)[N / 64], const float (&E)[N / 64],
                                               float *ro, float *fo, float c, float dt, float nu, float dx2,
                                               bool want_m, MetricAcc &m, int lane, double (&rho)[N / 64]) {
  constexpr int V = N / 64;
  float F[V], ul[V], Fl[V], ur[V];
#pragma unroll
  for (int i = 0; i < V; ++i) F[i] = __fmul_rn(n[i], u[i]);  // F_n = n*u (src/baseline_solver.py:70-71)
  left_of<V>(u, ul);
  left_of<V>(F, Fl);
  right_of<V>(u, ur);
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int cell = lane + 64 * i;
    const float n_new = continuity(n[i], F[i], Fl[i], c);
    const float u_new = velocity_classical(u[i], ul[i], ur[i], E[i], c, dt, nu, dx2);
    if (ro) {
      ro[cell] = n_new;
      ro[N + cell] = u_new;
    }
    if (fo) fo[cell] = F[i];
    if (want_m) m.add_nu(n_new, u_new);
    rho[i] = (double)__fsub_rn(n_new, 1.0f);
    n[i] = n_new;
    u[i] = u_new;
  }
}

template <int N>
__device__ __forceinline__ void fv_run_E(float (&E)[N / 64], const double2 (&v)[N / 64], bool imag, float *ro,
                                         MetricAcc &m, float *mo, int lane) {
#pragma unroll
  for (int i = 0; i < N / 64; ++i) {
    E[i] = (float)(imag ? v[i].y : v[i].x);
    if (ro) ro[2 * N + lane + 64 * i] = E[i];
    if (mo) m.add_E(E[i]);
  }
  if (mo) {
    m.wave_reduce();
    if (lane == 0) m.store(mo, N);
  }
}

// Channel MSE of one IC's state (x) against a row of a reference trajectory,
// in traj_mse_kernel's arithmetic and order: its thread 64w + l sums cells
// l + 64(w + 4k) in k order, each wave xor-reduces, then the 4 wave partials
// are added in w order (scripts/evaluation/evaluate_multi_ic.py:88-90).
template <int N>
__device__ __forceinline__ float mse_channel(const float (&x)[N / 64], const float *__restrict__ ref, int lane) {
  constexpr int V = N / 64, W = kFvThreads / 64;
  double p[W];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    p[w] = 0.0;
#pragma unroll
    for (int i = w; i < V; i += W) {
      const double d = (double)ref[lane + 64 * i] - (double)x[i];
      p[w] += d * d;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) p[w] += __shfl_xor(p[w], o, 64);
  }
  double t = 0.0;
#pragma unroll
  for (int w = 0; w < W; ++w) t += p[w];
  return (float)(t / N);
}
template <int N>
__device__ __forceinline__ void mse_row(const float (&n)[N / 64], const float (&u)[N / 64], const float (&E)[N / 64],
                                        const float *__restrict__ ref, float *mo, int lane) {
  const float m0 = mse_channel<N>(n, ref, lane), m1 = mse_channel<N>(u, ref + N, lane),
              m2 = mse_channel<N>(E, ref + 2 * N, lane);
  if (lane == 0) {
    mo[0] = m0;
    mo[1] = m1;
    mo[2] = m2;
  }
}

// state0 (IC stride ld_s0) and state_final may alias: a wave reads its pair
// whole before its last step writes it, and no other wave touches that pair.
// state_final may be NULL.  No pointer is __restrict__: hf_run_compare passes
// the hybrid trajectory as both state0 (its row 0) and ref.  ref/mse (both or neither): the per-step channel
// MSE [B][T+1][3] of the reference trajectory ref [B][T+1][3][N] minus this
// rollout (hf_run_compare's classical twin, scored as it steps).
template <int N, bool SCORE, bool TRI>
__global__ __launch_bounds__(64 * kFftWaves, N >= 1024 ? 1 : 2) void fv_run_fft_kernel(
    const float *state0, int64_t ld_s0, float *state_final, float *traj, const double *__restrict__ pc, float c,
    float dt, float nu, float dx2, float *flux_traj, float *metrics, const float *ref, float *mse, int B, int T) {
  constexpr int V = N / 64;
  constexpr int64_t S = 3LL * N;
  __shared__ double2 s_fft[kFftWaves][fft_lds_elems<N>()];
  // the plan's twiddles and 1/k, staged once: the step loop then issues no
  // global load, so no vmcnt wait holds a wave until its trajectory stores
  // have drained (stores and loads share the counter)
  // (TRI: the plan is h alone)
  __shared__ double2 s_plan[TRI ? 1 : N];
  if constexpr (!TRI) {
    for (int i = threadIdx.x; i < 2 * N; i += 64 * kFftWaves) reinterpret_cast<double *>(s_plan)[i] = pc[N + i];
    __syncthreads();
  }
  const double h = TRI ? pc[0] : 0.0;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;  // wave-uniform: scalar IC indices and bases
  const int64_t a = 2 * ((int64_t)blockIdx.x * kFftWaves + wave), b = a + 1;
  if (a >= B) return;  // a whole wave; nothing below synchronises the workgroup
  const bool two = b < B;
  const int64_t ldT = (T + 1) * S, ldM = (int64_t)(T + 1) * HF_NUM_METRICS;
  float na[V], ua[V], Ea[V], nb[V], ub[V], Eb[V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int cell = lane + 64 * i;
    na[i] = state0[a * ld_s0 + cell];
    ua[i] = state0[a * ld_s0 + N + cell];
    Ea[i] = state0[a * ld_s0 + 2 * N + cell];
    nb[i] = two ? state0[b * ld_s0 + cell] : 0.f;
    ub[i] = two ? state0[b * ld_s0 + N + cell] : 0.f;
    Eb[i] = two ? state0[b * ld_s0 + 2 * N + cell] : 0.f;
  }
  if constexpr (SCORE) {
    mse_row<N>(na, ua, Ea, ref + a * ldT, mse + a * (T + 1) * 3, lane);
    if (two) mse_row<N>(nb, ub, Eb, ref + b * ldT, mse + b * (T + 1) * 3, lane);
  }
  for (int t = 0; t < T; ++t) {
    float *ra = traj ? traj + a * ldT + (t + 1) * S : nullptr;
    float *rb = traj && two ? traj + b * ldT + (t + 1) * S : nullptr;
    float *fa = flux_traj ? flux_traj + a * (int64_t)T * N + (int64_t)t * N : nullptr;
    float *fb = flux_traj && two ? flux_traj + b * (int64_t)T * N + (int64_t)t * N : nullptr;
    float *ma_o = metrics ? metrics + a * ldM + (int64_t)(t + 1) * HF_NUM_METRICS : nullptr;
    float *mb_o = metrics && two ? metrics + b * ldM + (int64_t)(t + 1) * HF_NUM_METRICS : nullptr;
    MetricAcc ma, mb;
    ma.init();
    mb.init();
    double2 v[V];
    {
      double r[V];
      fv_update_regs<N>(na, ua, Ea, ra, fa, c, dt, nu, dx2, metrics != nullptr, ma, lane, r);
#pragma unroll
      for (int i = 0; i < V; ++i) v[i].x = r[i];
    }
    {
      double r[V];
      if (two) fv_update_regs<N>(nb, ub, Eb, rb, fb, c, dt, nu, dx2, metrics != nullptr, mb, lane, r);
#pragma unroll
      for (int i = 0; i < V; ++i) v[i].y = two ? r[i] : 0.0;
    }
    poisson_pair<N, TRI>(v, s_fft[wave], s_plan, reinterpret_cast<const double *>(s_plan) + N, h, lane);
    fv_run_E<N>(Ea, v, false, ra, ma, ma_o, lane);
    if (two) fv_run_E<N>(Eb, v, true, rb, mb, mb_o, lane);
    if constexpr (SCORE) {
      mse_row<N>(na, ua, Ea, ref + a * ldT + (t + 1) * S, mse + (a * (T + 1) + t + 1) * 3, lane);
      if (two) mse_row<N>(nb, ub, Eb, ref + b * ldT + (t + 1) * S, mse + (b * (T + 1) + t + 1) * 3, lane);
    }
  }
  if (!state_final) return;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int cell = lane + 64 * i;
    state_final[a * S + cell] = na[i];
    state_final[a * S + N + cell] = ua[i];
    state_final[a * S + 2 * N + cell] = Ea[i];
    if (two) {
      state_final[b * S + cell] = nb[i];
      state_final[b * S + N + cell] = ub[i];
      state_final[b * S + 2 * N + cell] = Eb[i];
    }
  }
}

// ------------------------------------- classical rollout, nx <= 64 (circulant)
// BaselineSolver.run over T steps in one launch for small chains (the
// reference's default nx = 64, src/baseline_solver.py:80-118): one WAVE per
// IC, lane i holds cell i's n, u, E in registers for the whole rollout; the
// chain neighbours come by lane shuffle, rho goes through a wave-private LDS
// row, and E is poisson_cell over it, exactly as fv_step_kernel<false>
// evaluates every expression (its cells all sit in its wave 0, so its
// workgroup reduction of the metrics is this wave's reduction followed by
// three +0.0 partials, reproduced below).  Bit-identical to T hf_step calls.
constexpr int kFvSmallMaxNx = 64;

__global__ __launch_bounds__(kFvThreads) void fv_run_small_kernel(const float *state0, float *state_final,
                                                                  float *traj, const double *__restrict__ pc, int nx,
                                                                  float c, float dt, float nu, float dx2,
                                                                  float *flux_traj, float *metrics, int B, int T,
                                                                  int tri) {
  __shared__ double s_c[kFvSmallMaxNx];
  __shared__ float s_rho[kFvThreads / 64][kFvSmallMaxNx];
  __shared__ double s_psi[kFvThreads / 64][kFvSmallMaxNx];  // tri: the wave's cyclic-reduction row
  if (!tri) {
    for (int i = threadIdx.x; i < nx; i += kFvThreads) s_c[i] = pc[i];
    __syncthreads();
  }
  const double h = tri ? pc[0] : 0.0;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), i = threadIdx.x & 63;  // wave-uniform
  const int64_t b = (int64_t)blockIdx.x * (kFvThreads / 64) + wave;
  if (b >= B) return;  // a whole wave; nothing below synchronises the workgroup
  const int64_t S = 3LL * nx, ldT = (T + 1) * S, ldM = (int64_t)(T + 1) * HF_NUM_METRICS;
  const bool on = i < nx;
  const int im = i == 0 ? nx - 1 : i - 1, ip = i >= nx - 1 ? 0 : i + 1;
  float n = on ? state0[b * S + i] : 0.f, u = on ? state0[b * S + nx + i] : 0.f,
        E = on ? state0[b * S + 2 * nx + i] : 0.f;
  float *rho = s_rho[wave];
  for (int t = 0; t < T; ++t) {
    const float F = __fmul_rn(n, u);  // F_n = n*u (:70-71)
    const float um = __shfl(u, im, 64), up = __shfl(u, ip, 64), Fm = __shfl(F, im, 64);
    const float n_new = continuity(n, F, Fm, c);
    const float u_new = velocity_classical(u, um, up, E, c, dt, nu, dx2);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the previous step's rho reads are done
    if (tri) {
      if (on) s_psi[wave][i] = (double)__fsub_rn(n_new, 1.0f);
    } else if (on) {
      rho[i] = __fsub_rn(n_new, 1.0f);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every lane's rho is in LDS
    float *row = traj ? traj + b * ldT + (int64_t)(t + 1) * S : nullptr;
    if (on) {
      if (row) {
        row[i] = n_new;
        row[nx + i] = u_new;
      }
      if (flux_traj) flux_traj[b * (int64_t)T * nx + (int64_t)t * nx + i] = F;
    }
    if (tri) tridiag_psi_wave<double>(s_psi[wave], nx, i);
    const float E_new = !on ? 0.f : tri ? (float)tri_E(s_psi[wave], i, nx, h) : poisson_cell(rho, s_c, i, nx);
    if (on && row) row[2 * nx + i] = E_new;
    n = n_new;
    u = u_new;
    E = E_new;
    if (metrics) {
      MetricAcc m;
      m.init();
      if (on) m.add(n, u, E);
      m.wave_reduce();
      if (i == 0) {
        MetricAcc w;  // block_metrics' sum over the workgroup's 4 wave partials
        w.init();
        w.energy += m.energy;
        w.charge += m.charge;
        w.maxdev = m.maxdev > w.maxdev ? m.maxdev : w.maxdev;
        w.finite &= m.finite;
        for (int k = 1; k < kFvThreads / 64; ++k) {
          w.energy += 0.0;
          w.charge += 0.0;
        }
        w.store(metrics + b * ldM + (int64_t)(t + 1) * HF_NUM_METRICS, nx);
      }
    }
  }
  if (on) {
    state_final[b * S + i] = n;
    state_final[b * S + nx + i] = u;
    state_final[b * S + 2 * nx + i] = E;
  }
}

// hf_poisson at FFT sizes: one wave per pair of ICs, as above.
template <int N>
__global__ __launch_bounds__(64 * kFftWaves, N >= 2048 ? 1 : 2) void poisson_fft_kernel(const float *__restrict__ n, int ld_n,
                                                                     float *__restrict__ E, int ld_E,
                                                                     const double *__restrict__ pc, int B) {
  constexpr int V = N / 64;
  __shared__ double2 s_fft[kFftWaves][fft_lds_elems<N>()];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;  // wave-uniform: scalar IC indices and bases
  const int64_t b0 = 2 * ((int64_t)blockIdx.x * kFftWaves + wave);
  if (b0 >= B) return;
  const bool two = b0 + 1 < B;
  double2 v[V];
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int cell = lane + 64 * i;
    v[i].x = (double)__fsub_rn(n[b0 * ld_n + cell], 1.0f);  // rho = n - n0 (:60)
    v[i].y = two ? (double)__fsub_rn(n[(b0 + 1) * ld_n + cell], 1.0f) : 0.0;
  }
  poisson_wave<N>(v, s_fft[wave], pc, lane);
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int cell = lane + 64 * i;
    E[b0 * ld_E + cell] = (float)(v[i].x / N);
    if (two) E[(b0 + 1) * ld_E + cell] = (float)(v[i].y / N);
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
  const int64_t b = blockIdx.x;
  for (int i = threadIdx.x; i < nx; i += kFvThreads) {
    L.c[i] = pc[i];
    L.rho[i] = __fsub_rn(n[b * ld_n + i], 1.0f);  // rho = n - n0 (:60)
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nx; i += kFvThreads) E[b * ld_E + i] = poisson_cell(L.rho, L.c, i, nx);
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

template <int N, bool TRI>
hipError_t fv_fft_launch(const float *in, int64_t ld_in, float *out, int64_t ld_out, const float *face_flux,
                         const double *pc, int B, float c, float dt, float nu, float dx2, float *flux_out,
                         int64_t ld_flux, float *metrics, int64_t ld_metrics, hipStream_t s) {
  const unsigned grid = (unsigned)((B + 2 * kFftWaves - 1) / (2 * kFftWaves));
  if (face_flux)
    hipLaunchKernelGGL((fv_step_fft_kernel<true, N, TRI>), dim3(grid), dim3(64 * kFftWaves), 0, s, in, ld_in, out,
                       ld_out, face_flux, pc, c, dt, nu, dx2, flux_out, ld_flux, metrics, ld_metrics, B);
  else
    hipLaunchKernelGGL((fv_step_fft_kernel<false, N, TRI>), dim3(grid), dim3(64 * kFftWaves), 0, s, in, ld_in, out,
                       ld_out, face_flux, pc, c, dt, nu, dx2, flux_out, ld_flux, metrics, ld_metrics, B);
  return hipGetLastError();
}
template <int N>
hipError_t fv_fft_launch_pm(const float *in, int64_t ld_in, float *out, int64_t ld_out, const float *face_flux,
                            const double *pc, int B, float c, float dt, float nu, float dx2, float *flux_out,
                            int64_t ld_flux, float *metrics, int64_t ld_metrics, int pm, hipStream_t s) {
  return pm == HF_POISSON_TRIDIAG
             ? fv_fft_launch<N, true>(in, ld_in, out, ld_out, face_flux, pc, B, c, dt, nu, dx2, flux_out, ld_flux,
                                      metrics, ld_metrics, s)
             : fv_fft_launch<N, false>(in, ld_in, out, ld_out, face_flux, pc, B, c, dt, nu, dx2, flux_out, ld_flux,
                                       metrics, ld_metrics, s);
}

bool poisson_mode_ok(int pm, int nx) {
  return pm == HF_POISSON_SPECTRAL || (pm == HF_POISSON_TRIDIAG && nx >= 1 && nx <= kTriMaxNx);
}

hipError_t launch_fv_step(const float *in, int64_t ld_in, float *out, int64_t ld_out,
                          const float *face_flux, const double *pc, int B, int nx, float c,
                          float dt, float nu, float dx2, float *flux_out, int64_t ld_flux,
                          float *metrics, int64_t ld_metrics, int pm, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (!poisson_mode_ok(pm, nx)) return hipErrorInvalidValue;
  const int tri = pm == HF_POISSON_TRIDIAG;
  if (poisson_uses_fft(nx)) {
    switch (nx) {
      case 256: return fv_fft_launch_pm<256>(in, ld_in, out, ld_out, face_flux, pc, B, c, dt, nu, dx2, flux_out, ld_flux, metrics, ld_metrics, pm, s);
      case 512: return fv_fft_launch_pm<512>(in, ld_in, out, ld_out, face_flux, pc, B, c, dt, nu, dx2, flux_out, ld_flux, metrics, ld_metrics, pm, s);
      case 1024: return fv_fft_launch_pm<1024>(in, ld_in, out, ld_out, face_flux, pc, B, c, dt, nu, dx2, flux_out, ld_flux, metrics, ld_metrics, pm, s);
      case 2048: return fv_fft_launch_pm<2048>(in, ld_in, out, ld_out, face_flux, pc, B, c, dt, nu, dx2, flux_out, ld_flux, metrics, ld_metrics, pm, s);
      default: return hipErrorInvalidValue;
    }
  }
  if (nx > kFvLdsMaxNx) {  // large nx: update, Poisson, metrics as three launches
    const dim3 grid((unsigned)B, (unsigned)((nx + kFvThreads - 1) / kFvThreads));  // ICs on x (no 65535 cap)
    if (face_flux)
      hipLaunchKernelGGL(fv_update_kernel<true>, grid, dim3(kFvThreads), 0, s, in, ld_in, out, ld_out, face_flux, nx,
                         c, dt, nu, dx2, flux_out, ld_flux);
    else
      hipLaunchKernelGGL(fv_update_kernel<false>, grid, dim3(kFvThreads), 0, s, in, ld_in, out, ld_out, face_flux,
                         nx, c, dt, nu, dx2, flux_out, ld_flux);
    if (tri)
      hipLaunchKernelGGL(poisson_tri_kernel, dim3((unsigned)B), dim3(kFvThreads), sizeof(double) * nx, s, out, ld_out,
                         out + 2 * (int64_t)nx, ld_out, pc, nx);
    else
      hipLaunchKernelGGL(poisson_tiled_kernel, grid, dim3(kFvThreads), 0, s, out, ld_out, out + 2 * (int64_t)nx, ld_out,
                         pc, nx);
    if (metrics)
      hipLaunchKernelGGL(state_metrics_kernel, dim3(B), dim3(kFvThreads), 0, s, out, ld_out, nx, metrics, ld_metrics);
    return hipGetLastError();
  }
  const size_t lds = fv_lds_bytes(nx);
  if (face_flux)
    hipLaunchKernelGGL(fv_step_kernel<true>, dim3(B), dim3(kFvThreads), lds, s, in, ld_in, out,
                       ld_out, face_flux, pc, nx, c, dt, nu, dx2, flux_out, ld_flux, metrics,
                       ld_metrics, tri);
  else
    hipLaunchKernelGGL(fv_step_kernel<false>, dim3(B), dim3(kFvThreads), lds, s, in, ld_in, out,
                       ld_out, face_flux, pc, nx, c, dt, nu, dx2, flux_out, ld_flux, metrics,
                       ld_metrics, tri);
  return hipGetLastError();
}

template <int N, bool TRI>
hipError_t fv_run_fft_launch(const float *state0, int64_t ld_s0, float *state_final, float *traj, const double *pc,
                             int B, int T, float c, float dt, float nu, float dx2, float *flux_traj, float *metrics,
                             const float *ref, float *mse, hipStream_t s) {
  const unsigned grid = (unsigned)((B + 2 * kFftWaves - 1) / (2 * kFftWaves));
  if (mse)
    hipLaunchKernelGGL((fv_run_fft_kernel<N, true, TRI>), dim3(grid), dim3(64 * kFftWaves), 0, s, state0, ld_s0,
                       state_final, traj, pc, c, dt, nu, dx2, flux_traj, metrics, ref, mse, B, T);
  else
    hipLaunchKernelGGL((fv_run_fft_kernel<N, false, TRI>), dim3(grid), dim3(64 * kFftWaves), 0, s, state0, ld_s0,
                       state_final, traj, pc, c, dt, nu, dx2, flux_traj, metrics, ref, mse, B, T);
  return hipGetLastError();
}
template <int N>
hipError_t fv_run_fft_launch_pm(const float *state0, int64_t ld_s0, float *state_final, float *traj, const double *pc,
                                int B, int T, float c, float dt, float nu, float dx2, float *flux_traj, float *metrics,
                                const float *ref, float *mse, int pm, hipStream_t s) {
  return pm == HF_POISSON_TRIDIAG
             ? fv_run_fft_launch<N, true>(state0, ld_s0, state_final, traj, pc, B, T, c, dt, nu, dx2, flux_traj,
                                          metrics, ref, mse, s)
             : fv_run_fft_launch<N, false>(state0, ld_s0, state_final, traj, pc, B, T, c, dt, nu, dx2, flux_traj,
                                           metrics, ref, mse, s);
}

bool fv_run_fused(int nx) { return (poisson_uses_fft(nx) && nx <= kFvRunMaxNx) || (nx >= 1 && nx <= kFvSmallMaxNx); }

hipError_t launch_fv_run(const float *state0, int64_t ld_s0, float *state_final, float *traj, const double *pc, int B,
                         int nx, int T, float c, float dt, float nu, float dx2, float *flux_traj, float *metrics,
                         const float *ref, float *mse, int pm, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if ((ref == nullptr) != (mse == nullptr) || !poisson_mode_ok(pm, nx)) return hipErrorInvalidValue;
  if (nx <= kFvSmallMaxNx) {  // contiguous states; no scoring at these nx (the fused hybrid kernel has its twin)
    if (mse || ld_s0 != 3LL * nx || !state_final) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)((B + kFvThreads / 64 - 1) / (kFvThreads / 64));
    hipLaunchKernelGGL(fv_run_small_kernel, dim3(grid), dim3(kFvThreads), 0, s, state0, state_final, traj, pc, nx, c,
                       dt, nu, dx2, flux_traj, metrics, B, T, pm == HF_POISSON_TRIDIAG ? 1 : 0);
    return hipGetLastError();
  }
  switch (fv_run_fused(nx) ? nx : 0) {
    case 256: return fv_run_fft_launch_pm<256>(state0, ld_s0, state_final, traj, pc, B, T, c, dt, nu, dx2, flux_traj, metrics, ref, mse, pm, s);
    case 512: return fv_run_fft_launch_pm<512>(state0, ld_s0, state_final, traj, pc, B, T, c, dt, nu, dx2, flux_traj, metrics, ref, mse, pm, s);
    case 1024: return fv_run_fft_launch_pm<1024>(state0, ld_s0, state_final, traj, pc, B, T, c, dt, nu, dx2, flux_traj, metrics, ref, mse, pm, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_state_metrics(const float *st, int64_t ld, int B, int nx, float *metrics,
                                int64_t ld_metrics, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(state_metrics_kernel, dim3(B), dim3(kFvThreads), 0, s, st, ld, nx, metrics,
                     ld_metrics);
  return hipGetLastError();
}

template <int N>
hipError_t poisson_fft_launch(const float *n, int ld_n, float *E, int ld_E, const double *pc, int B, hipStream_t s) {
  const unsigned grid = (unsigned)((B + 2 * kFftWaves - 1) / (2 * kFftWaves));
  hipLaunchKernelGGL((poisson_fft_kernel<N>), dim3(grid), dim3(64 * kFftWaves), 0, s, n, ld_n, E, ld_E, pc, B);
  return hipGetLastError();
}

hipError_t launch_poisson(const float *n, int ld_n, float *E, int ld_E, const double *pc, int B,
                          int nx, int pm, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  if (!poisson_mode_ok(pm, nx)) return hipErrorInvalidValue;
  if (pm == HF_POISSON_TRIDIAG) {
    hipLaunchKernelGGL(poisson_tri_kernel, dim3((unsigned)B), dim3(kFvThreads), sizeof(double) * nx, s, n,
                       (int64_t)ld_n, E, (int64_t)ld_E, pc, nx);
    return hipGetLastError();
  }
  switch (poisson_uses_fft(nx) ? nx : 0) {
    case 256: return poisson_fft_launch<256>(n, ld_n, E, ld_E, pc, B, s);
    case 512: return poisson_fft_launch<512>(n, ld_n, E, ld_E, pc, B, s);
    case 1024: return poisson_fft_launch<1024>(n, ld_n, E, ld_E, pc, B, s);
    case 2048: return poisson_fft_launch<2048>(n, ld_n, E, ld_E, pc, B, s);
    default: break;
  }
  if (nx > kFvLdsMaxNx) {
    hipLaunchKernelGGL(poisson_tiled_kernel, dim3((unsigned)B, (unsigned)((nx + kFvThreads - 1) / kFvThreads)),
                       dim3(kFvThreads), 0, s, n, (int64_t)ld_n, E, (int64_t)ld_E, pc, nx);
    return hipGetLastError();
  }
  const size_t lds = fv_lds_bytes(nx);
  hipLaunchKernelGGL(poisson_kernel, dim3(B), dim3(kFvThreads), lds, s, n, ld_n, E, ld_E, pc, nx);
  return hipGetLastError();
}

}  // namespace hf
