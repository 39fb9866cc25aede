// Fused FluxGNN message passing on the periodic 1-D chain, float32 MFMA.
//
// Reference: src/flux_gnn.py:40-67 (forward), src/graph_constructor.py:34-38
// (chain edges), src/hybrid_solver.py:34-73 (the step / rollout it feeds).
//
// Mapping (one wave = 64 cells of one IC, hidden state resident in VGPRs):
//   Every GEMM is computed transposed, Out^T[n][m] = sum_k W[n][k] X[m][k], on
//   v_mfma_f32_16x16x4_f32 tiles with A = weights (rows n), B = activations
//   (columns m = cells).  Lane l of a 16x16 accumulator then holds cell
//   m = 16*mt + (l&15) and features n = 16*nt + 4*(l>>4) + r, r = 0..3 — which
//   is directly the B-operand fragment of the next layer if the k order of a
//   k-step is (nt, r) -> k = 16*nt + 4*(l>>4) + r.  The weight A fragments are
//   packed on the host in that permuted k order (capi.cpp), so activations
//   never leave registers between layers.
//   Cells lie along the 16 lanes of a DPP row, so the chain neighbours i-1 /
//   i+1 of the mean aggregation (deg = 2 on the chain, src/flux_gnn.py:55-59)
//   are row_shr:1 / row_shl:1, with the lane that falls off the row patched
//   from the adjacent m-tile by row_ror (periodic wrap inside the IC).
//   The edge MLP uses the P/Q split: z(i->j) = W_a h_i + W_b h_j + b, so P and
//   Q are per-node GEMMs (K=128) and each edge only adds a shifted pair.
#include "hf_device.h"
#include "hf_internal.h"

namespace hf {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// GFX9 DPP controls.
constexpr int kRowShl1 = 0x101;
constexpr int kRowShr1 = 0x111;
constexpr int kRowRor1 = 0x121;
constexpr int kRowRor15 = 0x12F;

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
// Lanes whose DPP source falls outside their row keep `old`.
template <int CTRL>
__device__ __forceinline__ float dpp_over(float old, float v) {
  return __int_as_float(
      __builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Value of cell m+1 for every lane (periodic over the MT m-tiles of the wave).
template <int MT>
__device__ __forceinline__ void right_nb(const float (&v)[MT], float (&r)[MT]) {
  float rot[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) rot[mt] = dpp_mov<kRowRor15>(v[mt]);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) r[mt] = dpp_over<kRowShl1>(rot[(mt + 1) % MT], v[mt]);
}
// Value of cell m-1 for every lane.
template <int MT>
__device__ __forceinline__ void left_nb(const float (&v)[MT], float (&l)[MT]) {
  float rot[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) rot[mt] = dpp_mov<kRowRor1>(v[mt]);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) l[mt] = dpp_over<kRowShr1>(rot[(mt + MT - 1) % MT], v[mt]);
}

__device__ __forceinline__ f4 relu4(f4 v) {
  return f4{relu(v.x), relu(v.y), relu(v.z), relu(v.w)};
}

__device__ __forceinline__ f4 ldf4(const float *p) { return *reinterpret_cast<const f4 *>(p); }

// A fragments of one k-step for all kNT output tiles: 8 consecutive floats per lane.
__device__ __forceinline__ void load_afrag(const float *p, float (&a)[kNT]) {
  f4 a0 = ldf4(p), a1 = ldf4(p + 4);
  a[0] = a0.x; a[1] = a0.y; a[2] = a0.z; a[3] = a0.w;
  a[4] = a1.x; a[5] = a1.y; a[6] = a1.z; a[7] = a1.w;
}

// FluxGNN forward for the MT*16 cells of this wave.  feat[mt] is the lane's
// input feature (index l>>4 of [n,u,E,x]) of cell 16*mt + (l&15).  Returns the
// edge fluxes of (i -> i+1) in ffwd and of (i+1 -> i) in fbwd for cell i, on
// every lane of the cell's column.
template <int MT>
__device__ __forceinline__ void gnn_chain(const ChainW &W, const float (&feat)[MT],
                                          float (&ffwd)[MT], float (&fbwd)[MT]) {
  const int lane = threadIdx.x & 63;
  const int g4 = 4 * (lane >> 4);
  f4 h[MT][kNT];

  // input MLP: h0 = ReLU(W_in x + b_in), K = 4 = one MFMA per tile   (src/flux_gnn.py:49)
  {
    float a[kNT];
    load_afrag(W.win + lane * kNT, a);
#pragma unroll
    for (int nt = 0; nt < kNT; ++nt) {
      const f4 bias = ldf4(W.bin + 16 * nt + g4);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) h[mt][nt] = relu4(mfma4(a[nt], feat[mt], bias));
    }
  }

  // message passing: h = ReLU(W_l [h ; (h[i+1]+h[i-1])/2] + b_l)        (src/flux_gnn.py:53-60)
  for (int l = 0; l < W.layers; ++l) {
    const float *wl = W.wl + (size_t)l * (2 * kKS * 64 * kNT) + lane * kNT;
    const float *bl = W.bl + l * kH + g4;
    f4 acc[MT][kNT];
#pragma unroll
    for (int nt = 0; nt < kNT; ++nt) {
      const f4 bias = ldf4(bl + 16 * nt);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt][nt] = bias;
    }
#pragma unroll
    for (int s = 0; s < kKS; ++s) {  // self half of the input, k = 16*(s>>2) + 4g + (s&3)
      float a[kNT];
      load_afrag(wl + s * (64 * kNT), a);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const float b = h[mt][s >> 2][s & 3];
#pragma unroll
        for (int nt = 0; nt < kNT; ++nt) acc[mt][nt] = mfma4(a[nt], b, acc[mt][nt]);
      }
    }
#pragma unroll
    for (int s = 0; s < kKS; ++s) {  // aggregated half, k = 128 + same order
      float a[kNT];
      load_afrag(wl + (kKS + s) * (64 * kNT), a);
      float v[MT], vl[MT], vr[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) v[mt] = h[mt][s >> 2][s & 3];
      left_nb<MT>(v, vl);
      right_nb<MT>(v, vr);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        // index_add_ of h[i+1] then h[i-1], divided by deg = 2 (exact)
        const float b = __fmul_rn(__fadd_rn(vr[mt], vl[mt]), 0.5f);
#pragma unroll
        for (int nt = 0; nt < kNT; ++nt) acc[mt][nt] = mfma4(a[nt], b, acc[mt][nt]);
      }
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < kNT; ++nt) h[mt][nt] = relu4(acc[mt][nt]);
  }

  // edge readout, P/Q split: z_fwd(i) = P(i) + Q(i+1), z_bwd(i) = P(i+1) + Q(i),
  // P = W_e[:, :H] h + b_e, Q = W_e[:, H:] h; flux = w2 . ReLU(z) + b2   (src/flux_gnn.py:62-66)
  float pf[MT], pb[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) pf[mt] = pb[mt] = 0.f;
  for (int ot = 0; ot < kNT; ++ot) {
    f4 P[MT], Q[MT];
    const f4 be = ldf4(W.be + 16 * ot + g4);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      P[mt] = be;
      Q[mt] = f4{0.f, 0.f, 0.f, 0.f};
    }
    const float *we = W.we + (size_t)ot * (kKS * 64 * 2) + lane * 2;
#pragma unroll
    for (int s = 0; s < kKS; ++s) {
      const float2 a = *reinterpret_cast<const float2 *>(we + s * 128);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const float b = h[mt][s >> 2][s & 3];
        P[mt] = mfma4(a.x, b, P[mt]);
        Q[mt] = mfma4(a.y, b, Q[mt]);
      }
    }
    const f4 w2 = ldf4(W.w2 + 16 * ot + g4);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float pv[MT], qv[MT], pr[MT], qr[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        pv[mt] = P[mt][r];
        qv[mt] = Q[mt][r];
      }
      right_nb<MT>(pv, pr);
      right_nb<MT>(qv, qr);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        pf[mt] = fmaf(w2[r], relu(__fadd_rn(pv[mt], qr[mt])), pf[mt]);
        pb[mt] = fmaf(w2[r], relu(__fadd_rn(pr[mt], qv[mt])), pb[mt]);
      }
    }
  }
  // the 128-feature dot product is split over the 4 lane groups of a column
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    pf[mt] += __shfl_xor(pf[mt], 16, 64);
    pf[mt] += __shfl_xor(pf[mt], 32, 64);
    pb[mt] += __shfl_xor(pb[mt], 16, 64);
    pb[mt] += __shfl_xor(pb[mt], 32, 64);
    ffwd[mt] = pf[mt] + W.b2;
    fbwd[mt] = pb[mt] + W.b2;
  }
}

// ---------------------------------------------------------------------------
// FluxGNN.forward on B chains, one wave per (IC, window).
//  EXACT: nx == 16*MT, the wave owns the whole periodic IC, every face exact.
//  else : MT == 4 window of 64 cells starting at w*55-4 (mod nx); faces
//         [4,58] of the window (55 per window) are exact, the rest discarded.
template <int MT, bool EXACT>
__global__ __launch_bounds__(64, 1) void chain_flux_kernel(ChainW W, const float *__restrict__ nf,
                                                           const float *__restrict__ state,
                                                           int64_t ld_state,
                                                           const float *__restrict__ x, int nx,
                                                           int nwin, float *__restrict__ fe,
                                                           float *__restrict__ ff) {
  const int lane = threadIdx.x;
  const int j = lane & 15, g = lane >> 4;
  const int b = blockIdx.x / nwin;
  const int w = blockIdx.x - b * nwin;
  const int start = EXACT ? 0 : w * kWinFaces - kWinHalo;
  float feat[MT];
  int cell[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    int cidx = start + 16 * mt + j;
    cidx %= nx;
    if (cidx < 0) cidx += nx;
    cell[mt] = cidx;
    if (nf) {
      feat[mt] = nf[((int64_t)b * nx + cidx) * kIn + g];
    } else {
      feat[mt] = g < 3 ? state[(int64_t)b * ld_state + (int64_t)g * nx + cidx] : x[cidx];
    }
  }
  float f_fwd[MT], f_bwd[MT];
  gnn_chain<MT>(W, feat, f_fwd, f_bwd);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int wc = 16 * mt + j;
    int face = cell[mt];
    bool ok = true;
    if (!EXACT) {
      face = w * kWinFaces + (wc - kWinHalo);
      ok = wc >= kWinHalo && wc < kWinHalo + kWinFaces && face < nx;
    }
    if (!ok) continue;
    if (fe && g == 0) fe[(int64_t)b * 2 * nx + face] = f_fwd[mt];
    if (fe && g == 1) fe[(int64_t)b * 2 * nx + nx + face] = f_bwd[mt];
    if (ff && g == 2) ff[(int64_t)b * nx + face] = face_flux(f_fwd[mt], f_bwd[mt]);
  }
}

// ---------------------------------------------------------------------------
// Persistent hybrid rollout, one wave per IC, nx = 16*MT: T steps of
// GNN -> symmetrise -> continuity -> Burgers -> spectral Poisson with the
// state held in LDS (src/hybrid_solver.py:34-73).
template <int MT>
__global__ __launch_bounds__(64, 1) void chain_rollout_kernel(
    ChainW W, const float *__restrict__ state0, float *__restrict__ state_final,
    const float *__restrict__ x, const double *__restrict__ pc, int T, float c, float dt,
    float *__restrict__ traj, float *__restrict__ flux_traj, float *__restrict__ metrics) {
  constexpr int NX = 16 * MT;
  __shared__ float s_st[4 * NX];  // n | u | E | x
  __shared__ float s_F[NX];
  __shared__ float s_rho[NX];
  __shared__ double s_c[NX];
  const int lane = threadIdx.x;
  const int j = lane & 15, g = lane >> 4;
  const int64_t b = blockIdx.x;
  const float *st0 = state0 + b * 3 * NX;
  for (int i = lane; i < 3 * NX; i += 64) s_st[i] = st0[i];
  if (lane < NX) {
    s_st[3 * NX + lane] = x[lane];
    s_c[lane] = pc[lane];
  }
  __syncthreads();
  float *tj = traj ? traj + b * (int64_t)(T + 1) * 3 * NX : nullptr;
  float *mt_out = metrics ? metrics + b * (int64_t)(T + 1) * HF_NUM_METRICS : nullptr;
  auto emit = [&](int t) {
    if (tj)
      for (int i = lane; i < 3 * NX; i += 64) tj[(int64_t)t * 3 * NX + i] = s_st[i];
    if (mt_out) {
      MetricAcc m;
      m.init();
      if (lane < NX) m.add(s_st[lane], s_st[NX + lane], s_st[2 * NX + lane]);
      m.wave_reduce();
      if (lane == 0) m.store(mt_out + t * HF_NUM_METRICS, NX);
    }
  };
  emit(0);
  for (int t = 0; t < T; ++t) {
    float feat[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) feat[mt] = s_st[g * NX + 16 * mt + j];
    float f_fwd[MT], f_bwd[MT];
    gnn_chain<MT>(W, feat, f_fwd, f_bwd);
    if (g == 0) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) s_F[16 * mt + j] = face_flux(f_fwd[mt], f_bwd[mt]);
    }
    __syncthreads();
    float n_new = 0.f, u_new = 0.f;
    if (lane < NX) {
      const int im = lane == 0 ? NX - 1 : lane - 1;
      const float F = s_F[lane];
      n_new = continuity(s_st[lane], F, s_F[im], c);
      u_new = velocity_hybrid(s_st[NX + lane], s_st[NX + im], s_st[2 * NX + lane], c, dt);
      s_rho[lane] = __fsub_rn(n_new, 1.0f);
      if (flux_traj) flux_traj[(b * T + t) * NX + lane] = F;
    }
    __syncthreads();
    if (lane < NX) {
      const float E_new = poisson_cell(s_rho, s_c, lane, NX);
      s_st[lane] = n_new;
      s_st[NX + lane] = u_new;
      s_st[2 * NX + lane] = E_new;
    }
    __syncthreads();
    emit(t + 1);
  }
  float *out = state_final + b * 3 * NX;
  for (int i = lane; i < 3 * NX; i += 64) out[i] = s_st[i];
}

template <int MT>
hipError_t rollout_mt(const ChainW &w, const float *state0, float *state_final, const float *x,
                      const double *pc, int B, int T, float c, float dt, float *traj,
                      float *flux_traj, float *metrics, hipStream_t s) {
  hipLaunchKernelGGL(chain_rollout_kernel<MT>, dim3(B), dim3(64), 0, s, w, state0, state_final, x,
                     pc, T, c, dt, traj, flux_traj, metrics);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_chain_flux(const ChainW &w, const float *nf, const float *state, int64_t ld_state,
                             const float *x, int B, int nx, float *flux_edge, float *flux_face,
                             hipStream_t s) {
  if (B <= 0) return hipSuccess;
  switch (nx) {
    case 16:
      hipLaunchKernelGGL((chain_flux_kernel<1, true>), dim3(B), dim3(64), 0, s, w, nf, state,
                         ld_state, x, nx, 1, flux_edge, flux_face);
      return hipGetLastError();
    case 32:
      hipLaunchKernelGGL((chain_flux_kernel<2, true>), dim3(B), dim3(64), 0, s, w, nf, state,
                         ld_state, x, nx, 1, flux_edge, flux_face);
      return hipGetLastError();
    case 48:
      hipLaunchKernelGGL((chain_flux_kernel<3, true>), dim3(B), dim3(64), 0, s, w, nf, state,
                         ld_state, x, nx, 1, flux_edge, flux_face);
      return hipGetLastError();
    case 64:
      hipLaunchKernelGGL((chain_flux_kernel<4, true>), dim3(B), dim3(64), 0, s, w, nf, state,
                         ld_state, x, nx, 1, flux_edge, flux_face);
      return hipGetLastError();
    default: {
      const int nwin = (nx + kWinFaces - 1) / kWinFaces;
      const int64_t blocks = (int64_t)B * nwin;
      if (blocks > 0x7fffffff) return hipErrorInvalidValue;
      hipLaunchKernelGGL((chain_flux_kernel<4, false>), dim3((unsigned)blocks), dim3(64), 0, s, w,
                         nf, state, ld_state, x, nx, nwin, flux_edge, flux_face);
      return hipGetLastError();
    }
  }
}

hipError_t launch_chain_rollout(const ChainW &w, const float *state0, float *state_final,
                                const float *x, const double *pc, int B, int nx, int T, float c,
                                float dt, float *traj, float *flux_traj, float *metrics,
                                hipStream_t s) {
  if (B <= 0) return hipSuccess;
  switch (nx) {
    case 16: return rollout_mt<1>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, s);
    case 32: return rollout_mt<2>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, s);
    case 48: return rollout_mt<3>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, s);
    case 64: return rollout_mt<4>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace hf
