// Small-batch persistent hybrid rollout, float32 (v_mfma_f32_16x16x4_f32):
// one IC per 4-wave workgroup, the output features split across the waves.
//
// Reference: src/flux_gnn.py:40-67 (forward), src/hybrid_solver.py:34-73.
//
// chain_rollout_kernel (chain_common.h) puts one IC on one wave and four ICs
// on a workgroup, so a batch of B ICs occupies B/4 CUs: at the 256-IC config
// (BASELINE configs[1]) only 64 of the 256 CUs work.  Here the four waves of a
// workgroup share ONE IC: wave w computes output tiles 2w, 2w+1 (32 of the 128
// features) of every layer for all 16*MT cells, and readout tiles 2w, 2w+1.
// Each layer's new h is exchanged through LDS (every wave needs all 128
// features as the next GEMM's B operand), and the four partial edge-flux dot
// products are summed through LDS.  B ICs then occupy B CUs.
//
// Each wave reads only its own A fragments, so there is no shared weight ring:
// a wave streams its private, linearly packed fragment stream (capi.cpp
// pack_chain_split) straight from L2 into registers, four units ahead.  A unit
// is one float4 per lane: two update-layer k-steps of the wave's two tiles
// (16 MFMAs), or one readout k-step of its two (P, Q) tile pairs (16 MFMAs).
// The cell layout, aggregation and FV/Poisson arithmetic are those of
// chain_common.h; only the order of the fp32 sums over feature tiles in the
// edge readout differs (four partial dot products, then their sum).
#include <utility>

#include "chain_common.h"

namespace hf {
namespace {

using namespace chain;

constexpr int kSplitDepth = 4;  // units in flight per wave

// Private fragment stream of one wave: units [0, total) of float4 per lane,
// consumed cyclically (one pass per GNN forward).
// Buffer loads with the unit offset in an SGPR and the lane offset in a fixed
// VGPR: no per-load VALU address arithmetic beside the f32 MFMAs.
struct SplitFeed {
  __amdgpu_buffer_rsrc_t rsrc;  // this wave's stream
  int lane_off;                 // lane * 16 bytes
  int total;                    // units per pass
  int next;                     // unit index of the next load
  f4 buf[kSplitDepth];
  __device__ __forceinline__ void init(const void *wave_base, int units, int lane) {
    total = units;
    rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(wave_base), 0, units * 1024, 0x00020000);
    lane_off = lane * 16;
  }
  __device__ __forceinline__ void load(int slot) {
    buf[slot] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, lane_off, next * 1024, 0));
    next = next + 1 == total ? 0 : next + 1;
  }
  __device__ __forceinline__ void prime() {
    next = 0;
#pragma unroll
    for (int i = 0; i < kSplitDepth; ++i) load(i);
  }
  // Unit I of the pass (I % depth is the slot); refills the slot.
  template <int I>
  __device__ __forceinline__ f4 take() {
    constexpr int slot = I % kSplitDepth;
    const f4 a = buf[slot];
    load(slot);
    return a;
  }
};

// LDS plan (floats): small weights | h exchange, double-buffered by layer
// parity, [2][nt 8][mt 4][lane 64][4] | IC scratch | partial fluxes [wave 4][2][64].
constexpr int kHxFloats = 2 * kNT * 4 * 64 * 4;
constexpr int kRedFloats = kWaves * 2 * 64;
constexpr int kSplitLds = kSmallFloats + kHxFloats + kWaveScratchFloats + kRedFloats;

__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// Two k-steps (unit U of the layer) for the wave's two output tiles.  k-steps
// 0..31 multiply h, 32..63 the neighbour sum h[i+1] + h[i-1] (1/deg folded
// into the packed W_b).  The sums are formed in place, one 16-value burst per
// feature tile right after the last k-step that needs that tile of h.
// (Exchanging each wave's own sums through LDS instead, 32 VALU per layer
// rather than 128, measured slower overall: the extra LDS traffic, barrier
// and registers outweigh the VALU saved.)
template <int MT, int U>
__device__ __forceinline__ void split_layer_unit(SplitFeed &F, f4 (&h)[MT][kNT], f4 (&acc)[MT][2]) {
  const f4 a = F.take<U>();
  constexpr int s0 = (2 * U) % kKS, s1 = (2 * U + 1) % kKS;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    acc[mt][0] = mfma4(a[0], h[mt][s0 >> 2][s0 & 3], acc[mt][0]);
    acc[mt][1] = mfma4(a[1], h[mt][s0 >> 2][s0 & 3], acc[mt][1]);
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    acc[mt][0] = mfma4(a[2], h[mt][s1 >> 2][s1 & 3], acc[mt][0]);
    acc[mt][1] = mfma4(a[3], h[mt][s1 >> 2][s1 & 3], acc[mt][1]);
  }
#ifndef HF_DIAG_NONB  // timing diagnostic only: results are wrong
  if constexpr (2 * U + 1 < kKS && (s1 & 3) == 3) {  // tile s1/4 of h consumed: h <- neighbour sums
    constexpr int nt = s1 >> 2;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v[MT], sum[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) v[mt] = h[mt][nt][r];
      nb_sum<MT>(v, sum);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) h[mt][nt][r] = sum[mt];
    }
  }
#endif
}

template <int MT, int... U>
__device__ __forceinline__ void split_layer(SplitFeed &F, f4 (&h)[MT][kNT], f4 (&acc)[MT][2],
                                            std::integer_sequence<int, U...>) {
  (split_layer_unit<MT, U>(F, h, acc), ...);
}

// Readout k-step S: P and Q of the wave's two output tiles.
template <int MT, int S>
__device__ __forceinline__ void split_readout_unit(SplitFeed &F, const f4 (&h)[MT][kNT], f4 (&P)[2][MT],
                                                   f4 (&Q)[2][MT]) {
  const f4 a = F.take<S>();
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const float b = h[mt][S >> 2][S & 3];
    P[0][mt] = mfma4(a[0], b, P[0][mt]);
    Q[0][mt] = mfma4(a[1], b, Q[0][mt]);
    P[1][mt] = mfma4(a[2], b, P[1][mt]);
    Q[1][mt] = mfma4(a[3], b, Q[1][mt]);
  }
}

template <int MT, int... S>
__device__ __forceinline__ void split_readout(SplitFeed &F, const f4 (&h)[MT][kNT], f4 (&P)[2][MT], f4 (&Q)[2][MT],
                                              std::integer_sequence<int, S...>) {
  (split_readout_unit<MT, S>(F, h, P, Q), ...);
}

// FluxGNN forward for the IC, this wave's share.  On return the face flux
// F = 0.5*(f_fwd + f_bwd) of every cell is in s_F (wave 0 writes it).
template <int MT>
__device__ __forceinline__ void split_gnn(const ChainW &W, const Small &S, SplitFeed &F, float *hx, float *red,
                                          int wave, int lane, const float (&feat)[MT], float *s_F) {
  const int j = lane & 15, g4 = 4 * (lane >> 4);
  f4 h[MT][kNT];
  input_layer<MT>(S, lane, feat, h);
  // message passing: h = ReLU(W_l [h ; (h[i+1]+h[i-1])/2] + b_l)        (src/flux_gnn.py:53-60)
  for (int l = 0; l < W.layers; ++l) {
    // b_l enters each chain as its initial accumulator (the C operand of its
    // first MFMA), as in CoreF32
    f4 acc[MT][2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const f4 bias = ldf4(S.bl + l * kH + 16 * (2 * wave + t) + g4);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt][t] = bias;
    }
    split_layer<MT>(F, h, acc, std::make_integer_sequence<int, kKS>{});
    // double-buffered by layer parity: a wave may write layer l+1's tiles
    // while a slower one still reads layer l's
    f4 *hx4 = reinterpret_cast<f4 *>(hx) + (l & 1) * (kNT * 4 * 64);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int nt = 2 * wave + t;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) hx4[(nt * 4 + mt) * 64 + lane] = relu4(acc[mt][t]);
    }
    lds_barrier();  // every wave's tiles in LDS
#pragma unroll
    for (int nt = 0; nt < kNT; ++nt)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) h[mt][nt] = hx4[(nt * 4 + mt) * 64 + lane];
  }

  // edge readout, P/Q split, tiles 2w, 2w+1 of this wave           (src/flux_gnn.py:62-66)
  f4 P[2][MT], Q[2][MT];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const f4 be = ldf4(S.be + 16 * (2 * wave + t) + g4);  // b_e as P's initial accumulator, as CoreF32
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      P[t][mt] = be;
      Q[t][mt] = f4{0.f, 0.f, 0.f, 0.f};
    }
  }
  split_readout<MT>(F, h, P, Q, std::make_integer_sequence<int, kKS>{});
  float pf[MT], pb[MT], ff[MT], fb[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) pf[mt] = pb[mt] = 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int ot = 2 * wave + t;
    readout_epilogue<MT, true>(P[t], Q[t], ldf4(S.be + 16 * ot + g4), ldf4(S.w2 + 16 * ot + g4), pf, pb);
  }
  readout_finish<MT>(pf, pb, 0.f, ff, fb);
  if (lane < 16) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      red[(wave * 2 + 0) * 64 + cell_of<MT>(mt, j)] = ff[mt];
      red[(wave * 2 + 1) * 64 + cell_of<MT>(mt, j)] = fb[mt];
    }
  }
  lds_barrier();
  if (wave == 0 && lane < 16 * MT) {
    float sf = 0.f, sb = 0.f;  // partial dots added in w order, as CoreF32
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      sf = __fadd_rn(sf, red[(w * 2 + 0) * 64 + lane]);
      sb = __fadd_rn(sb, red[(w * 2 + 1) * 64 + lane]);
    }
    s_F[lane] = face_flux(__fadd_rn(sf, W.b2), __fadd_rn(sb, W.b2));
  }
}

template <int MT>
__global__ __launch_bounds__(256, 1) void chain_rollout_split_kernel(
    ChainW W, const float *__restrict__ state0, float *__restrict__ state_final, const float *__restrict__ x,
    const double *__restrict__ pc, int B, int T, float c, float dt, float *__restrict__ traj,
    float *__restrict__ flux_traj, float *__restrict__ metrics) {
  constexpr int NX = 16 * MT;
  __shared__ f4 lds4[kSplitLds / 4];
  float *lds = reinterpret_cast<float *>(lds4);
  const Small S = stage_small(W, lds);
  float *hx = lds + kSmallFloats;
  float *scratch = hx + kHxFloats;
  float *red = scratch + kWaveScratchFloats;
  float *s_st = scratch;  // n | u | E | x   (4 x 64)
  float *s_F = scratch + 4 * 64;
  float *s_rho = scratch + 5 * 64;
  double *s_c = reinterpret_cast<double *>(scratch + 6 * 64);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, j = lane & 15, g = lane >> 4;
  const int64_t b = blockIdx.x;
  const float *st0 = state0 + b * 3 * NX;
  if (wave == 0) {
    for (int i = lane; i < 3 * NX; i += 64) s_st[(i / NX) * 64 + i % NX] = st0[i];
    if (lane < NX) {
      s_st[3 * 64 + lane] = x[lane];
      s_c[lane] = pc[lane];
    }
  }
  SplitFeed F;
  const int units = (W.layers + 1) * kKS;
  F.init(reinterpret_cast<const char *>(W.split) + (int64_t)wave * units * 1024, units, lane);
  F.prime();
  __syncthreads();
  float *tj = traj ? traj + b * (int64_t)(T + 1) * 3 * NX : nullptr;
  float *mt_out = metrics ? metrics + b * (int64_t)(T + 1) * HF_NUM_METRICS : nullptr;
  float *ftj = flux_traj ? flux_traj + b * (int64_t)T * NX : nullptr;
  auto emit = [&](int t) {  // wave 0
    if (tj)
      for (int i = lane; i < 3 * NX; i += 64) tj[(int64_t)t * 3 * NX + i] = s_st[(i / NX) * 64 + i % NX];
    if (mt_out) {
      MetricAcc m;
      m.init();
      if (lane < NX) m.add(s_st[lane], s_st[64 + lane], s_st[128 + lane]);
      m.wave_reduce();
      if (lane == 0) m.store(mt_out + t * HF_NUM_METRICS, NX);
    }
  };
  if (wave == 0) emit(0);
  for (int t = 0; t < T; ++t) {
    float feat[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) feat[mt] = s_st[g * 64 + cell_of<MT>(mt, j)];
    split_gnn<MT>(W, S, F, hx, red, wave, lane, feat, s_F);
    if (wave == 0) {  // src/hybrid_solver.py:45-63, one cell per lane
      wave_lds_sync();
      float n_new = 0.f, u_new = 0.f;
      if (lane < NX) {
        const int im = lane == 0 ? NX - 1 : lane - 1;
        const float Fv = s_F[lane];
        n_new = continuity(s_st[lane], Fv, s_F[im], c);
        u_new = velocity_hybrid(s_st[64 + lane], s_st[64 + im], s_st[128 + lane], c, dt);
        s_rho[lane] = __fsub_rn(n_new, 1.0f);
        if (ftj) ftj[(int64_t)t * NX + lane] = Fv;
      }
      wave_lds_sync();
      if (lane < NX) {
        const float E_new = poisson_cell(s_rho, s_c, lane, NX);
        s_st[lane] = n_new;
        s_st[64 + lane] = u_new;
        s_st[128 + lane] = E_new;
      }
      wave_lds_sync();
      emit(t + 1);
    }
    lds_barrier();  // new state visible to every wave
  }
  if (wave != 0) return;
  float *out = state_final + b * 3 * NX;
  for (int i = lane; i < 3 * NX; i += 64) out[i] = s_st[(i / NX) * 64 + i % NX];
}

template <int MT>
hipError_t split_launch(const ChainW &w, const float *state0, float *state_final, const float *x, const double *pc,
                        int B, int T, float c, float dt, float *traj, float *flux_traj, float *metrics,
                        hipStream_t s) {
  hipLaunchKernelGGL((chain_rollout_split_kernel<MT>), dim3(B), dim3(64 * kWaves), 0, s, w, state0, state_final,
                     x, pc, B, T, c, dt, traj, flux_traj, metrics);
  return hipGetLastError();
}

}  // namespace

// Whether the feature-split kernel beats the IC-per-wave kernel for B ICs:
// it runs B workgroups of one IC instead of B/4 workgroups of four, each at
// about 0.28x the time (a quarter of the MFMAs plus the h exchange).
bool chain_rollout_prefers_split(const ChainW &w, int B) {
  if (w.prec != kPrecF32 || w.split == nullptr || B <= 0) return false;
  const int cus = chain::resident_groups();
  const int64_t waves_rounds = ((int64_t)B + 4LL * cus - 1) / (4LL * cus);  // IC-per-wave kernel
  const int64_t split_rounds = ((int64_t)B + cus - 1) / cus;
  return split_rounds * 28 < waves_rounds * 100;
}

hipError_t launch_chain_rollout_split(const ChainW &w, const float *state0, float *state_final, const float *x,
                                      const double *pc, int B, int nx, int T, float c, float dt, float *traj,
                                      float *flux_traj, float *metrics, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  switch (nx) {
    case 16: return split_launch<1>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, s);
    case 32: return split_launch<2>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, s);
    case 48: return split_launch<3>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, s);
    case 64: return split_launch<4>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace hf
