// Fused FluxGNN on the periodic chain, exact float32: v_mfma_f32_16x16x4_f32.
//
// Reference: src/flux_gnn.py:40-67 (forward), src/graph_constructor.py:34-38
// (chain edges), src/hybrid_solver.py:34-73 (the step / rollout it feeds).
//
// Every GEMM is computed transposed, Out^T[n][m] = sum_k W[n][k] X[m][k],
// with A = weights (rows n) and B = activations (columns m = cells).  The
// 16x16 accumulator of one layer is, lane for lane, the B-operand fragment of
// the next layer when the k order of a k-step is (nt, r) -> k = 16*nt +
// 4*(l>>4) + r; the weight fragments are packed on the host in that permuted
// order (capi.cpp pack_chain_f32), so activations never leave registers.
// The mean aggregation (h[i+1] + h[i-1]) / 2 (deg = 2 on the chain,
// src/flux_gnn.py:55-59) is formed from lane shifts on the input side, in
// float32, exactly as the reference's index_add_ / bincount.  The edge MLP
// uses the P/Q split z(i->j) = W_a h_i + W_b h_j + b: two per-node K=128
// GEMMs plus a shifted add.
#include "chain_common.h"

namespace hf {
namespace {

using namespace chain;

// D = weight chunks in flight ahead of the one consumed, SLOTS = ring slots
// (chain_common.h Ring): 2 in 4 for the IC-per-wave kernels; the cell-split
// kernels consume a chunk in a quarter of the time (16 cells per wave) and run
// deeper (kCellsAhead).
template <int D = 2, int SLOTS = kRingSlots>
struct CoreF32T {
  static constexpr int kNW = kWaves;   // waves sharing the weight ring
  static constexpr int kWGPerCU = 1;   // persistent flux kernel: workgroups per CU
  static constexpr int kStreamOffset = 0;  // bytes of the packed stream before chunk 0
  static constexpr int kSlots = SLOTS;
  static constexpr int kAhead = D;
  static constexpr int kWinMT = 4;     // m-tiles per wave in the windowed flux kernel
  // units per ring chunk: 4 (8 KiB chunks); 8 (16 KiB, half the barriers)
  // measured no faster, for the IC-per-wave and the cell-split kernels alike
  static constexpr int kUPC = 4;
  static constexpr int kChunkFloats = 512 * kUPC;  // 4 units of 2 KiB (2 ds_read_b128 per lane)
  static constexpr int kParkFloats = 0;
  using R_t = Ring<kChunkFloats, kNW, kSlots, kAhead>;

  // Register-prefetched weight feed.  A chunk is 4 units; unit u is the lane's
  // fragments 2u, 2u+1 and feeds 32 MFMAs (one update k-step, or four readout
  // k-steps of P and Q).  The ds_reads of unit u+1 are issued before the MFMAs
  // of unit u, so LDS latency hides under a whole unit of matrix work; the
  // ring's wait + barrier for chunk p+1 moves to before the last unit of p.
  // The feed runs continuously over forward passes (begin() once per kernel).
  struct Feed {
    const float *slot;
    f4 cur[2];
  };
  static __device__ __forceinline__ void load_unit(Feed &F, int u, int lane) {
    F.cur[0] = ldf4(F.slot + ((2 * u) * 64 + lane) * 4);
    F.cur[1] = ldf4(F.slot + ((2 * u + 1) * 64 + lane) * 4);
  }
  static __device__ __forceinline__ void begin(R_t &R, Feed &F) {
    F.slot = R.next();
    load_unit(F, 0, R.lane);
  }
  // Hand out unit U of the current chunk and start reading the next unit.
  template <int U>
  static __device__ __forceinline__ void take(R_t &R, Feed &F, f4 (&a)[2]) {
    a[0] = F.cur[0];
    a[1] = F.cur[1];
    if constexpr (U == kUPC - 1) F.slot = R.next();
#ifndef HF_DIAG_NODS  // timing diagnostic only: results are wrong
    load_unit(F, (U + 1) % kUPC, R.lane);
#endif
  }
  // B operand of flat k-step KS (0..63) of an update layer: k-steps 0..31 read
  // h itself, 32..63 the neighbour mean (h[i+1] + h[i-1]) / 2.  H = CellHalo:
  // a cell-split wave (MT = 1), its boundary neighbours from X's halos.
  template <int MT, int KS, class H>
  static __device__ __forceinline__ void b_operand(const f4 (&h)[MT][kNT], float (&b)[MT], const H &X) {
    constexpr int s = KS % kKS;  // k-step within its 128-wide half
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) b[mt] = h[mt][s >> 2][s & 3];
#ifdef HF_DIAG_NONB  // timing diagnostic only: results are wrong
    if constexpr (false) {
#else
    if constexpr (KS >= kKS) {
#endif
      if constexpr (H::kOn) {
        static_assert(MT == 1, "cell-split waves hold 16 cells");
        b[0] = nb_sum_halo(b[0], X.l[s >> 2][s & 3], X.r[s >> 2][s & 3]);
      } else {
        float sum[MT];
        nb_sum<MT>(b, sum);  // index_add_ of h[i+1], h[i-1]; the / deg 2 is folded into W_b
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) b[mt] = sum[mt];
      }
    }
  }

  // Update-layer k-step KS (unit KS & 3 of its chunk).  b holds this k-step's
  // B operand on entry and the next k-step's on exit: the next operand's lane
  // shifts are interleaved with this k-step's MFMAs instead of stalling the
  // matrix pipe between m-tiles.
  template <int MT, int KS, class H>
  static __device__ __forceinline__ void layer_step(R_t &R, Feed &F, const f4 (&h)[MT][kNT], float (&b)[MT],
                                                    f4 (&acc)[MT][kNT], const H &X) {
    f4 a[2];
    take<KS % kUPC>(R, F, a);
    float bn[MT];
    if constexpr (KS + 1 < 2 * kKS) b_operand<MT, KS + 1>(h, bn, X);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < kNT; ++nt) acc[mt][nt] = mfma4(a[nt >> 2][nt & 3], b[mt], acc[mt][nt]);
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // next unit's ds_reads first
    if constexpr (KS + 1 >= kKS && KS + 1 < 2 * kKS) {
      // one VALU per m-tile for the next operand, after every other MFMA
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, MT * kNT - 2 * MT, 0);
    } else {
      __builtin_amdgcn_sched_group_barrier(0x008, MT * kNT, 0);
    }
    if constexpr (KS + 1 < 2 * kKS) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) b[mt] = bn[mt];
    }
  }
  template <int MT, int KS0, class H>
  static __device__ __forceinline__ void layer_chunk(R_t &R, Feed &F, const f4 (&h)[MT][kNT], float (&b)[MT],
                                                     f4 (&acc)[MT][kNT], const H &X) {
    layer_step<MT, KS0 + 0>(R, F, h, b, acc, X);
    layer_step<MT, KS0 + 1>(R, F, h, b, acc, X);
    layer_step<MT, KS0 + 2>(R, F, h, b, acc, X);
    layer_step<MT, KS0 + 3>(R, F, h, b, acc, X);
  }

  // One readout unit: k-steps s = 16*HH + 4*U + i for P (W_e[:, :H]) and Q (W_e[:, H:]).
  template <int MT, int HH, int U>
  static __device__ __forceinline__ void readout_unit(R_t &R, Feed &F, const f4 (&h)[MT][kNT], f4 (&P)[MT],
                                                      f4 (&Q)[MT]) {
    f4 a[2];
    take<(4 * HH + U) % kUPC>(R, F, a);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int s = 16 * HH + 4 * U + i;
      const float ap = a[i >> 1][2 * (i & 1)], aq = a[i >> 1][2 * (i & 1) + 1];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const float b = h[mt][s >> 2][s & 3];
        P[mt] = mfma4(ap, b, P[mt]);
        Q[mt] = mfma4(aq, b, Q[mt]);
      }
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // next unit's ds_reads first
    __builtin_amdgcn_sched_group_barrier(0x008, 8 * MT, 0);
    // close the unit's region: otherwise the DS group above may be filled with
    // a LATER unit's reads and this unit's prefetch lands just before its use
    __builtin_amdgcn_sched_barrier(0);
  }
  template <int MT, int HH>
  static __device__ __forceinline__ void readout_chunk(R_t &R, Feed &F, const f4 (&h)[MT][kNT], f4 (&P)[MT],
                                                       f4 (&Q)[MT]) {
    readout_unit<MT, HH, 0>(R, F, h, P, Q);
    readout_unit<MT, HH, 1>(R, F, h, P, Q);
    readout_unit<MT, HH, 2>(R, F, h, P, Q);
    readout_unit<MT, HH, 3>(R, F, h, P, Q);
  }

  // Edge readout of a cell-split wave (MT = 1): all 8 output tiles' P and Q
  // first, then column j = 0 of each through LDS (P(i+1), Q(i+1) of lane 15
  // live on the right wave), then the epilogues and partial dots in the same
  // order as gnn_impl's readout, so the fluxes are bit-identical to it.
  static __device__ __forceinline__ void readout_cells(const ChainW &W, const Small &S, R_t &R, Feed &F,
                                                       const f4 (&h)[1][kNT], float (&ffwd)[1], float (&fbwd)[1],
                                                       CellHalo &X) {
    const int lane = R.lane, j = lane & 15, g = lane >> 4, g4 = 4 * g;
    f4 P[kNT][1], Q[kNT][1];
#pragma unroll
    for (int ot = 0; ot < kNT; ++ot) {
      P[ot][0] = ldf4(S.be + 16 * ot + g4);  // b_e as P's initial accumulator
      Q[ot][0] = f4{0.f, 0.f, 0.f, 0.f};
      readout_chunk<1, 0>(R, F, h, P[ot], Q[ot]);
      readout_chunk<1, 1>(R, F, h, P[ot], Q[ot]);
      if (j == 0) {
        X.xq[((X.wave * kNT + ot) * 2 + 0) * 4 + g] = P[ot][0];
        X.xq[((X.wave * kNT + ot) * 2 + 1) * 4 + g] = Q[ot][0];
      }
    }
    lds_barrier();
    float sf = 0.f, sb = 0.f;
#pragma unroll
    for (int w = 0; w < kNT / 2; ++w) {
      float pf = 0.f, pb = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int ot = 2 * w + t;
        const f4 prh = X.xq[((X.rw * kNT + ot) * 2 + 0) * 4 + g];
        const f4 qrh = X.xq[((X.rw * kNT + ot) * 2 + 1) * 4 + g];
        const f4 w2 = ldf4(S.w2 + 16 * ot + g4);
        readout_row_halo<0>(P[ot][0], Q[ot][0], prh, qrh, w2, pf, pb);
        readout_row_halo<1>(P[ot][0], Q[ot][0], prh, qrh, w2, pf, pb);
        readout_row_halo<2>(P[ot][0], Q[ot][0], prh, qrh, w2, pf, pb);
        readout_row_halo<3>(P[ot][0], Q[ot][0], prh, qrh, w2, pf, pb);
      }
      float pf1[1] = {pf}, pb1[1] = {pb}, ff[1], fb[1];
      readout_finish<1>(pf1, pb1, 0.f, ff, fb);
      sf = __fadd_rn(sf, ff[0]);
      sb = __fadd_rn(sb, fb[0]);
    }
    ffwd[0] = __fadd_rn(sf, W.b2);
    fbwd[0] = __fadd_rn(sb, W.b2);
  }

  // FluxGNN forward for the MT*16 cells of this wave.  feat[mt] is the lane's
  // input feature (index l>>4 of [n,u,E,x]) of cell cell_of<MT>(mt, l&15).  Returns
  // the edge fluxes of (i -> i+1) in ffwd and of (i+1 -> i) in fbwd for cell
  // i, on every lane of the cell's column.  Consumes one pass of the stream.
  template <int MT>
  static __device__ __forceinline__ void gnn(const ChainW &W, const Small &S, R_t &R, Feed &F, float * /*park*/,
                                             const float (&feat)[MT], float (&ffwd)[MT], float (&fbwd)[MT]) {
    NoHalo X;
    gnn_impl<MT, NoHalo>(W, S, R, F, feat, ffwd, fbwd, X);
  }
  // A cell-split wave: 16 consecutive cells of an IC spread over several
  // waves (chain_rollout_cells_kernel below), boundary columns exchanged through X.
  static __device__ __forceinline__ void gnn_cells(const ChainW &W, const Small &S, R_t &R, Feed &F,
                                                   const float (&feat)[1], float (&ffwd)[1], float (&fbwd)[1],
                                                   CellHalo &X) {
    gnn_impl<1, CellHalo>(W, S, R, F, feat, ffwd, fbwd, X);
  }

  template <int MT, class H>
  static __device__ __forceinline__ void gnn_impl(const ChainW &W, const Small &S, R_t &R, Feed &F,
                                                  const float (&feat)[MT], float (&ffwd)[MT], float (&fbwd)[MT],
                                                  H &X) {
    const int lane = R.lane;
    const int g4 = 4 * (lane >> 4);
    f4 h[MT][kNT];
    input_layer<MT>(S, lane, feat, h);
    if constexpr (H::kOn) X.exchange(h);

    // message passing: h = ReLU(W_l [h ; (h[i+1]+h[i-1])/2] + b_l)        (src/flux_gnn.py:53-60)
    for (int l = 0; l < W.layers; ++l) {
      // b_l enters every chain as its initial accumulator (the C operand of
      // its first MFMA): no bias add in the epilogue
      f4 acc[MT][kNT];
#pragma unroll
      for (int nt = 0; nt < kNT; ++nt) {
        const f4 bias = ldf4(S.bl + l * kH + 16 * nt + g4);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[mt][nt] = bias;
      }
      float b[MT];
      b_operand<MT, 0>(h, b, X);
      layer_chunk<MT, 0>(R, F, h, b, acc, X);
      layer_chunk<MT, 4>(R, F, h, b, acc, X);
      layer_chunk<MT, 8>(R, F, h, b, acc, X);
      layer_chunk<MT, 12>(R, F, h, b, acc, X);
      layer_chunk<MT, 16>(R, F, h, b, acc, X);
      layer_chunk<MT, 20>(R, F, h, b, acc, X);
      layer_chunk<MT, 24>(R, F, h, b, acc, X);
      layer_chunk<MT, 28>(R, F, h, b, acc, X);
      layer_chunk<MT, 32>(R, F, h, b, acc, X);
      layer_chunk<MT, 36>(R, F, h, b, acc, X);
      layer_chunk<MT, 40>(R, F, h, b, acc, X);
      layer_chunk<MT, 44>(R, F, h, b, acc, X);
      layer_chunk<MT, 48>(R, F, h, b, acc, X);
      layer_chunk<MT, 52>(R, F, h, b, acc, X);
      layer_chunk<MT, 56>(R, F, h, b, acc, X);
      layer_chunk<MT, 60>(R, F, h, b, acc, X);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < kNT; ++nt) h[mt][nt] = relu4(acc[mt][nt]);
      if constexpr (H::kOn) {
        if (l + 1 < W.layers) X.exchange(h);
      }
    }
    if constexpr (H::kOn) {
      readout_cells(W, S, R, F, h, ffwd, fbwd, X);
      return;
    }

    // edge readout, P/Q split (src/flux_gnn.py:62-66).  The 128-feature dot
    // w2 . ReLU(z) is summed as four partial dots over tile pairs (2w, 2w+1),
    // then added in w order; readout_cells keeps the same order, so both
    // rollout kernels give bit-identical results and a batch is invariant to
    // which of them its size selects.
    float sf[MT], sb[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) sf[mt] = sb[mt] = 0.f;
    for (int w = 0; w < kNT / 2; ++w) {
      float pf[MT], pb[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) pf[mt] = pb[mt] = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int ot = 2 * w + t;
        f4 P[MT], Q[MT];
        const f4 be = ldf4(S.be + 16 * ot + g4);  // b_e enters P as the C operand of its first MFMA
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          P[mt] = be;
          Q[mt] = f4{0.f, 0.f, 0.f, 0.f};
        }
        readout_chunk<MT, 0>(R, F, h, P, Q);
        readout_chunk<MT, 1>(R, F, h, P, Q);
        readout_epilogue<MT, true>(P, Q, be, ldf4(S.w2 + 16 * ot + g4), pf, pb);
      }
      float ff[MT], fb[MT];
      readout_finish<MT>(pf, pb, 0.f, ff, fb);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        sf[mt] = __fadd_rn(sf[mt], ff[mt]);
        sb[mt] = __fadd_rn(sb[mt], fb[mt]);
      }
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      ffwd[mt] = __fadd_rn(sf[mt], W.b2);
      fbwd[mt] = __fadd_rn(sb[mt], W.b2);
    }
  }
};

using CoreF32 = CoreF32T<>;

// ---------------------------------------------------------------------------
// Cell-split persistent rollout for small batches: an IC of NX = 16*WPI cells
// on WPI waves (16 consecutive cells each, CoreF32 at MT = 1), 4/WPI ICs per
// workgroup (WPI = 3: one IC and a shadow wave that keeps the weight ring's
// lockstep and writes nothing).  B ICs occupy B*WPI/4 CUs' worth of waves
// instead of B/4, for the same per-cell arithmetic as chain_rollout_kernel:
// every MFMA chain, neighbour sum, readout partial dot and FV/Poisson
// expression is evaluated in the same order, so the results are bit-identical
// to it.  The four waves share the LDS weight ring as in chain_rollout_kernel;
// per layer they swap boundary columns of h (CellHalo), per step column 0 of
// the readout accumulators.  The IC's first wave does FV + Poisson + outputs
// for all its cells, one per lane (src/hybrid_solver.py:45-63).
#ifndef HF_CELLS_AHEAD
#define HF_CELLS_AHEAD 4
#endif
constexpr int kCellsAhead = HF_CELLS_AHEAD;
using CellCore = CoreF32T<kCellsAhead, kCellsAhead + 1>;
constexpr int kXhF4 = 2 * kWaves * 2 * 4 * kNT;  // CellHalo::xh
constexpr int kXqF4 = kWaves * kNT * 2 * 4;      // CellHalo::xq
constexpr int kCellsLds =
    CellCore::kSlots * CellCore::kChunkFloats + kSmallFloats + kWaves * kWaveScratchFloats + 4 * (kXhF4 + kXqF4);

template <int WPI>
__global__ __launch_bounds__(256, 1) void chain_rollout_cells_kernel(
    ChainW W, const float *state0, float *state_final,  // may alias (read whole before written)
    const float *__restrict__ x,
    const double *__restrict__ pc, int B, int T, float c, float dt, float *__restrict__ traj,
    float *__restrict__ flux_traj, float *__restrict__ metrics) {
  constexpr int NX = 16 * WPI;
  constexpr int IPW = kWaves / WPI;  // ICs per workgroup
  constexpr int kRingFloats = CellCore::kSlots * CellCore::kChunkFloats;
  __shared__ f4 lds4[kCellsLds / 4];
  float *lds = reinterpret_cast<float *>(lds4);
  const Small S = stage_small(W, lds + kRingFloats);
  auto R = make_ring<CellCore>(W, lds);
  const int wave = R.wave, lane = R.lane, j = lane & 15, g = lane >> 4;
  const bool shadow = wave >= IPW * WPI;
  const int slot = shadow ? 0 : wave / WPI;  // IC of this wave within the workgroup
  const int pos = shadow ? 0 : wave % WPI;   // cells 16*pos .. 16*pos + 15 of it
  const bool lead = !shadow && pos == 0;
  CellHalo X;
  X.xh = reinterpret_cast<f4 *>(lds + kRingFloats + kSmallFloats + kWaves * kWaveScratchFloats);
  X.xq = X.xh + kXhF4;
  X.wave = wave;
  X.lane = lane;
  X.par = 0;
  X.lw = shadow ? wave : slot * WPI + (pos + WPI - 1) % WPI;  // periodic chain
  X.rw = shadow ? wave : slot * WPI + (pos + 1) % WPI;
  float *scratch = lds + kRingFloats + kSmallFloats + slot * kWaveScratchFloats;
  float *s_st = scratch;  // n | u | E | x   (4 x 64)
  float *s_F = scratch + 4 * 64;
  float *s_rho = scratch + 5 * 64;
  double *s_c = reinterpret_cast<double *>(scratch + 6 * 64);
  const int b_raw = blockIdx.x * IPW + slot;
  const bool live = b_raw < B;
  const int64_t b = live ? b_raw : B - 1;  // a missing IC mirrors the last one and writes nothing
  if (lead) {
    const float *st0 = state0 + b * 3 * NX;
    for (int i = lane; i < 3 * NX; i += 64) s_st[(i / NX) * 64 + i % NX] = st0[i];
    if (lane < NX) {
      s_st[3 * 64 + lane] = x[lane];
      s_c[lane] = pc[lane];
    }
  }
  __syncthreads();  // small weights + IC state visible (no DMA in flight yet)
  const bool out = lead && live;
  float *tj = (traj && out) ? traj + b * (int64_t)(T + 1) * 3 * NX : nullptr;
  float *mt_out = (metrics && out) ? metrics + b * (int64_t)(T + 1) * HF_NUM_METRICS : nullptr;
  float *ftj = (flux_traj && out) ? flux_traj + b * (int64_t)T * NX : nullptr;
  auto emit = [&](int t) {  // lead wave
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
  if (lead) emit(0);
  R.prime();
  CellCore::Feed F;
  CellCore::begin(R, F);
  for (int t = 0; t < T; ++t) {
    const float feat[1] = {s_st[g * 64 + 16 * pos + j]};
    float ff[1], fb[1];
    CellCore::gnn_cells(W, S, R, F, feat, ff, fb, X);
    if (!shadow && g == 0) s_F[16 * pos + j] = face_flux(ff[0], fb[0]);
    lds_barrier();  // every wave's face fluxes in s_F
#ifdef HF_DIAG_NOFV  // timing diagnostic only: results are wrong (no FV, Poisson or outputs per step)
    if (false) {
#else
    if (lead) {     // src/hybrid_solver.py:45-63, one cell per lane
#endif
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
  R.drain();
  if (!out) return;
  float *dst = state_final + b * 3 * NX;
  for (int i = lane; i < 3 * NX; i += 64) dst[i] = s_st[(i / NX) * 64 + i % NX];
}

// FluxGNN.forward on B chains of 16*WPI cells, cell-split as above (the
// small-batch counterpart of chain_flux_kernel<CoreF32, MT, true>, bit-identical to it).
template <int WPI>
__global__ __launch_bounds__(256, 1) void chain_flux_cells_kernel(ChainW W, const float *__restrict__ nf,
                                                                  const float *__restrict__ state, int64_t ld_state,
                                                                  const float *__restrict__ x, int B,
                                                                  float *__restrict__ fe, float *__restrict__ ff) {
  constexpr int NX = 16 * WPI;
  constexpr int IPW = kWaves / WPI;
  constexpr int kRingFloats = CellCore::kSlots * CellCore::kChunkFloats;
  __shared__ f4 lds4[kCellsLds / 4];
  float *lds = reinterpret_cast<float *>(lds4);
  const Small S = stage_small(W, lds + kRingFloats);
  auto R = make_ring<CellCore>(W, lds);
  const int wave = R.wave, lane = R.lane, j = lane & 15, g = lane >> 4;
  const bool shadow = wave >= IPW * WPI;
  const int slot = shadow ? 0 : wave / WPI, pos = shadow ? 0 : wave % WPI;
  CellHalo X;
  X.xh = reinterpret_cast<f4 *>(lds + kRingFloats + kSmallFloats + kWaves * kWaveScratchFloats);
  X.xq = X.xh + kXhF4;
  X.wave = wave;
  X.lane = lane;
  X.par = 0;
  X.lw = shadow ? wave : slot * WPI + (pos + WPI - 1) % WPI;
  X.rw = shadow ? wave : slot * WPI + (pos + 1) % WPI;
  const int b_raw = blockIdx.x * IPW + slot;
  const bool out = !shadow && b_raw < B;
  const int64_t b = b_raw < B ? b_raw : B - 1;
  const int cell = 16 * pos + j;
  const float feat[1] = {nf ? nf[(b * NX + cell) * kIn + g]
                            : (g < 3 ? state[b * ld_state + (int64_t)g * NX + cell] : x[cell])};
  __syncthreads();  // small weights staged (no DMA in flight yet)
  R.prime();
  CellCore::Feed F;
  CellCore::begin(R, F);
  float f_fwd[1], f_bwd[1];
  CellCore::gnn_cells(W, S, R, F, feat, f_fwd, f_bwd, X);
  R.drain();
  if (!out) return;
  if (fe && g == 0) fe[b * 2 * NX + cell] = f_fwd[0];
  if (fe && g == 1) fe[b * 2 * NX + NX + cell] = f_bwd[0];
  if (ff && g == 2) ff[b * NX + cell] = face_flux(f_fwd[0], f_bwd[0]);
}

template <int WPI>
hipError_t flux_cells_launch(const ChainW &w, const float *nf, const float *state, int64_t ld_state, const float *x,
                             int B, float *fe, float *ff, hipStream_t s) {
  constexpr int IPW = kWaves / WPI;
  hipLaunchKernelGGL((chain_flux_cells_kernel<WPI>), dim3((B + IPW - 1) / IPW), dim3(64 * kWaves), 0, s, w, nf,
                     state, ld_state, x, B, fe, ff);
  return hipGetLastError();
}

template <int WPI>
hipError_t cells_launch(const ChainW &w, const float *state0, float *state_final, const float *x, const double *pc,
                        int B, int T, float c, float dt, float *traj, float *flux_traj, float *metrics,
                        hipStream_t s) {
  constexpr int IPW = kWaves / WPI;
  hipLaunchKernelGGL((chain_rollout_cells_kernel<WPI>), dim3((B + IPW - 1) / IPW), dim3(64 * kWaves), 0, s, w,
                     state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics);
  return hipGetLastError();
}

}  // namespace

// Whether the cell-split kernel beats the IC-per-wave kernel for B ICs of nx
// cells: its workgroups carry 4/WPI ICs at about 1/WPI of the IC-per-wave
// kernel's time per step (plus the exchanges), against 4 ICs per workgroup.
bool chain_rollout_prefers_cells(const ChainW &w, int B, int nx) {
  if (w.prec != kPrecF32 || B <= 0 || (nx != 32 && nx != 48 && nx != 64)) return false;
  const int wpi = nx / 16, ipw = kWaves / wpi;
  const int64_t cus = chain::resident_groups();
  const int64_t wave_rounds = ((int64_t)B + 4 * cus - 1) / (4 * cus);
  const int64_t cell_rounds = ((int64_t)B + ipw * cus - 1) / (ipw * cus);
  return cell_rounds * (100 + 15 * wpi) < wave_rounds * 100 * wpi;
}

hipError_t launch_chain_rollout_cells(const ChainW &w, const float *state0, float *state_final, const float *x,
                                      const double *pc, int B, int nx, int T, float c, float dt, float *traj,
                                      float *flux_traj, float *metrics, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  switch (nx) {
    case 32: return cells_launch<2>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, s);
    case 48: return cells_launch<3>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, s);
    case 64: return cells_launch<4>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_chain_flux_f32(const ChainW &w, const float *nf, const float *state, int64_t ld_state,
                                 const float *x, int B, int nx, float *fe, float *ff, hipStream_t s) {
  // small batches: each chain spread over nx/16 waves, as the rollout
  if (chain_rollout_prefers_cells(w, B, nx)) {
    switch (nx) {
      case 32: return flux_cells_launch<2>(w, nf, state, ld_state, x, B, fe, ff, s);
      case 48: return flux_cells_launch<3>(w, nf, state, ld_state, x, B, fe, ff, s);
      case 64: return flux_cells_launch<4>(w, nf, state, ld_state, x, B, fe, ff, s);
      default: break;
    }
  }
  return chain::launch_flux_core<CoreF32>(w, nf, state, ld_state, x, B, nx, fe, ff, s);
}

hipError_t launch_chain_rollout_f32(const ChainW &w, const float *state0, float *state_final, const float *x,
                                    const double *pc, int B, int nx, int T, float c, float dt, float *traj,
                                    float *flux_traj, float *metrics, const RolloutExtras &ex, hipStream_t s) {
  // small batches: each IC spread over nx/16 waves (cell-split kernel)
  if (ex.mse == nullptr && ex.metrics_cl == nullptr && chain_rollout_prefers_cells(w, B, nx))
    return launch_chain_rollout_cells(w, state0, state_final, x, pc, B, nx, T, c, dt, traj, flux_traj, metrics, s);
  return chain::launch_rollout_core<CoreF32>(w, state0, state_final, x, pc, B, nx, T, c, dt, traj, flux_traj,
                                             metrics, ex, s);
}

}  // namespace hf
