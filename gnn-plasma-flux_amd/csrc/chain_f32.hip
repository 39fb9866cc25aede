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
template <int D = 2, int SLOTS = kRingSlots, bool LDR = false, bool DEF = false>
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
  // barrier schedule of one cell-split pass (the loader wave's,
  // chain_rollout_cells_kernel): 16 ring chunks per update layer, no other barrier
  static constexpr int kLayerChunks = 16;
  static constexpr bool kLayerBarrier = false;
  // LDR: a loader wave issues the ring DMA; DEF: each wave's DMA for chunk p+D
  // is issued after unit 0's fragment reads of chunk p, not at the barrier
  using R_t = Ring<kChunkFloats, kNW, kSlots, kAhead, DEF, LDR>;

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
    load_unit(F, 0, R.lane);  // (DEF: the DMA this next() owes goes out in take<0>)
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
#ifndef HF_F32_DEFU
#define HF_F32_DEFU 0
#endif
    // after unit DEFU+1's fragment reads of the new chunk (A/B: HF_F32_DEFU 0..2)
    if constexpr (DEF && U == HF_F32_DEFU) R.issue_pending();
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
      if constexpr (H::kSecond) {  // the readout's backward: [dP ; dQ], no neighbour sum
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) b[mt] = X.q[mt][s >> 2][s & 3];
      } else if constexpr (H::kOn) {
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
  // TP (a TileStore): tile KS/2 of h goes to array tl (tl >= 0) after k-step KS
  // (odd KS), so a pass stores its B operand spread over its first 2*MT*kNT k-steps.
  template <int MT, int KS, class H, class TP = NoTape>
  static __device__ __forceinline__ void layer_step(R_t &R, Feed &F, const f4 (&h)[MT][kNT], float (&b)[MT],
                                                    f4 (&acc)[MT][kNT], H &X, const TP &T = TP{}, int tl = -1) {
    f4 a[2];
    take<KS % kUPC>(R, F, a);
    if constexpr (H::kOn && KS == kUPC) X.read();  // the ring barrier of take<kUPC-1> follows every publish
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
    if constexpr (TP::kOn && KS % 2 == 1 && KS / 2 < MT * kNT) {
      if (tl >= 0) T.template put_tile<MT, KS / 2>(tl, h, R.lane);
    }
  }
  template <int MT, int KS0, class H, class TP = NoTape>
  static __device__ __forceinline__ void layer_chunk(R_t &R, Feed &F, const f4 (&h)[MT][kNT], float (&b)[MT],
                                                     f4 (&acc)[MT][kNT], H &X, const TP &T = TP{}, int tl = -1) {
    layer_step<MT, KS0 + 0>(R, F, h, b, acc, X, T, tl);
    layer_step<MT, KS0 + 1>(R, F, h, b, acc, X, T, tl);
    layer_step<MT, KS0 + 2>(R, F, h, b, acc, X, T, tl);
    layer_step<MT, KS0 + 3>(R, F, h, b, acc, X, T, tl);
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

  // Edge readout of a cell-split wave (MT = 1), pipelined tile by tile: tile
  // ot's column j = 0 of P and Q is published through LDS after its MFMAs
  // (P(i+1), Q(i+1) of lane 15 live on the right wave), read after the ring
  // barrier that ends tile ot+1's first chunk, and tile ot's epilogue runs
  // under tile ot+1's second chunk; only the last tile needs a barrier of its
  // own.  Epilogues and partial dots run in gnn_impl's readout order, so the
  // fluxes are bit-identical to it.
  static __device__ __forceinline__ void readout_cells(const ChainW &W, const Small &S, R_t &R, Feed &F,
                                                       const f4 (&h)[1][kNT], float (&ffwd)[1], float (&fbwd)[1],
                                                       CellHalo &X) {
    const int lane = R.lane, j = lane & 15, g = lane >> 4, g4 = 4 * g;
    float pf = 0.f, pb = 0.f, sf = 0.f, sb = 0.f;
    // epilogue of tile ot (after the barrier that follows its publish); a tile
    // pair's partial dots are summed across the lane groups after its second tile
    auto epilogue = [&](int ot, const f4 &P, const f4 &Q) {
      const f4 prh = X.xq[((X.rw * kNT + ot) * 2 + 0) * 4 + g];
      const f4 qrh = X.xq[((X.rw * kNT + ot) * 2 + 1) * 4 + g];
      const f4 w2 = ldf4(S.w2 + 16 * ot + g4);
      readout_row_halo<0>(P, Q, prh, qrh, w2, pf, pb);
      readout_row_halo<1>(P, Q, prh, qrh, w2, pf, pb);
      readout_row_halo<2>(P, Q, prh, qrh, w2, pf, pb);
      readout_row_halo<3>(P, Q, prh, qrh, w2, pf, pb);
      if (ot & 1) {
        float pf1[1] = {pf}, pb1[1] = {pb}, ff[1], fb[1];
        readout_finish<1>(pf1, pb1, 0.f, ff, fb);
        sf = __fadd_rn(sf, ff[0]);
        sb = __fadd_rn(sb, fb[0]);
        pf = pb = 0.f;
      }
    };
    f4 Pp, Qp;  // the previous tile's accumulators
#pragma unroll
    for (int ot = 0; ot < kNT; ++ot) {
      f4 P[1], Q[1];
      P[0] = ldf4(S.be + 16 * ot + g4);  // b_e as P's initial accumulator
      Q[0] = f4{0.f, 0.f, 0.f, 0.f};
      readout_chunk<1, 0>(R, F, h, P, Q);  // ends with the ring barrier
      if (ot > 0) epilogue(ot - 1, Pp, Qp);
      readout_chunk<1, 1>(R, F, h, P, Q);
      if (j == 0) {
        X.xq[((X.wave * kNT + ot) * 2 + 0) * 4 + g] = P[0];
        X.xq[((X.wave * kNT + ot) * 2 + 1) * 4 + g] = Q[0];
      }
      Pp = P[0];
      Qp = Q[0];
    }
    lds_barrier();
    epilogue(kNT - 1, Pp, Qp);
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
    gnn_impl<MT, NoHalo>(W, S, R, F, feat, ffwd, fbwd, X, NoTape{});
  }
  // The same pass storing the activation tape (chain_train_fwd_kernel).
  template <int MT>
  static __device__ __forceinline__ void gnn_tape(const ChainW &W, const Small &S, R_t &R, Feed &F,
                                                  const float (&feat)[MT], float (&ffwd)[MT], float (&fbwd)[MT],
                                                  const TrainTape &T) {
    NoHalo X;
    gnn_impl<MT, NoHalo>(W, S, R, F, feat, ffwd, fbwd, X, T);
  }
  // A cell-split wave: 16 consecutive cells of an IC spread over several
  // waves (chain_rollout_cells_kernel below), boundary columns exchanged through X.
  static __device__ __forceinline__ void gnn_cells(const ChainW &W, const Small &S, R_t &R, Feed &F,
                                                   const float (&feat)[1], float (&ffwd)[1], float (&fbwd)[1],
                                                   CellHalo &X) {
    gnn_impl<1, CellHalo>(W, S, R, F, feat, ffwd, fbwd, X, NoTape{});
  }

  template <int MT, class H, class TP>
  static __device__ __forceinline__ void gnn_impl(const ChainW &W, const Small &S, R_t &R, Feed &F,
                                                  const float (&feat)[MT], float (&ffwd)[MT], float (&fbwd)[MT],
                                                  H &X, const TP &T) {
    const int lane = R.lane;
    const int g4 = 4 * (lane >> 4);
    f4 h[MT][kNT];
    input_layer<MT>(S, lane, feat, h);
    if constexpr (TP::kOn) T.template put_mask<MT>(0, h, lane);
    // cell-split waves: the boundary columns are published here and read
    // after the ring barrier that ends the next layer's first chunk
    // (layer_step<4>), long before the first neighbour-sum k-step (32)
    if constexpr (H::kOn) X.publish(h);

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
      layer_chunk<MT, 0>(R, F, h, b, acc, X, T, l);
      layer_chunk<MT, 4>(R, F, h, b, acc, X, T, l);
      layer_chunk<MT, 8>(R, F, h, b, acc, X, T, l);
      layer_chunk<MT, 12>(R, F, h, b, acc, X, T, l);
      layer_chunk<MT, 16>(R, F, h, b, acc, X, T, l);
      layer_chunk<MT, 20>(R, F, h, b, acc, X, T, l);
      layer_chunk<MT, 24>(R, F, h, b, acc, X, T, l);
      layer_chunk<MT, 28>(R, F, h, b, acc, X, T, l);
      layer_chunk<MT, 32>(R, F, h, b, acc, X, T, l);
      layer_chunk<MT, 36>(R, F, h, b, acc, X, T, l);
      layer_chunk<MT, 40>(R, F, h, b, acc, X, T, l);
      layer_chunk<MT, 44>(R, F, h, b, acc, X, T, l);
      layer_chunk<MT, 48>(R, F, h, b, acc, X, T, l);
      layer_chunk<MT, 52>(R, F, h, b, acc, X, T, l);
      layer_chunk<MT, 56>(R, F, h, b, acc, X, T, l);
      layer_chunk<MT, 60>(R, F, h, b, acc, X, T, l);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < kNT; ++nt) h[mt][nt] = relu4(acc[mt][nt]);
      if constexpr (TP::kOn) T.template put_mask<MT>(l + 1, h, lane);
      if constexpr (H::kOn) {
        if (l + 1 < W.layers) X.publish(h);
      }
    }
    if constexpr (H::kOn) {
      readout_cells(W, S, R, F, h, ffwd, fbwd, X);
      return;
    }

    if constexpr (TP::kOn) T.template put_all<MT>(W.layers, h, lane);  // h[L] (one burst)
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
        if constexpr (TP::kOn) T.template put_pq<MT>(ot, P, Q, lane);
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

#ifndef HF_F32_DEFER
#define HF_F32_DEFER 1
#endif
using CoreF32 = CoreF32T<2, kRingSlots, false, HF_F32_DEFER != 0>;

// ---------------------------------------------------------------------------
// Cell-split small-batch kernels (chain_common.h) on the f32 core at MT = 1.
#ifndef HF_CELLS_AHEAD
#define HF_CELLS_AHEAD 4
#endif
constexpr int kCellsAhead = HF_CELLS_AHEAD;
// The cell-split kernels' core: a fifth (loader) wave issues the weight
// ring's DMA, so the four compute waves carry none (chain_common.h Ring
// LOADER).  HF_CELLS_LOADER=0 builds the four-wave form (A/B).
#ifndef HF_CELLS_LOADER
#define HF_CELLS_LOADER 1
#endif
using CellCoreLd = CoreF32T<kCellsAhead, kCellsAhead + 1, HF_CELLS_LOADER != 0>;
}  // namespace

// Whether the cell-split kernel beats the IC-per-wave kernel for B ICs of nx
// cells: its workgroups carry 4/WPI ICs at about 1/WPI of the IC-per-wave
// kernel's time per step (plus the exchanges), against 4 ICs per workgroup.
bool chain_rollout_prefers_cells(const ChainW &w, int B, int nx) {
  if (B <= 0 || (nx != 32 && nx != 48 && nx != 64)) return false;  // every precision has a cell-split core
  const int wpi = nx / 16, ipw = kWaves / wpi;
  const int64_t cus = chain::resident_groups();
  const int64_t wave_rounds = ((int64_t)B + 4 * cus - 1) / (4 * cus);
  const int64_t cell_rounds = ((int64_t)B + ipw * cus - 1) / (ipw * cus);
  return cell_rounds * (100 + 15 * wpi) < wave_rounds * 100 * wpi;
}

hipError_t launch_chain_rollout_cells(const ChainW &w, const float *state0, float *state_final, const float *x,
                                      const double *pc, int B, int nx, int T, float c, float dt, float *traj,
                                      float *flux_traj, float *metrics, int pm, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  switch (nx) {
    case 32: return cells_launch<CellCoreLd, 2>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, pm, s);
    case 48: return cells_launch<CellCoreLd, 3>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, pm, s);
    case 64: return cells_launch<CellCoreLd, 4>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, pm, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_chain_flux_f32(const ChainW &w, const float *nf, const float *state, int64_t ld_state,
                                 const float *x, int B, int nx, float *fe, float *ff, hipStream_t s) {
  // small batches: each chain spread over nx/16 waves, as the rollout
  if (chain_rollout_prefers_cells(w, B, nx)) {
    switch (nx) {
      case 32: return flux_cells_launch<CellCoreLd, 2>(w, nf, state, ld_state, x, B, fe, ff, s);
      case 48: return flux_cells_launch<CellCoreLd, 3>(w, nf, state, ld_state, x, B, fe, ff, s);
      case 64: return flux_cells_launch<CellCoreLd, 4>(w, nf, state, ld_state, x, B, fe, ff, s);
      default: break;
    }
  }
  return chain::launch_flux_core<CoreF32>(w, nf, state, ld_state, x, B, nx, fe, ff, s);
}

// ---------------------------------------------------------------------------
// Fused training forward (train_chain.hip launch_chain_forward_train at
// nx in {16, 32, 48, 64}, FluxGNN(4, 128, L <= 8)).
namespace {
__device__ __forceinline__ int kperm_dev(int s, int lane) { return 16 * (s >> 2) + 4 * (lane >> 4) + (s & 3); }

// The f32 chain stream and small arrays of capi.cpp pack_chain (kPrecF32),
// built on the device from state-dict-ordered parameters (GraphW view): the
// optimizer changes them every step, so the host pack is no option.  One
// thread per packed float: the stream's nstream floats, then the small arrays
// (win [2][64][4], b_in, b_l[L], b_e, w2).
__device__ __forceinline__ void pack_chain_f32_at(const GraphW &w, float *__restrict__ stream, int64_t nstream,
                                                  float *__restrict__ small, int64_t idx) {
  const int L = w.layers;
  if (idx < nstream) {
    const int c = (int)(idx >> 11), rem = (int)(idx & 2047), j = rem >> 8, lane = (rem >> 2) & 63, cc = rem & 3;
    float v;
    if (c < 16 * L) {  // update layer l, chunk gi: k-step s, output tile nt
      const int l = c >> 4, s = 4 * (c & 15) + (j >> 1), nt = 4 * (j & 1) + cc;
      const int k = (s < kKS ? 0 : kH) + kperm_dev(s % kKS, lane);
      v = w.w_l[l * w.lsw + (int64_t)(16 * nt + (lane & 15)) * 2 * kH + k];
      if (s >= kKS) v *= 0.5f;  // the mean's 1/deg folded into W_b (exact)
    } else {  // readout tile ot, half hh: P (cc even) / Q (odd) of k-step s
      const int r = c - 16 * L, ot = r >> 1, s = 16 * (r & 1) + 2 * j + (cc >> 1);
      v = w.w_e[(int64_t)(16 * ot + (lane & 15)) * 2 * kH + (cc & 1) * kH + kperm_dev(s, lane)];
    }
    stream[idx] = v;
    return;
  }
  const int i = (int)(idx - nstream);
  if (i >= 512 + kH * (3 + L)) return;
  float v;
  if (i < 512) {
    const int lane = (i >> 2) & 63, nt = 4 * (i >> 8) + (i & 3);
    v = w.w_in[(16 * nt + (lane & 15)) * kIn + (lane >> 4)];
  } else if (i < 512 + kH) {
    v = w.b_in[i - 512];
  } else if (i < 512 + kH * (1 + L)) {
    const int o = i - 512 - kH;
    v = w.b_l[(o / kH) * w.lsb + o % kH];
  } else if (i < 512 + kH * (2 + L)) {
    v = w.b_e[i - 512 - kH * (1 + L)];
  } else {
    v = w.w_2[i - 512 - kH * (2 + L)];
  }
  small[i] = v;
}
__global__ void pack_chain_f32_kernel(GraphW w, float *__restrict__ stream, int64_t nstream, float *__restrict__ small) {
  pack_chain_f32_at(w, stream, nstream, small, (int64_t)blockIdx.x * 256 + threadIdx.x);
}

// The update layers' transposed weights for chain_train_bwd_kernel, in the
// f32 stream format, layers L-1 .. 0: A(n, k) = W_l[k][n] (k < H: W_a^T) or
// W_l[k - H][H + n] / 2 (W_b^T with the mean's 1/deg).
// ro: the readout's [W_a^T | W_b^T] of edge_mlp.0 first (16 chunks, no 1/deg).
__device__ __forceinline__ void pack_chain_bwd_f32_at(const GraphW &w, float *__restrict__ stream, int64_t nstream,
                                                      int ro, int64_t idx) {
  if (idx >= nstream) return;
  const int c = (int)(idx >> 11), rem = (int)(idx & 2047), j = rem >> 8, lane = (rem >> 2) & 63, cc = rem & 3;
  const bool readout = ro && c < 16;
  const int l = w.layers - 1 - ((c - (ro ? 16 : 0)) >> 4), s = 4 * (c & 15) + (j >> 1);
  const int n = 16 * (4 * (j & 1) + cc) + (lane & 15), k = kperm_dev(s % kKS, lane);
  const float *W = readout ? w.w_e : w.w_l + l * w.lsw;
  const float half = readout ? 1.f : 0.5f;
  stream[idx] = s < kKS ? W[(int64_t)k * 2 * kH + n] : half * W[(int64_t)k * 2 * kH + kH + n];
}
__global__ void pack_chain_bwd_f32_kernel(GraphW w, float *__restrict__ stream, int64_t nstream, int ro) {
  pack_chain_bwd_f32_at(w, stream, nstream, ro, (int64_t)blockIdx.x * 256 + threadIdx.x);
}
// Both packs in one launch (the training forward packs the backward's
// transposed stream too: the parameters do not change between the two passes
// of a step): threads [0, ftotal) the forward's, then the backward's.
__global__ void pack_chain_train_f32_kernel(GraphW w, float *__restrict__ stream, int64_t nstream,
                                            float *__restrict__ small, int64_t ftotal, float *__restrict__ bstream,
                                            int64_t nbstream, int ro) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx < ftotal) pack_chain_f32_at(w, stream, nstream, small, idx);
  else pack_chain_bwd_f32_at(w, bstream, nbstream, ro, idx - ftotal);
}

template <int MT>
int64_t train_blocks(int64_t B) {
  const int64_t groups = (B + CoreF32::kNW - 1) / CoreF32::kNW;
  const int64_t res = (int64_t)resident_groups() * CoreF32::kWGPerCU;
  return groups < res ? groups : res;
}
template <int MT>
hipError_t train_fwd_launch(const ChainW &cw, const float *b2p, const float *nf, int64_t B, float *fe, float *h0,
                            int64_t hstride, float *pq, unsigned *mbits, hipStream_t s) {
  hipLaunchKernelGGL((chain_train_fwd_kernel<CoreF32, MT>), dim3((unsigned)train_blocks<MT>(B)),
                     dim3(64 * CoreF32::kNW), 0, s, cw, b2p, nf, B, fe, h0, hstride, pq, mbits);
  return hipGetLastError();
}
template <int MT>
hipError_t train_bwd_launch(const ChainW &cw, int64_t B, float *g0, int64_t gstride, const unsigned *mbits,
                            const float *dPQ, const EdgeFold &ef, hipStream_t s) {
  hipLaunchKernelGGL((chain_train_bwd_kernel<CoreF32, MT>), dim3((unsigned)train_blocks<MT>(B)),
                     dim3(64 * CoreF32::kNW), 0, s, cw, B, g0, gstride, mbits, dPQ, ef);
  return hipGetLastError();
}
}  // namespace

int64_t chain_train_pack_bytes(int layers) {
  return (int64_t)chain_chunks(layers, kPrecF32) * chain_chunk_bytes(kPrecF32) +
         (int64_t)sizeof(float) * (512 + kH * (3 + layers));
}
int64_t chain_train_mask_bytes(int layers, int64_t N) { return (int64_t)(layers + 1) * N * 16; }
int64_t chain_train_bwd_pack_bytes(int layers) { return (int64_t)16 * (layers + 1) * chain_chunk_bytes(kPrecF32); }

hipError_t launch_chain_train_bwd_fused(const GraphW &w, int64_t B, int nx, float *g0, int64_t gstride,
                                        const unsigned *mbits, void *pack, const float *dPQ, hipStream_t s,
                                        const float *pq, const float *gflux, const float *w2, float *epart,
                                        bool prepacked) {
  // pq != nullptr: the readout's backward from the P/Q tape in this pass (EdgeFold), writing dPQ
  const EdgeFold ef{pq, gflux, w2, const_cast<float *>(dPQ), epart};
  const int L = w.layers;
  if (B <= 0 || (L == 0 && !dPQ)) return hipSuccess;
  float *stream = static_cast<float *>(pack);
  const int64_t nstream = (int64_t)16 * (L + (dPQ ? 1 : 0)) * 2048;
  if (!prepacked)
    hipLaunchKernelGGL(pack_chain_bwd_f32_kernel, dim3((unsigned)(nstream / 256)), dim3(256), 0, s, w, stream, nstream,
                       dPQ ? 1 : 0);
  ChainW cw{};
  cw.stream = stream;
  cw.layers = L;
  cw.prec = kPrecF32;
  switch (nx) {
    case 16: return train_bwd_launch<1>(cw, B, g0, gstride, mbits, dPQ, ef, s);
    case 32: return train_bwd_launch<2>(cw, B, g0, gstride, mbits, dPQ, ef, s);
    case 48: return train_bwd_launch<3>(cw, B, g0, gstride, mbits, dPQ, ef, s);
    case 64: return train_bwd_launch<4>(cw, B, g0, gstride, mbits, dPQ, ef, s);
    default: return hipErrorInvalidValue;
  }
}

bool chain_train_fused_ok(const GraphW &w, int nx) {
  return w.in_dim == kIn && w.hidden == kH && w.layers >= 0 && w.layers <= kMaxChainLayers &&
         (nx == 16 || nx == 32 || nx == 48 || nx == 64);
}

hipError_t launch_chain_train_fwd_fused(const GraphW &w, const float *nf, int64_t B, int nx, float *fe, float *h0,
                                        int64_t hstride, float *pq, unsigned *mbits, void *pack, hipStream_t s,
                                        void *bpack, int ro) {
  if (B <= 0) return hipSuccess;
  const int L = w.layers;
  float *stream = static_cast<float *>(pack);
  const int64_t nstream = (int64_t)chain_chunks(L, kPrecF32) * chain_chunk_bytes(kPrecF32) / 4;
  float *small = stream + nstream;
  const int64_t total = nstream + 512 + kH * (3 + L);
  if (bpack) {  // + the backward's stream (launch_chain_train_bwd_fused with prepacked)
    const int64_t nb = (int64_t)16 * (L + (ro ? 1 : 0)) * 2048;
    hipLaunchKernelGGL(pack_chain_train_f32_kernel, dim3((unsigned)((total + nb + 255) / 256)), dim3(256), 0, s, w,
                       stream, nstream, small, total, static_cast<float *>(bpack), nb, ro);
  } else {
    hipLaunchKernelGGL(pack_chain_f32_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, w, stream,
                       nstream, small);
  }
  ChainW cw{};
  cw.stream = stream;
  cw.win = small;
  cw.bin = small + 512;
  cw.bl = small + 512 + kH;
  cw.be = small + 512 + kH * (1 + L);
  cw.w2 = small + 512 + kH * (2 + L);
  cw.b2 = 0.f;  // read from w.b_2 on the device
  cw.layers = L;
  cw.prec = kPrecF32;
  switch (nx) {
    case 16: return train_fwd_launch<1>(cw, w.b_2, nf, B, fe, h0, hstride, pq, mbits, s);
    case 32: return train_fwd_launch<2>(cw, w.b_2, nf, B, fe, h0, hstride, pq, mbits, s);
    case 48: return train_fwd_launch<3>(cw, w.b_2, nf, B, fe, h0, hstride, pq, mbits, s);
    case 64: return train_fwd_launch<4>(cw, w.b_2, nf, B, fe, h0, hstride, pq, mbits, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_chain_rollout_f32(const ChainW &w, const float *state0, float *state_final, const float *x,
                                    const double *pc, int B, int nx, int T, float c, float dt, float *traj,
                                    float *flux_traj, float *metrics, const RolloutExtras &ex, hipStream_t s) {
  // small batches: each IC spread over nx/16 waves (cell-split kernel)
  if (ex.mse == nullptr && ex.metrics_cl == nullptr && chain_rollout_prefers_cells(w, B, nx))
    return launch_chain_rollout_cells(w, state0, state_final, x, pc, B, nx, T, c, dt, traj, flux_traj, metrics,
                                      ex.poisson, s);
  return chain::launch_rollout_core<CoreF32>(w, state0, state_final, x, pc, B, nx, T, c, dt, traj, flux_traj,
                                             metrics, ex, s);
}

}  // namespace hf
