// Fused FluxGNN on the periodic chain, fp32-accurate on the fp16 matrix
// cores (precision "f16x3"): v_mfma_f32_16x16x32_f16.  bf16 is chain_bf16.hip.
//
// Reference: src/flux_gnn.py:40-67, src/hybrid_solver.py:34-73.
//
// F16x3 keeps float32-level accuracy at ~5x the f32 MFMA rate: every weight
// and every activation is split into two fp16 terms, x = x_hi + x_lo with
// x_hi = fp16(x), x_lo = fp16(x - x_hi) (22 significant bits), and each
// product is accumulated in f32 as a_lo b_hi + a_hi b_lo + a_hi b_hi (the
// dropped a_lo b_lo is 2^-22 relative).  Measured against an fp64 evaluation
// the edge fluxes carry 5.4e-7 error, the same as the reference's own float32
// CPU evaluation (4.7e-7).
//
// Fragments: for 16x16x32, lane l holds A[row l&15][k = 8(l>>4) + e] and
// B[k = 8(l>>4) + e][col l&15], e = 0..7.  The B fragment of k-block kb is the
// two 16x16 accumulator tiles 2kb, 2kb+1 of the previous layer (features
// 16(2kb + (e>>2)) + 4(l>>4) + (e&3)): the activations never leave registers
// and the host packs the weights in the same permuted k order.
//
// Aggregation by linearity: W_b (h[i+1] + h[i-1]) / 2 = (G[i+1] + G[i-1]) / 2
// with G = W_b h, so the split activations of a k-block feed both W_a and W_b
// (the split fragments are twice the size of bf16's, so no second set of
// neighbour-sum fragments) and the neighbour lane shifts run on the G
// accumulators.
//
// Schedule (as the bf16 core): a layer is walked in output-pair order (pair q
// = tiles 2q, 2q+1 = the next layer's k-block q, 4 units of 48 MFMAs at MT=4),
// the epilogue of pair q-1 (neighbour sums of G, ReLU, fp16 hi/lo split) is
// spread over pair q's units, the new fragments of pairs 0..2 are parked in
// LDS, and pair 3's epilogue runs under the next layer's first three k-blocks
// (or the first readout tile).  Every value is formed by the same operations
// in the same order as a whole-layer epilogue would.
#include "chain_common.h"

namespace hf {
namespace {

using namespace chain;

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

// the two fp16 terms of one value pair: hi = fp16(v), lo = fp16(v - hi) (exact difference)
struct Split {
  unsigned hi, lo;
};
__device__ __forceinline__ Split split_pair(float a, float b) {
  const h2 h = __builtin_convertvector(f2{a, b}, h2);
  const f2 back = __builtin_convertvector(h, f2);
  return {__builtin_bit_cast(unsigned, h), __builtin_bit_cast(unsigned, __builtin_convertvector(f2{a, b} - back, h2))};
}

// A split fragment: [0] = hi terms, [1] = lo terms.
struct Frag {
  u4 v[2];
};
// a_lo b_hi + a_hi b_lo + a_hi b_hi, small terms first
__device__ __forceinline__ f4 mma3(const Frag &a, const Frag &b, f4 c) {
  const h8 ah = __builtin_bit_cast(h8, a.v[0]), al = __builtin_bit_cast(h8, a.v[1]);
  const h8 bh = __builtin_bit_cast(h8, b.v[0]), bl = __builtin_bit_cast(h8, b.v[1]);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c, 0, 0, 0);
}

// Closes one unit's scheduling region: the next unit's 8 ds_reads first, then
// one MFMA and up to NV VALU at a time (see chain_bf16.hip).
template <int NM, int NV>
__device__ __forceinline__ void interleave() {
  __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
}

// UPC = units (4 split fragments, 8 KiB) per ring chunk: 1 (8 KiB chunks,
// 4 slots: fits beside the rollout's per-IC scratch) or 2 (16 KiB, 3 slots).
template <int UPC, bool LDR = false, bool DEF = false>
struct CoreF16x3T {
  static constexpr int kNW = kWaves;
  static constexpr int kWGPerCU = 1;
  static constexpr int kStreamOffset = 0;
  static constexpr int kUPC = UPC;
  static constexpr int kSlots = UPC == 2 ? 3 : 4;
  static constexpr int kAhead = 2;
  static constexpr int kWinMT = 4;
  static constexpr int kChunkFloats = 2048 * UPC;
  static constexpr int kKB = kH / 32;
  // parked fragments of k-blocks 0..2: [kb 3][mt 4][term 2][lane 64][4 dwords]
  static constexpr int kParkFloats = 3 * 4 * 2 * 64 * 4;
  // LDR: a loader wave issues the ring DMA; DEF: each wave's DMA owed by a
  // next() is issued after the following unit's fragment reads
  using R_t = Ring<kChunkFloats, kNW, kSlots, 2, DEF, LDR>;

  template <int MT>
  struct Acts {
    Frag h[MT][kKB];  // split B fragments of h
  };
  // One output pair's accumulators: W_a h (+ bias) and G = W_b h.
  template <int MT>
  struct PairAcc {
    f4 a[MT][2], g[MT][2];
  };

  // Register-prefetched weight feed: the next unit's 8 ds_read_b128 issue
  // before this unit's MFMAs; the ring's wait + barrier for chunk p+1 precede
  // the last unit of chunk p.
  struct Feed {
    const float *slot;
    Frag cur[4];
  };
  static __device__ __forceinline__ void load_unit(Feed &F, int u, int lane) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        F.cur[i].v[s] = __builtin_bit_cast(u4, ldf4(F.slot + (((4 * u + i) * 2 + s) * 64 + lane) * 4));
  }
  static __device__ __forceinline__ void begin(R_t &R, Feed &F) {
    F.slot = R.next();
    load_unit(F, 0, R.lane);
    if constexpr (DEF && UPC == 1) R.issue_pending();  // (UPC > 1: take<0> issues it)
  }
  template <int U>
  static __device__ __forceinline__ void take(R_t &R, Feed &F, Frag (&w)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = F.cur[i];
    if constexpr (U == UPC - 1) F.slot = R.next();
#ifndef HF_DIAG_NODS  // timing diagnostic only: results are wrong
    load_unit(F, (U + 1) % UPC, R.lane);
#endif
    if constexpr (DEF && U == 0) R.issue_pending();
  }

  static __device__ __forceinline__ float *park_at(float *park, int kb, int mt, int s, int lane) {
    return park + (((kb * 4 + mt) * 2 + s) * 64 + lane) * 4;
  }

  // Dword K (tile t = K>>1, rows 2(K&1), 2(K&1)+1) of the new k-block
  // fragment from one output pair: h = ReLU(acc + 0.5*(G[i+1] + G[i-1]))
  // (src/flux_gnn.py:55-60; 0.5*x is exact), split into fp16 hi/lo.
  template <int MT, int K>
  static __device__ __forceinline__ void piece(const PairAcc<MT> &p, Frag (&nh)[MT]) {
    constexpr int t = K >> 1, r = 2 * (K & 1);
#ifdef HF_DIAG_NOPIECE  // timing diagnostic only: results are wrong (no epilogue VALU)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      nh[mt].v[0][K] = __float_as_uint(p.a[mt][t][r]);
      nh[mt].v[1][K] = __float_as_uint(p.g[mt][t][r]);
    }
    return;
#endif
    float v[2][MT];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      float gv[MT], gs[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) gv[mt] = p.g[mt][t][r + e];
      nb_sum<MT>(gv, gs);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) v[e][mt] = relu(fmaf(gs[mt], 0.5f, p.a[mt][t][r + e]));
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const Split sp = split_pair(v[0][mt], v[1][mt]);
      nh[mt].v[0][K] = sp.hi;
      nh[mt].v[1][K] = sp.lo;
    }
  }

  // One unit of an update pair: k-block KB, fragments (t, W_a | W_b) = w[2t + ab].
  template <int MT, int KB, int U>
  static __device__ __forceinline__ void unit(R_t &R, Feed &F, const Acts<MT> &X, PairAcc<MT> &p) {
    Frag w[4];
    take<U>(R, F, w);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        if (i & 1) p.g[mt][i >> 1] = mma3(w[i], X.h[mt][KB], p.g[mt][i >> 1]);
        else p.a[mt][i >> 1] = mma3(w[i], X.h[mt][KB], p.a[mt][i >> 1]);
      }
  }

  template <int MT>
  static __device__ __forceinline__ void init_pair(const float *bias, int q, int g4, PairAcc<MT> &p) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const f4 b = ldf4(bias + 16 * (2 * q + t) + g4);  // b_l enters as the first MFMA's C operand
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        p.a[mt][t] = b;
        p.g[mt][t] = f4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }

  // Output pair q >= 1, with the epilogue of pair q-1 (prev) spread over its
  // 4 units and parked as k-block q-1.
  template <int MT>
  static __device__ __forceinline__ void pair_with_prev(R_t &R, Feed &F, const Acts<MT> &X, const float *bias, int q,
                                                        int g4, PairAcc<MT> &p, const PairAcc<MT> &prev, float *park,
                                                        int lane) {
    init_pair<MT>(bias, q, g4, p);
    Frag nh[MT];
    unit<MT, 0, 0 % UPC>(R, F, X, p);
    piece<MT, 0>(prev, nh);
    interleave<12 * MT, 1>();
    unit<MT, 1, 1 % UPC>(R, F, X, p);
    piece<MT, 1>(prev, nh);
    interleave<12 * MT, 1>();
    unit<MT, 2, 2 % UPC>(R, F, X, p);
    piece<MT, 2>(prev, nh);
    interleave<12 * MT, 1>();
    unit<MT, 3, 3 % UPC>(R, F, X, p);
    piece<MT, 3>(prev, nh);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int s = 0; s < 2; ++s) *reinterpret_cast<u4 *>(park_at(park, q - 1, mt, s, lane)) = nh[mt].v[s];
    interleave<12 * MT, 1>();
  }

  // Pair 0 of a layer after another: k-blocks 0..2 from the park, k-block 3
  // from the previous layer's pair 3 (pend), finished under the first units.
  template <int MT>
  static __device__ __forceinline__ void pair0_after(R_t &R, Feed &F, Acts<MT> &X, const float *bias, int g4,
                                                     PairAcc<MT> &p, const PairAcc<MT> &pend, float *park,
                                                     int lane) {
    wave_lds_sync();  // this wave's park writes of the previous layer have landed
#pragma unroll
    for (int kb = 0; kb < 3; ++kb)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int s = 0; s < 2; ++s) X.h[mt][kb].v[s] = __builtin_bit_cast(u4, ldf4(park_at(park, kb, mt, s, lane)));
    init_pair<MT>(bias, 0, g4, p);
    Frag nh[MT];
    unit<MT, 0, 0 % UPC>(R, F, X, p);
    piece<MT, 0>(pend, nh);
    piece<MT, 1>(pend, nh);
    interleave<12 * MT, 1>();
    unit<MT, 1, 1 % UPC>(R, F, X, p);
    piece<MT, 2>(pend, nh);
    interleave<12 * MT, 1>();
    unit<MT, 2, 2 % UPC>(R, F, X, p);
    piece<MT, 3>(pend, nh);
    interleave<12 * MT, 1>();
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) X.h[mt][3] = nh[mt];
    unit<MT, 3, 3 % UPC>(R, F, X, p);
    interleave<12 * MT, 0>();
  }

  template <int MT>
  static __device__ __forceinline__ void pair0_first(R_t &R, Feed &F, const Acts<MT> &X, const float *bias, int g4,
                                                     PairAcc<MT> &p) {
    init_pair<MT>(bias, 0, g4, p);
    unit<MT, 0, 0 % UPC>(R, F, X, p);
    interleave<12 * MT, 0>();
    unit<MT, 1, 1 % UPC>(R, F, X, p);
    interleave<12 * MT, 0>();
    unit<MT, 2, 2 % UPC>(R, F, X, p);
    interleave<12 * MT, 0>();
    unit<MT, 3, 3 % UPC>(R, F, X, p);
    interleave<12 * MT, 0>();
  }

  template <int MT>
  static __device__ __forceinline__ void pairs_rest(R_t &R, Feed &F, const Acts<MT> &X, const float *bias, int g4,
                                                    PairAcc<MT> &p0, PairAcc<MT> &pend, float *park, int lane) {
    PairAcc<MT> p1, p2;
    pair_with_prev<MT>(R, F, X, bias, 1, g4, p1, p0, park, lane);
    pair_with_prev<MT>(R, F, X, bias, 2, g4, p2, p1, park, lane);
    pair_with_prev<MT>(R, F, X, bias, 3, g4, pend, p2, park, lane);
  }

  // Readout unit U of output tile ot (fragment i = 2*(kb - 2U) + (P|Q)), ring index T.
  template <int MT, int U, int T>
  static __device__ __forceinline__ void ro_unit(R_t &R, Feed &F, const Acts<MT> &X, f4 (&P)[MT], f4 (&Q)[MT]) {
    Frag w[4];
    take<T>(R, F, w);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kb = 2 * U + (i >> 1);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        if (i & 1) Q[mt] = mma3(w[i], X.h[mt][kb], Q[mt]);
        else P[mt] = mma3(w[i], X.h[mt][kb], P[mt]);
      }
    }
  }

  template <int MT>
  static __device__ __forceinline__ void init_ro(const Small &S, int ot, int g4, f4 (&P)[MT], f4 (&Q)[MT]) {
    const f4 be = ldf4(S.be + 16 * ot + g4);  // b_e enters P as the C operand of its first MFMA
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      P[mt] = be;
      Q[mt] = f4{0.f, 0.f, 0.f, 0.f};
    }
  }

  // Readout tile ot >= 1 (ring indices 0, 1 % UPC), with the epilogue of tile
  // ot-1 (rows in order, as readout_epilogue) spread over its two units.
  template <int MT>
  static __device__ __forceinline__ void ro_tile(R_t &R, Feed &F, const Acts<MT> &X, const Small &S, int ot,
                                                 int g4, f4 (&P)[MT], f4 (&Q)[MT], float (&pf)[MT],
                                                 float (&pb)[MT]) {
    f4 Pn[MT], Qn[MT];
    init_ro<MT>(S, ot, g4, Pn, Qn);
    const f4 w2 = ldf4(S.w2 + 16 * (ot - 1) + g4);
    ro_unit<MT, 0, 0>(R, F, X, Pn, Qn);
    readout_row<MT, 0, true>(P, Q, w2, w2, pf, pb);
    readout_row<MT, 1, true>(P, Q, w2, w2, pf, pb);
    interleave<12 * MT, 1>();
    ro_unit<MT, 1, 1 % UPC>(R, F, X, Pn, Qn);
    readout_row<MT, 2, true>(P, Q, w2, w2, pf, pb);
    readout_row<MT, 3, true>(P, Q, w2, w2, pf, pb);
    interleave<12 * MT, 1>();
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      P[mt] = Pn[mt];
      Q[mt] = Qn[mt];
    }
  }

  // Edge readout, P/Q split (src/flux_gnn.py:62-66), pipelined tile by tile;
  // the last layer's pair 3 (pend) is activated under the first readout unit.
  template <int MT>
  static __device__ __forceinline__ void readout(const ChainW &W, const Small &S, R_t &R, Feed &F, Acts<MT> &X,
                                                 const PairAcc<MT> &pend, float *park, int lane, int g4,
                                                 float (&ffwd)[MT], float (&fbwd)[MT]) {
    wave_lds_sync();
#pragma unroll
    for (int kb = 0; kb < 3; ++kb)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int s = 0; s < 2; ++s) X.h[mt][kb].v[s] = __builtin_bit_cast(u4, ldf4(park_at(park, kb, mt, s, lane)));
    float pf[MT], pb[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) pf[mt] = pb[mt] = 0.f;
    f4 P[MT], Q[MT];
    init_ro<MT>(S, 0, g4, P, Q);
    {
      Frag nh[MT];
      ro_unit<MT, 0, 0>(R, F, X, P, Q);
      piece<MT, 0>(pend, nh);
      piece<MT, 1>(pend, nh);
      piece<MT, 2>(pend, nh);
      piece<MT, 3>(pend, nh);
      interleave<12 * MT, 1>();
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) X.h[mt][3] = nh[mt];
      ro_unit<MT, 1, 1 % UPC>(R, F, X, P, Q);
      interleave<12 * MT, 0>();
    }
    // tiles 1..7 (two units each, so every tile starts a ring chunk)
    for (int ot = 1; ot < kNT; ++ot) ro_tile<MT>(R, F, X, S, ot, g4, P, Q, pf, pb);
    {
      const f4 w2 = ldf4(S.w2 + 16 * (kNT - 1) + g4);
      readout_epilogue<MT, true>(P, Q, w2, w2, pf, pb);
    }
    readout_finish<MT>(pf, pb, W.b2, ffwd, fbwd);
  }

  template <int MT>
  static __device__ __forceinline__ void gnn(const ChainW &W, const Small &S, R_t &R, Feed &F, float *park,
                                             const float (&feat)[MT], float (&ffwd)[MT], float (&fbwd)[MT]) {
    const int lane = R.lane;
    const int g4 = 4 * (lane >> 4);
    Acts<MT> X;
    PairAcc<MT> pend;
    {
      f4 h[MT][kNT];
      input_layer<MT>(S, lane, feat, h);  // f32 MFMA, ReLU applied
#pragma unroll
      for (int kb = 0; kb < kKB; ++kb)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int t = k >> 1, r = 2 * (k & 1);
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const Split sp = split_pair(h[mt][2 * kb + t][r], h[mt][2 * kb + t][r + 1]);
            X.h[mt][kb].v[0][k] = sp.hi;
            X.h[mt][kb].v[1][k] = sp.lo;
          }
        }
      if (W.layers == 0) {
        // no update layer: hand the readout the input layer's output the way
        // a last layer would (k-blocks 0..2 parked, tiles 6, 7 pending with
        // G = 0, so the epilogue returns ReLU(h) = h)
#pragma unroll
        for (int kb = 0; kb < 3; ++kb)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int s = 0; s < 2; ++s) *reinterpret_cast<u4 *>(park_at(park, kb, mt, s, lane)) = X.h[mt][kb].v[s];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            pend.a[mt][t] = h[mt][6 + t];
            pend.g[mt][t] = f4{0.f, 0.f, 0.f, 0.f};
          }
      }
    }
    // message passing (src/flux_gnn.py:53-60), pair-pipelined
    if (W.layers > 0) {
      PairAcc<MT> p0;
      pair0_first<MT>(R, F, X, S.bl, g4, p0);
      pairs_rest<MT>(R, F, X, S.bl, g4, p0, pend, park, lane);
    }
    for (int l = 1; l < W.layers; ++l) {
      const float *bias = S.bl + l * kH;
      PairAcc<MT> p0;
      pair0_after<MT>(R, F, X, bias, g4, p0, pend, park, lane);
      pairs_rest<MT>(R, F, X, bias, g4, p0, pend, park, lane);
    }
    readout<MT>(W, S, R, F, X, pend, park, lane, g4, ffwd, fbwd);
  }
};

// ---------------------------------------------------------------------------
// Cell-split f16x3 core for small batches (chain_common.h
// chain_rollout_cells_kernel / chain_flux_cells_kernel): 16 cells per wave,
// an IC over nx/16 waves, CoreF16x3T's arithmetic MFMA chain for chain (so a
// batch gets the IC-per-wave kernels' bits whichever kernel its size
// selects), laid out like chain_bf16.hip's CellBF16: a layer's four output
// pairs, then the G values of the edge columns traded through LDS around one
// barrier, then the epilogue; the readout trades column 0 of P and Q.
template <bool LDR = false>
struct CellF16x3T {
  using Base = CoreF16x3T<1, LDR>;  // the rollout's ring: 8 KiB chunks (one unit), 4 slots
  // barrier schedule of one pass (the loader wave's, chain_rollout_cells_kernel):
  // 16 ring chunks per update layer, then the G trade's barrier
  static constexpr int kLayerChunks = 16;
  static constexpr bool kLayerBarrier = true;
  static constexpr int kNW = Base::kNW;
  static constexpr int kSlots = Base::kSlots;
  static constexpr int kChunkFloats = Base::kChunkFloats;
  static constexpr int kStreamOffset = 0;
  using R_t = typename Base::R_t;
  using Feed = typename Base::Feed;
  static __device__ __forceinline__ void begin(R_t &R, Feed &F) { Base::begin(R, F); }

  static __device__ __forceinline__ void gnn_cells(const ChainW &W, const Small &S, R_t &R, Feed &F,
                                                   const float (&feat)[1], float (&ffwd)[1], float (&fbwd)[1],
                                                   CellHalo &X) {
    const int lane = R.lane, g4 = 4 * (lane >> 4), g = lane >> 4, j = lane & 15;
    typename Base::template Acts<1> A;
    {
      f4 h[1][kNT];
      input_layer<1>(S, lane, feat, h);  // f32 MFMA, ReLU applied
#pragma unroll
      for (int kb = 0; kb < Base::kKB; ++kb)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int t = k >> 1, r = 2 * (k & 1);
          const Split sp = split_pair(h[0][2 * kb + t][r], h[0][2 * kb + t][r + 1]);
          A.h[0][kb].v[0][k] = sp.hi;
          A.h[0][kb].v[1][k] = sp.lo;
        }
    }
    // message passing (src/flux_gnn.py:53-60)
    for (int l = 0; l < W.layers; ++l) {
      const float *bias = S.bl + l * kH;
      typename Base::template PairAcc<1> acc[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        Base::template init_pair<1>(bias, q, g4, acc[q]);
        Base::template unit<1, 0, 0>(R, F, A, acc[q]);
        interleave<12, 0>();
        Base::template unit<1, 1, 0>(R, F, A, acc[q]);
        interleave<12, 0>();
        Base::template unit<1, 2, 0>(R, F, A, acc[q]);
        interleave<12, 0>();
        Base::template unit<1, 3, 0>(R, F, A, acc[q]);
        interleave<12, 0>();
      }
      {
        f4 G[1][kNT];
#pragma unroll
        for (int t = 0; t < kNT; ++t) G[0][t] = acc[t >> 1].g[0][t & 1];
        X.exchange(G);  // X.l / X.r: G of cell 16*pos - 1 / 16*pos + 16
      }
      // h = ReLU(acc + 0.5*(G[i-1] + G[i+1])), split into fp16 hi/lo (Base::piece)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int K = 0; K < 4; ++K) {
          const int tt = K >> 1, t = 2 * q + tt, r0 = 2 * (K & 1);
          float v[2];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int r = r0 + e;
            const float gv = acc[q].g[0][tt][r];
            const float gl = dpp_over<kRowShr1>(X.l[t][r], gv), gr = dpp_over<kRowShl1>(X.r[t][r], gv);
            v[e] = relu(fmaf(__fadd_rn(gl, gr), 0.5f, acc[q].a[0][tt][r]));
          }
          const Split sp = split_pair(v[0], v[1]);
          A.h[0][q].v[0][K] = sp.hi;
          A.h[0][q].v[1][K] = sp.lo;
        }
    }
    // edge readout, P/Q split (src/flux_gnn.py:62-66): all 8 tiles, column 0
    // of P and Q through LDS, then the epilogue rows in Base::readout's order
    f4 P[kNT][1], Q[kNT][1];
#pragma unroll
    for (int ot = 0; ot < kNT; ++ot) {
      Base::template init_ro<1>(S, ot, g4, P[ot], Q[ot]);
      Base::template ro_unit<1, 0, 0>(R, F, A, P[ot], Q[ot]);
      interleave<12, 0>();
      Base::template ro_unit<1, 1, 0>(R, F, A, P[ot], Q[ot]);
      interleave<12, 0>();
      if (j == 0) {
        X.xq[((X.wave * kNT + ot) * 2 + 0) * 4 + g] = P[ot][0];
        X.xq[((X.wave * kNT + ot) * 2 + 1) * 4 + g] = Q[ot][0];
      }
    }
    lds_barrier();
    float pf = 0.f, pb = 0.f;
#pragma unroll
    for (int ot = 0; ot < kNT; ++ot) {
      const f4 prh = X.xq[((X.rw * kNT + ot) * 2 + 0) * 4 + g];
      const f4 qrh = X.xq[((X.rw * kNT + ot) * 2 + 1) * 4 + g];
      const f4 w2 = ldf4(S.w2 + 16 * ot + g4);
      readout_row_halo<0>(P[ot][0], Q[ot][0], prh, qrh, w2, pf, pb);
      readout_row_halo<1>(P[ot][0], Q[ot][0], prh, qrh, w2, pf, pb);
      readout_row_halo<2>(P[ot][0], Q[ot][0], prh, qrh, w2, pf, pb);
      readout_row_halo<3>(P[ot][0], Q[ot][0], prh, qrh, w2, pf, pb);
    }
    float pf1[1] = {pf}, pb1[1] = {pb};
    readout_finish<1>(pf1, pb1, W.b2, ffwd, fbwd);
  }
};
#ifndef HF_CELLS_LOADER
#define HF_CELLS_LOADER 1
#endif
using CellF16x3Ld = CellF16x3T<HF_CELLS_LOADER != 0>;  // with a loader wave (the cell-split kernels)
#ifndef HF_K32_DEFER
#define HF_K32_DEFER 1
#endif
constexpr bool kK32Defer = HF_K32_DEFER != 0;  // IC-per-wave f16x3 cores: deferred ring DMA (CoreF16x3T DEF)

}  // namespace

hipError_t launch_chain_flux_k32(const ChainW &w, const float *nf, const float *state, int64_t ld_state,
                                 const float *x, int B, int nx, float *fe, float *ff, hipStream_t s) {
  if (w.prec != kPrecF16x3) return launch_chain_flux_bf16(w, nf, state, ld_state, x, B, nx, fe, ff, s);
  if (chain_rollout_prefers_cells(w, B, nx)) {  // small batches: each chain over nx/16 waves
    switch (nx) {
      case 32: return chain::flux_cells_launch<CellF16x3Ld, 2>(w, nf, state, ld_state, x, B, fe, ff, s);
      case 48: return chain::flux_cells_launch<CellF16x3Ld, 3>(w, nf, state, ld_state, x, B, fe, ff, s);
      case 64: return chain::flux_cells_launch<CellF16x3Ld, 4>(w, nf, state, ld_state, x, B, fe, ff, s);
      default: break;
    }
  }
  if (nx == 16 || nx == 32 || nx == 48 || nx == 64)
    return chain::launch_flux_core<CoreF16x3T<1, false, kK32Defer>>(w, nf, state, ld_state, x, B, nx, fe, ff, s);
  return chain::launch_flux_windowed<CoreF16x3T<2, false, kK32Defer>>(w, nf, state, ld_state, x, B, nx, fe, ff, s);
}

hipError_t launch_chain_rollout_k32(const ChainW &w, const float *state0, float *state_final, const float *x,
                                    const double *pc, int B, int nx, int T, float c, float dt, float *traj,
                                    float *flux_traj, float *metrics, const RolloutExtras &ex, hipStream_t s) {
  if (w.prec == kPrecF16x3 && ex.mse == nullptr && ex.metrics_cl == nullptr && chain_rollout_prefers_cells(w, B, nx)) {
    switch (nx) {  // small batches: each IC over nx/16 waves (cell-split kernel, same bits)
      case 32: return chain::cells_launch<CellF16x3Ld, 2>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, ex.poisson, s);
      case 48: return chain::cells_launch<CellF16x3Ld, 3>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, ex.poisson, s);
      case 64: return chain::cells_launch<CellF16x3Ld, 4>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, ex.poisson, s);
      default: break;
    }
  }
  if (w.prec == kPrecF16x3)
    return chain::launch_rollout_core<CoreF16x3T<1, false, kK32Defer>>(w, state0, state_final, x, pc, B, nx, T, c, dt, traj,
                                                     flux_traj, metrics, ex, s);
  return launch_chain_rollout_bf16(w, state0, state_final, x, pc, B, nx, T, c, dt, traj, flux_traj, metrics, ex,
                                   s);
}

}  // namespace hf
