// Fused FluxGNN on the periodic chain in bf16 (BASELINE config 4, "bf16 MLP
// weights"): v_mfma_f32_16x16x32_bf16, bf16 weights and activations, fp32
// accumulate.
//
// Reference: src/flux_gnn.py:40-67 (forward), src/hybrid_solver.py:34-73.
//
// Same transposed-GEMM scheme as the other chain cores (chain_common.h): a
// 16x16 accumulator tile holds 16 cells along the lanes, and the output tile
// pair (2q, 2q+1) of one layer is, lane for lane, k-block q of the next
// layer's B operand (element e of the 8-wide fragment = tile 2q + (e>>2),
// row e&3; capi.cpp packs the weights in that k order).  The neighbour sum
// h[i+1] + h[i-1] is taken in fp32 on the interleaved cell layout (one VALU per
// value) and rounded into its own B fragments; the 1/deg is folded into W_b.
//
// Why a separate core: at 16 cycles per v_mfma_f32_16x16x32_bf16 the layer
// epilogue (ReLU, neighbour sums, bf16 packing: ~3 VALU per activated value)
// costs as much issue time as the matrix work, and with one wave per SIMD
// nothing overlaps an epilogue that waits for its whole layer.  This core
// walks each layer in OUTPUT-PAIR order (pair q = tiles 2q, 2q+1, accumulated
// over the 4 k-blocks of h and the 4 of the neighbour sums: 64 MFMAs at
// MT=4) and spreads the epilogue of pair q-1 over the MFMAs of pair q, one
// fragment dword per unit of 16 MFMAs.  The new fragments of pairs 0..2 are
// parked in LDS (the old ones still feed the layer) and read back when the
// layer ends; the epilogue of pair 3 runs under the first three k-blocks of
// the next layer's pair 0 (or the first readout tile), which produce nothing
// it needs.  The readout is pipelined the same way, tile by tile.
#include "chain_common.h"

namespace hf {
namespace {

using namespace chain;

typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef __bf16 b2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

// bf16(a) in the low half, bf16(b) in the high half (v_cvt_pk_bf16_f32, RNE, NaN stays NaN)
__device__ __forceinline__ unsigned pk_bf16(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f2{a, b}, b2));
}
__device__ __forceinline__ f4 mma(const u4 &a, const u4 &b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8, a), __builtin_bit_cast(b8, b), c, 0, 0, 0);
}

// Closes one unit's scheduling region: the next unit's 4 ds_reads first (so
// LDS latency hides under this unit's matrix work), then one MFMA and up to NV
// VALU (epilogue work of the previous pair) at a time.  The sched_barrier keeps
// the next unit's reads from being picked for this unit's DS group.
template <int NM, int NV>
__device__ __forceinline__ void interleave() {
  __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
}

// NW = waves per workgroup sharing the weight ring; the kernels use NW = 4
// (one wave per SIMD, up to 64 cells per wave).  NW = 8 (two waves per SIMD
// at 191 registers, 32-cell windows) was measured for the windowed flux
// kernel: per FLOP 7 % faster, but 32-cell windows recompute 41 % halo
// against 19 % at 64 cells, so cfg4 ran at 2.18 M IC-steps/s against 2.41 M.
// WMT = m-tiles per wave of the windowed flux kernel: 80-cell windows (WMT = 5,
// 389 registers, 8 KiB chunks, the only ring that fits beside a 5-tile park)
// recompute 13 % halo instead of 16 % but ran 2.7 % slower at cfg4.
// UPC = units (4 fragments, 4 KiB) per ring chunk: 2 (8 KiB chunks, 4 slots)
// or 4 (16 KiB chunks, 3 slots: half the ring barriers, +16 KiB of LDS, which
// the windowed flux kernel has and the rollout, with its per-IC scratch, has not).
template <int NW, int UPC = 2, int WMT = (NW == 8 ? 2 : 4)>
struct CoreBF16T {
  static constexpr int kNW = NW;
  static constexpr int kUPC = UPC;
  static constexpr int kSlots = UPC == 4 ? 3 : 4;
  static constexpr int kWinMT = WMT;  // m-tiles per wave in the windowed flux kernel
  static constexpr int kParkMT = kWinMT;          // largest MT the park holds
  static constexpr int kChunkFloats = 1024 * UPC;
  static constexpr int kKB = kH / 32;        // k-blocks per 128-wide operand
  // parked fragments of k-blocks 0..2: [kb 3][h|agg 2][mt kParkMT][lane 64][4 dwords]
  static constexpr int kParkFloats = 3 * 2 * kParkMT * 64 * 4;
  using R_t = Ring<kChunkFloats, NW, kSlots>;

  template <int MT>
  struct Acts {
    u4 h[MT][kKB], a[MT][kKB];  // B fragments of h and of its neighbour sums
  };

  // Register-prefetched weight feed: the next unit's 4 ds_read_b128 issue
  // before this unit's MFMAs; the ring's wait + barrier for chunk p+1 precede
  // the last unit of chunk p.  Runs continuously over forward passes.
  struct Feed {
    const float *slot;
    u4 cur[4];
  };
  static __device__ __forceinline__ void load_unit(Feed &F, int u, int lane) {
#pragma unroll
    for (int i = 0; i < 4; ++i) F.cur[i] = __builtin_bit_cast(u4, ldf4(F.slot + ((4 * u + i) * 64 + lane) * 4));
  }
  static __device__ __forceinline__ void begin(R_t &R, Feed &F) {
    F.slot = R.next();
    load_unit(F, 0, R.lane);
  }
  template <int U>
  static __device__ __forceinline__ void take(R_t &R, Feed &F, u4 (&w)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = F.cur[i];
    if constexpr (U == UPC - 1) F.slot = R.next();
#ifndef HF_DIAG_NODS  // timing diagnostic only: results are wrong
    load_unit(F, (U + 1) % UPC, R.lane);
#endif
  }

  static __device__ __forceinline__ float *park_at(float *park, int kb, int ha, int mt, int lane) {
    return park + (((kb * 2 + ha) * kParkMT + mt) * 64 + lane) * 4;
  }

  // Dword K (tile t = K>>1, rows 2(K&1), 2(K&1)+1) of the k-block fragments
  // made from one output pair's accumulators: ReLU, then (AGG) the fp32
  // neighbour sums (src/flux_gnn.py:55-59; / deg is in W_b), then bf16 pairs.
  template <int MT, int K, bool AGG>
  static __device__ __forceinline__ void piece(const f4 (&acc)[MT][2], u4 (&nh)[MT], u4 (&na)[MT]) {
    constexpr int t = K >> 1, r = 2 * (K & 1);
#ifdef HF_DIAG_NOPIECE  // timing diagnostic only: results are wrong (no epilogue VALU)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) nh[mt][K] = na[mt][K] = __float_as_uint(acc[mt][t][r]);
    return;
#endif
    float v0[MT], v1[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      v0[mt] = relu(acc[mt][t][r]);
      v1[mt] = relu(acc[mt][t][r + 1]);
      nh[mt][K] = pk_bf16(v0[mt], v1[mt]);
    }
    if constexpr (AGG) {
      float s0[MT], s1[MT];
#ifdef HF_DIAG_NONB  // timing diagnostic only: results are wrong
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) s0[mt] = v0[mt], s1[mt] = v1[mt];
#else
      nb_sum<MT>(v0, s0);
      nb_sum<MT>(v1, s1);
#endif
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) na[mt][K] = pk_bf16(s0[mt], s1[mt]);
    }
  }

  // One unit of an update pair: k-block KB, fragments (t, W_a | W_b/2) = w[2t + ab].
  template <int MT, int KB, int U>
  static __device__ __forceinline__ void unit(R_t &R, Feed &F, const Acts<MT> &X, f4 (&acc)[MT][2]) {
    u4 w[4];
    take<U>(R, F, w);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        acc[mt][i >> 1] = mma(w[i], (i & 1) ? X.a[mt][KB] : X.h[mt][KB], acc[mt][i >> 1]);
  }

  template <int MT>
  static __device__ __forceinline__ void init_pair(const float *bias, int q, int g4, f4 (&acc)[MT][2]) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const f4 b = ldf4(bias + 16 * (2 * q + t) + g4);  // b_l enters as the first MFMA's C operand
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt][t] = b;
    }
  }

  // Output pair q >= 1 of an update layer, with the epilogue of pair q-1
  // (prev) spread over its 4 units and parked as k-block q-1.
  template <int MT>
  static __device__ __forceinline__ void pair_with_prev(R_t &R, Feed &F, const Acts<MT> &X, const float *bias, int q,
                                                        int g4, f4 (&acc)[MT][2], const f4 (&prev)[MT][2],
                                                        float *park, int lane) {
    init_pair<MT>(bias, q, g4, acc);
    u4 nh[MT], na[MT];
    unit<MT, 0, 0 % UPC>(R, F, X, acc);
    piece<MT, 0, true>(prev, nh, na);
    interleave<4 * MT, 2>();
    unit<MT, 1, 1 % UPC>(R, F, X, acc);
    piece<MT, 1, true>(prev, nh, na);
    interleave<4 * MT, 2>();
    unit<MT, 2, 2 % UPC>(R, F, X, acc);
    piece<MT, 2, true>(prev, nh, na);
    interleave<4 * MT, 2>();
    unit<MT, 3, 3 % UPC>(R, F, X, acc);
    piece<MT, 3, true>(prev, nh, na);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      *reinterpret_cast<u4 *>(park_at(park, q - 1, 0, mt, lane)) = nh[mt];
      *reinterpret_cast<u4 *>(park_at(park, q - 1, 1, mt, lane)) = na[mt];
    }
    interleave<4 * MT, 2>();
  }

  // Pair 0 of a layer that follows another: k-blocks 0..2 come back from the
  // park, k-block 3 is the previous layer's pair 3 (pend), finished under the
  // first three units.
  template <int MT>
  static __device__ __forceinline__ void pair0_after(R_t &R, Feed &F, Acts<MT> &X, const float *bias, int g4,
                                                     f4 (&acc)[MT][2], const f4 (&pend)[MT][2], float *park,
                                                     int lane) {
    wave_lds_sync();  // this wave's park writes of the previous layer have landed
#pragma unroll
    for (int kb = 0; kb < 3; ++kb)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        X.h[mt][kb] = __builtin_bit_cast(u4, ldf4(park_at(park, kb, 0, mt, lane)));
        X.a[mt][kb] = __builtin_bit_cast(u4, ldf4(park_at(park, kb, 1, mt, lane)));
      }
    init_pair<MT>(bias, 0, g4, acc);
    u4 nh[MT], na[MT];
    unit<MT, 0, 0 % UPC>(R, F, X, acc);
    piece<MT, 0, true>(pend, nh, na);
    piece<MT, 1, true>(pend, nh, na);
    interleave<4 * MT, 4>();
    unit<MT, 1, 1 % UPC>(R, F, X, acc);
    piece<MT, 2, true>(pend, nh, na);
    interleave<4 * MT, 2>();
    unit<MT, 2, 2 % UPC>(R, F, X, acc);
    piece<MT, 3, true>(pend, nh, na);
    interleave<4 * MT, 2>();
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      X.h[mt][3] = nh[mt];
      X.a[mt][3] = na[mt];
    }
    unit<MT, 3, 3 % UPC>(R, F, X, acc);
    interleave<4 * MT, 0>();
  }

  // Pair 0 of the first layer (X complete from the input layer).
  template <int MT>
  static __device__ __forceinline__ void pair0_first(R_t &R, Feed &F, const Acts<MT> &X, const float *bias, int g4,
                                                     f4 (&acc)[MT][2]) {
    init_pair<MT>(bias, 0, g4, acc);
    unit<MT, 0, 0 % UPC>(R, F, X, acc);
    interleave<4 * MT, 0>();
    unit<MT, 1, 1 % UPC>(R, F, X, acc);
    interleave<4 * MT, 0>();
    unit<MT, 2, 2 % UPC>(R, F, X, acc);
    interleave<4 * MT, 0>();
    unit<MT, 3, 3 % UPC>(R, F, X, acc);
    interleave<4 * MT, 0>();
  }

  // Pairs 1..3 of a layer; returns pair 3's accumulators (its epilogue is pending).
  template <int MT>
  static __device__ __forceinline__ void pairs_rest(R_t &R, Feed &F, const Acts<MT> &X, const float *bias, int g4,
                                                    f4 (&acc0)[MT][2], f4 (&pend)[MT][2], float *park, int lane) {
    f4 acc1[MT][2], acc2[MT][2];
    pair_with_prev<MT>(R, F, X, bias, 1, g4, acc1, acc0, park, lane);
    pair_with_prev<MT>(R, F, X, bias, 2, g4, acc2, acc1, park, lane);
    pair_with_prev<MT>(R, F, X, bias, 3, g4, pend, acc2, park, lane);
  }

  // Readout unit U of output tile ot: fragment i = 2*(kb - 2U) + (P|Q), kb = 2U, 2U+1;
  // T = its index in the ring chunk.
  template <int MT, int U, int T>
  static __device__ __forceinline__ void ro_unit(R_t &R, Feed &F, const Acts<MT> &X, f4 (&P)[MT], f4 (&Q)[MT]) {
    u4 w[4];
    take<T>(R, F, w);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int kb = 2 * U + (i >> 1);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        if (i & 1) Q[mt] = mma(w[i], X.h[mt][kb], Q[mt]);
        else P[mt] = mma(w[i], X.h[mt][kb], P[mt]);
      }
    }
  }

  // Rows 2RP, 2RP+1 of one readout tile's epilogue: z_fwd(i) = P(i) + Q(i+1),
  // z_bwd(i) = P(i+1) + Q(i) (b_e already in P); partial += w2 . ReLU(z)
  // (src/flux_gnn.py:62-66), rows in order as readout_epilogue.
  template <int MT, int RP>
  static __device__ __forceinline__ void ro_piece(const f4 (&P)[MT], const f4 (&Q)[MT], const f4 &w2, float (&pf)[MT],
                                                  float (&pb)[MT]) {
#pragma unroll
    for (int r = 2 * RP; r < 2 * RP + 2; ++r) {
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

  template <int MT>
  static __device__ __forceinline__ void init_ro(const Small &S, int ot, int g4, f4 (&P)[MT], f4 (&Q)[MT]) {
    const f4 be = ldf4(S.be + 16 * ot + g4);  // b_e enters P as the C operand of its first MFMA
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      P[mt] = be;
      Q[mt] = f4{0.f, 0.f, 0.f, 0.f};
    }
  }

  // Readout tile ot >= 1 (ring indices T0, T0+1), with the epilogue of tile
  // ot-1 (P, Q on entry; tile ot's on exit) spread over its two units.
  template <int MT, int T0>
  static __device__ __forceinline__ void ro_tile(R_t &R, Feed &F, const Acts<MT> &X, const Small &S, int ot,
                                                 int g4, f4 (&P)[MT], f4 (&Q)[MT], float (&pf)[MT],
                                                 float (&pb)[MT]) {
    f4 Pn[MT], Qn[MT];
    init_ro<MT>(S, ot, g4, Pn, Qn);
    const f4 w2 = ldf4(S.w2 + 16 * (ot - 1) + g4);
    ro_unit<MT, 0, T0>(R, F, X, Pn, Qn);
    ro_piece<MT, 0>(P, Q, w2, pf, pb);
    interleave<4 * MT, 3>();
    ro_unit<MT, 1, T0 + 1>(R, F, X, Pn, Qn);
    ro_piece<MT, 1>(P, Q, w2, pf, pb);
    interleave<4 * MT, 3>();
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      P[mt] = Pn[mt];
      Q[mt] = Qn[mt];
    }
  }

  // Edge readout, P/Q split (src/flux_gnn.py:62-66), pipelined tile by tile.
  // The last layer's pair 3 (pend) is still to be activated: h of k-blocks
  // 0..2 comes from the park, k-block 3 is finished under the first readout unit.
  template <int MT>
  static __device__ __forceinline__ void readout(const ChainW &W, const Small &S, R_t &R, Feed &F, Acts<MT> &X,
                                                 const f4 (&pend)[MT][2], float *park, int lane, int g4,
                                                 float (&ffwd)[MT], float (&fbwd)[MT]) {
    wave_lds_sync();
#pragma unroll
    for (int kb = 0; kb < 3; ++kb)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) X.h[mt][kb] = __builtin_bit_cast(u4, ldf4(park_at(park, kb, 0, mt, lane)));
    float pf[MT], pb[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) pf[mt] = pb[mt] = 0.f;
    f4 P[MT], Q[MT];
    init_ro<MT>(S, 0, g4, P, Q);
    {
      u4 nh[MT], na[MT];
      ro_unit<MT, 0, 0>(R, F, X, P, Q);
      piece<MT, 0, false>(pend, nh, na);
      piece<MT, 1, false>(pend, nh, na);
      piece<MT, 2, false>(pend, nh, na);
      piece<MT, 3, false>(pend, nh, na);
      interleave<4 * MT, 3>();
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) X.h[mt][3] = nh[mt];
      ro_unit<MT, 1, 1>(R, F, X, P, Q);
      interleave<4 * MT, 0>();
    }
    // tiles 1..7; an odd tile starts mid-chunk when a chunk holds two tiles
    constexpr int kOdd = UPC == 4 ? 2 : 0;
    for (int ot = 1; ot < kNT - 1; ot += 2) {
      ro_tile<MT, kOdd>(R, F, X, S, ot, g4, P, Q, pf, pb);
      ro_tile<MT, 0>(R, F, X, S, ot + 1, g4, P, Q, pf, pb);
    }
    ro_tile<MT, kOdd>(R, F, X, S, kNT - 1, g4, P, Q, pf, pb);
    {
      const f4 w2 = ldf4(S.w2 + 16 * (kNT - 1) + g4);
      ro_piece<MT, 0>(P, Q, w2, pf, pb);
      ro_piece<MT, 1>(P, Q, w2, pf, pb);
    }
    readout_finish<MT>(pf, pb, W.b2, ffwd, fbwd);
  }

  template <int MT>
  static __device__ __forceinline__ void gnn(const ChainW &W, const Small &S, R_t &R, Feed &F, float *park,
                                             const float (&feat)[MT], float (&ffwd)[MT], float (&fbwd)[MT]) {
    const int lane = R.lane;
    const int g4 = 4 * (lane >> 4);
    Acts<MT> X;
    f4 pend[MT][2];
    {
      f4 h[MT][kNT];
      input_layer<MT>(S, lane, feat, h);  // f32 MFMA, ReLU applied
#pragma unroll
      for (int kb = 0; kb < kKB; ++kb)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int t = k >> 1, r = 2 * (k & 1);
          float v0[MT], v1[MT], s0[MT], s1[MT];
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            v0[mt] = h[mt][2 * kb + t][r];
            v1[mt] = h[mt][2 * kb + t][r + 1];
            X.h[mt][kb][k] = pk_bf16(v0[mt], v1[mt]);
          }
          nb_sum<MT>(v0, s0);
          nb_sum<MT>(v1, s1);
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) X.a[mt][kb][k] = pk_bf16(s0[mt], s1[mt]);
        }
      if (W.layers == 0) {
        // no update layer: hand the readout the input layer's output the way
        // a last layer would (k-blocks 0..2 parked, tiles 6, 7 pending; ReLU is idempotent)
#pragma unroll
        for (int kb = 0; kb < 3; ++kb)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) *reinterpret_cast<u4 *>(park_at(park, kb, 0, mt, lane)) = X.h[mt][kb];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          pend[mt][0] = h[mt][6];
          pend[mt][1] = h[mt][7];
        }
      }
    }
    // message passing (src/flux_gnn.py:53-60), pair-pipelined
    if (W.layers > 0) {
      f4 acc0[MT][2];
      pair0_first<MT>(R, F, X, S.bl, g4, acc0);
      pairs_rest<MT>(R, F, X, S.bl, g4, acc0, pend, park, lane);
    }
    for (int l = 1; l < W.layers; ++l) {
      const float *bias = S.bl + l * kH;
      f4 acc0[MT][2];
      pair0_after<MT>(R, F, X, bias, g4, acc0, pend, park, lane);
      pairs_rest<MT>(R, F, X, bias, g4, acc0, pend, park, lane);
    }
    readout<MT>(W, S, R, F, X, pend, park, lane, g4, ffwd, fbwd);
  }
};

}  // namespace

hipError_t launch_chain_flux_bf16(const ChainW &w, const float *nf, const float *state, int64_t ld_state,
                                  const float *x, int B, int nx, float *fe, float *ff, hipStream_t s) {
  if (nx == 16 || nx == 32 || nx == 48 || nx == 64)
    return chain::launch_flux_core<CoreBF16T<4>>(w, nf, state, ld_state, x, B, nx, fe, ff, s);
  // windowed (e.g. cfg4's 1024 cells): 16 KiB chunks in 3 slots
  return chain::launch_flux_windowed<CoreBF16T<4, 4>>(w, nf, state, ld_state, x, B, nx, fe, ff, s);
}

hipError_t launch_chain_rollout_bf16(const ChainW &w, const float *state0, float *state_final, const float *x,
                                     const double *pc, int B, int nx, int T, float c, float dt, float *traj,
                                     float *flux_traj, float *metrics, const RolloutExtras &ex, hipStream_t s) {
  return chain::launch_rollout_core<CoreBF16T<4>>(w, state0, state_final, x, pc, B, nx, T, c, dt, traj, flux_traj,
                                              metrics, ex, s);
}

}  // namespace hf
