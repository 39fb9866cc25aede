// Fused FluxGNN on the periodic chain on the K=32 matrix cores:
// v_mfma_f32_16x16x32_f16 (mode F16x3) and v_mfma_f32_16x16x32_bf16 (BF16).
//
// Reference: src/flux_gnn.py:40-67, src/hybrid_solver.py:34-73.
//
// F16x3 keeps float32-level accuracy at ~5x the f32 MFMA rate: every weight
// and every activation is split into two fp16 terms, x = x_hi + x_lo with
// x_hi = fp16(x), x_lo = fp16(x - x_hi) (22 significant bits), and each
// product is accumulated in f32 as a_hi b_hi + a_hi b_lo + a_lo b_hi (the
// dropped a_lo b_lo is 2^-22 relative).  Measured against an fp64 evaluation
// the edge fluxes carry 5.4e-7 error, the same as the reference's own float32
// CPU evaluation (4.7e-7).  BF16 (BASELINE config 4) is a single bf16 product
// with bf16-rounded weights and activations.
//
// Fragments: for 16x16x32, lane l holds A[row l&15][k = 8(l>>4) + e] and
// B[k = 8(l>>4) + e][col l&15], e = 0..7.  The B fragment of k-block kb is the
// two 16x16 accumulator tiles 2kb, 2kb+1 of the previous layer (features
// 16(2kb + (e>>2)) + 4(l>>4) + (e&3)): the activations never leave registers
// and the host packs the weights in the same permuted k order.
//
// Aggregation by linearity: W_b (h[i+1] + h[i-1]) / 2 = (G[i+1] + G[i-1]) / 2
// with G = W_b h, so the split activations of a k-block feed both W_a and W_b
// and the neighbour lane shifts run once per layer on the G accumulators.
#include "chain_common.h"

namespace hf {
namespace {

using namespace chain;

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f8 __attribute__((ext_vector_type(8)));

struct ModeF16x3 {
  static constexpr int kNS = 2;              // fp16 terms per operand
  [[maybe_unused]] static constexpr int kMma = 3;  // MFMAs per product
  static constexpr int kChunkFloats = 4096;  // 16 KiB
  using T = h8;
  static __device__ __forceinline__ void split(const f8 &v, T (&o)[kNS]) {
    o[0] = __builtin_convertvector(v, h8);
    const f8 r = v - __builtin_convertvector(o[0], f8);  // exact: v and hi share the leading bits
    o[1] = __builtin_convertvector(r, h8);
  }
  // a_lo b_hi + a_hi b_lo + a_hi b_hi, small terms first
  static __device__ __forceinline__ f4 mma(const T (&a)[kNS], const T (&b)[kNS], f4 c) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[1], b[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[1], c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a[0], b[0], c, 0, 0, 0);
  }
};

template <class M>
struct CoreK32 {
  static constexpr int kNW = kWaves;   // waves sharing the weight ring
  static constexpr int kSlots = kRingSlots;
  static constexpr int kWinMT = 4;     // m-tiles per wave in the windowed flux kernel
  static constexpr int kChunkFloats = M::kChunkFloats;
  // first output half of a layer parked in LDS while the second half runs:
  // [mt 4][tile 4][lane 64][4] floats per wave
  static constexpr int kParkFloats = 4 * 4 * 64 * 4;
  static constexpr int kNS = M::kNS;
  static constexpr int kKB = kH / 32;  // k-blocks per 128-wide operand
  using T = typename M::T;
  using R_t = Ring<kChunkFloats>;

  struct Frag {
    T v[kNS];
  };
  struct Feed {};  // fragments are read per chunk (no register prefetch)
  static __device__ __forceinline__ void begin(R_t &, Feed &) {}

  static __device__ __forceinline__ Frag lds_frag(const float *slot, int j, int lane) {
    Frag f;
#pragma unroll
    for (int s = 0; s < kNS; ++s)
      f.v[s] = __builtin_bit_cast(T, ldf4(slot + ((j * kNS + s) * 64 + lane) * 4));
    return f;
  }

  // Activation tiles (2kb, 2kb+1) as the split B fragment of k-block kb.
  static __device__ __forceinline__ void frag_of(const f4 &a, const f4 &b, Frag &o) {
    const f8 v = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    M::split(v, o.v);
  }
  template <int MT>
  static __device__ __forceinline__ void to_frags(const f4 (&h)[MT][kNT], Frag (&B)[MT][kKB]) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int kb = 0; kb < kKB; ++kb) frag_of(h[mt][2 * kb], h[mt][2 * kb + 1], B[mt][kb]);
  }

  // Update-layer chunk (NTH, KB): W_a and W_b fragments of output tiles
  // 4*NTH .. 4*NTH+3 over k-block KB.  Fragment j = 2*ntl + (0: W_a, 1: W_b).
  template <int MT, int KB>
  static __device__ __forceinline__ void layer_chunk(R_t &R, const Frag (&B)[MT][kKB], f4 (&acc)[MT][4],
                                                     f4 (&gac)[MT][4]) {
    const float *slot = R.next();
#pragma unroll
    for (int ntl = 0; ntl < 4; ++ntl) {
      const Frag wa = lds_frag(slot, 2 * ntl, R.lane);
      const Frag wb = lds_frag(slot, 2 * ntl + 1, R.lane);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        acc[mt][ntl] = M::mma(wa.v, B[mt][KB].v, acc[mt][ntl]);
        gac[mt][ntl] = M::mma(wb.v, B[mt][KB].v, gac[mt][ntl]);
      }
    }
  }

  // h_new = ReLU(acc + (G[i+1] + G[i-1]) / 2) for one half of the output
  // tiles; the bias is already in acc (the C operand of its first MFMA).
  template <int MT>
  static __device__ __forceinline__ void layer_epilogue(const f4 (&acc)[MT][4], const f4 (&gac)[MT][4],
                                                        f4 (&out)[MT][4]) {
#pragma unroll
    for (int ntl = 0; ntl < 4; ++ntl) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float gv[MT], gs[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) gv[mt] = gac[mt][ntl][r];
        nb_sum<MT>(gv, gs);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          // acc + 0.5*(G[i+1] + G[i-1]): one rounding either way, 0.5*x is exact
          out[mt][ntl][r] = relu(fmaf(gs[mt], 0.5f, acc[mt][ntl][r]));
        }
      }
    }
  }

  template <int MT, int NTH>
  static __device__ __forceinline__ void layer_half(R_t &R, const Frag (&B)[MT][kKB], const float *bias, int g4,
                                                    f4 (&out)[MT][4]) {
    f4 acc[MT][4], gac[MT][4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const f4 b = ldf4(bias + 64 * NTH + 16 * n + g4);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        acc[mt][n] = b;
        gac[mt][n] = f4{0.f, 0.f, 0.f, 0.f};
      }
    }
    layer_chunk<MT, 0>(R, B, acc, gac);
    layer_chunk<MT, 1>(R, B, acc, gac);
    layer_chunk<MT, 2>(R, B, acc, gac);
    layer_chunk<MT, 3>(R, B, acc, gac);
    layer_epilogue<MT>(acc, gac, out);
  }

  // Readout chunk for output tile ot: fragment j = 2*kb + (0: P, 1: Q).
  template <int MT>
  static __device__ __forceinline__ void readout_chunk(R_t &R, const Frag (&B)[MT][kKB], f4 (&P)[MT], f4 (&Q)[MT]) {
    const float *slot = R.next();
#pragma unroll
    for (int kb = 0; kb < kKB; ++kb) {
      const Frag wp = lds_frag(slot, 2 * kb, R.lane);
      const Frag wq = lds_frag(slot, 2 * kb + 1, R.lane);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        P[mt] = M::mma(wp.v, B[mt][kb].v, P[mt]);
        Q[mt] = M::mma(wq.v, B[mt][kb].v, Q[mt]);
      }
    }
  }

  template <int MT>
  static __device__ __forceinline__ void gnn(const ChainW &W, const Small &S, R_t &R, Feed &, float *park,
                                             const float (&feat)[MT], float (&ffwd)[MT], float (&fbwd)[MT]) {
    const int lane = R.lane;
    const int g4 = 4 * (lane >> 4);
    Frag B[MT][kKB];
    {
      f4 h[MT][kNT];
      input_layer<MT>(S, lane, feat, h);
      to_frags<MT>(h, B);
    }
    // message passing (src/flux_gnn.py:53-60)
    for (int l = 0; l < W.layers; ++l) {
      const float *bias = S.bl + l * kH;
      {
        f4 lo[MT][4];
        layer_half<MT, 0>(R, B, bias, g4, lo);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int n = 0; n < 4; ++n) *reinterpret_cast<f4 *>(park + ((mt * 4 + n) * 64 + lane) * 4) = lo[mt][n];
      }
      {
        f4 hi[MT][4];
        layer_half<MT, 1>(R, B, bias, g4, hi);
        // new B fragments one k-block at a time (the old ones are dead now):
        // k-blocks 2, 3 from registers, then 0, 1 from the park, so f32
        // activations and fragments are never all live at once
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          frag_of(hi[mt][0], hi[mt][1], B[mt][2]);
          frag_of(hi[mt][2], hi[mt][3], B[mt][3]);
        }
      }
      wave_lds_sync();
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          frag_of(ldf4(park + ((mt * 4 + 2 * kb) * 64 + lane) * 4),
                  ldf4(park + ((mt * 4 + 2 * kb + 1) * 64 + lane) * 4), B[mt][kb]);
    }
    // edge readout, P/Q split (src/flux_gnn.py:62-66)
    float pf[MT], pb[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) pf[mt] = pb[mt] = 0.f;
    for (int ot = 0; ot < kNT; ++ot) {
      f4 P[MT], Q[MT];
      const f4 be = ldf4(S.be + 16 * ot + g4);  // b_e enters P as the C operand of its first MFMA
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        P[mt] = be;
        Q[mt] = f4{0.f, 0.f, 0.f, 0.f};
      }
      readout_chunk<MT>(R, B, P, Q);
      readout_epilogue<MT, true>(P, Q, be, ldf4(S.w2 + 16 * ot + g4), pf, pb);
    }
    readout_finish<MT>(pf, pb, W.b2, ffwd, fbwd);
  }
};

}  // namespace

hipError_t launch_chain_flux_k32(const ChainW &w, const float *nf, const float *state, int64_t ld_state,
                                 const float *x, int B, int nx, float *fe, float *ff, hipStream_t s) {
  if (w.prec == kPrecF16x3)
    return chain::launch_flux_core<CoreK32<ModeF16x3>>(w, nf, state, ld_state, x, B, nx, fe, ff, s);
  return launch_chain_flux_bf16(w, nf, state, ld_state, x, B, nx, fe, ff, s);
}

hipError_t launch_chain_rollout_k32(const ChainW &w, const float *state0, float *state_final, const float *x,
                                    const double *pc, int B, int nx, int T, float c, float dt, float *traj,
                                    float *flux_traj, float *metrics, const RolloutExtras &ex, hipStream_t s) {
  if (w.prec == kPrecF16x3)
    return chain::launch_rollout_core<CoreK32<ModeF16x3>>(w, state0, state_final, x, pc, B, nx, T, c, dt, traj,
                                                          flux_traj, metrics, ex, s);
  return launch_chain_rollout_bf16(w, state0, state_final, x, pc, B, nx, T, c, dt, traj, flux_traj, metrics, ex,
                                   s);
}

}  // namespace hf
