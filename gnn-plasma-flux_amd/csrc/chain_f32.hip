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

struct CoreF32 {
  static constexpr int kChunkFloats = 2048;  // 8 KiB: 4 k-steps x 8 tiles, or 16 k-steps x (P, Q)
  static constexpr int kParkFloats = 0;
  using R_t = Ring<kChunkFloats>;

  static __device__ __forceinline__ void read_chunk(const float *slot, int lane, f4 (&v)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = ldf4(slot + (j * 64 + lane) * 4);
  }

  // One update-layer chunk: k-steps s = 4*gi + q.  The first 8 chunks of a
  // layer read h itself, the last 8 the neighbour mean (h[i+1] + h[i-1]) / 2.
  template <int MT, int GI>
  static __device__ __forceinline__ void layer_chunk(R_t &R, const f4 (&h)[MT][kNT], f4 (&acc)[MT][kNT]) {
    f4 v[8];
    read_chunk(R.next(), R.lane, v);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      constexpr int kHalf = kKS / 4;
      const int s = (GI % kHalf) * 4 + q;  // k-step within its 128-wide half
      float b[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) b[mt] = h[mt][s >> 2][s & 3];
      if (GI >= kHalf) {
        float sum[MT];
        nb_sum<MT>(b, sum);  // index_add_ of h[i+1], h[i-1]
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) b[mt] = __fmul_rn(sum[mt], 0.5f);  // / deg 2 (exact)
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < kNT; ++nt) acc[mt][nt] = mfma4(v[2 * q + (nt >> 2)][nt & 3], b[mt], acc[mt][nt]);
    }
  }

  // One readout chunk: k-steps s = 16*HH + qq for P (W_e[:, :H]) and Q (W_e[:, H:]).
  template <int MT, int HH>
  static __device__ __forceinline__ void readout_chunk(R_t &R, const f4 (&h)[MT][kNT], f4 (&P)[MT], f4 (&Q)[MT]) {
    f4 v[8];
    read_chunk(R.next(), R.lane, v);
#pragma unroll
    for (int qq = 0; qq < 16; ++qq) {
      const int s = 16 * HH + qq;
      const float ap = v[qq >> 1][2 * (qq & 1)], aq = v[qq >> 1][2 * (qq & 1) + 1];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const float b = h[mt][s >> 2][s & 3];
        P[mt] = mfma4(ap, b, P[mt]);
        Q[mt] = mfma4(aq, b, Q[mt]);
      }
    }
  }

  // FluxGNN forward for the MT*16 cells of this wave.  feat[mt] is the lane's
  // input feature (index l>>4 of [n,u,E,x]) of cell 16*mt + (l&15).  Returns
  // the edge fluxes of (i -> i+1) in ffwd and of (i+1 -> i) in fbwd for cell
  // i, on every lane of the cell's column.  Consumes one pass of the stream.
  template <int MT>
  static __device__ __forceinline__ void gnn(const ChainW &W, const Small &S, R_t &R, float * /*park*/,
                                             const float (&feat)[MT],
                                             float (&ffwd)[MT], float (&fbwd)[MT]) {
    const int lane = R.lane;
    const int g4 = 4 * (lane >> 4);
    f4 h[MT][kNT];
    input_layer<MT>(S, lane, feat, h);

    // message passing: h = ReLU(W_l [h ; (h[i+1]+h[i-1])/2] + b_l)        (src/flux_gnn.py:53-60)
    for (int l = 0; l < W.layers; ++l) {
      f4 acc[MT][kNT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < kNT; ++nt) acc[mt][nt] = f4{0.f, 0.f, 0.f, 0.f};
      layer_chunk<MT, 0>(R, h, acc);
      layer_chunk<MT, 1>(R, h, acc);
      layer_chunk<MT, 2>(R, h, acc);
      layer_chunk<MT, 3>(R, h, acc);
      layer_chunk<MT, 4>(R, h, acc);
      layer_chunk<MT, 5>(R, h, acc);
      layer_chunk<MT, 6>(R, h, acc);
      layer_chunk<MT, 7>(R, h, acc);
      layer_chunk<MT, 8>(R, h, acc);
      layer_chunk<MT, 9>(R, h, acc);
      layer_chunk<MT, 10>(R, h, acc);
      layer_chunk<MT, 11>(R, h, acc);
      layer_chunk<MT, 12>(R, h, acc);
      layer_chunk<MT, 13>(R, h, acc);
      layer_chunk<MT, 14>(R, h, acc);
      layer_chunk<MT, 15>(R, h, acc);
#pragma unroll
      for (int nt = 0; nt < kNT; ++nt) {
        const f4 bias = ldf4(S.bl + l * kH + 16 * nt + g4);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) h[mt][nt] = relu4(acc[mt][nt] + bias);
      }
    }

    // edge readout, P/Q split (src/flux_gnn.py:62-66)
    float pf[MT], pb[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) pf[mt] = pb[mt] = 0.f;
    for (int ot = 0; ot < kNT; ++ot) {
      f4 P[MT], Q[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) P[mt] = Q[mt] = f4{0.f, 0.f, 0.f, 0.f};
      readout_chunk<MT, 0>(R, h, P, Q);
      readout_chunk<MT, 1>(R, h, P, Q);
      readout_epilogue<MT>(P, Q, ldf4(S.be + 16 * ot + g4), ldf4(S.w2 + 16 * ot + g4), pf, pb);
    }
    readout_finish<MT>(pf, pb, W.b2, ffwd, fbwd);
  }
};

}  // namespace

hipError_t launch_chain_flux_f32(const ChainW &w, const float *nf, const float *state, int64_t ld_state,
                                 const float *x, int B, int nx, float *fe, float *ff, hipStream_t s) {
  return chain::launch_flux_core<CoreF32>(w, nf, state, ld_state, x, B, nx, fe, ff, s);
}

hipError_t launch_chain_rollout_f32(const ChainW &w, const float *state0, float *state_final, const float *x,
                                    const double *pc, int B, int nx, int T, float c, float dt, float *traj,
                                    float *flux_traj, float *metrics, const RolloutExtras &ex, hipStream_t s) {
  return chain::launch_rollout_core<CoreF32>(w, state0, state_final, x, pc, B, nx, T, c, dt, traj, flux_traj,
                                             metrics, ex, s);
}

}  // namespace hf
