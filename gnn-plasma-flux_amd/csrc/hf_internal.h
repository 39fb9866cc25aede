// Internal declarations shared by the HIP translation units of libhybridflux.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hybridflux.h"

namespace hf {

// Width of the fused chain kernels: MODEL_CONFIG (src/config.py:19-23) is
// input_dim 4, hidden 128, 4 layers.  16x16x4 f32 MFMA tiles => 8 feature
// tiles of 16 and 32 k-steps of 4 per 128-wide half of a [h ; agg] input.
constexpr int kIn = 4;
constexpr int kH = 128;
constexpr int kNT = kH / 16;
constexpr int kKS = kH / 4;

// Window geometry of the halo-recompute chain kernel (any nx): a wave owns
// 64 consecutive cells; L update layers invalidate L cells at each window
// edge and the readout needs both cells of a face, so faces [L, 62 - L] of
// the window are exact.
constexpr int kWinCells = 64;
// exact faces per window of `cells` cells for L update layers: [L, cells - 2 - L]
// (55 at 64 cells and L = 4, 47 at L = 8)
__host__ __device__ inline int win_faces_of(int layers, int cells = kWinCells) { return cells - 2 * layers - 1; }

// Packed weights (device) for the chain kernels; see capi.cpp pack_chain_*
// for the exact index maps.  The big matrices form ONE stream of chunks,
// consumed in order through an LDS ring (chain_common.h):
//  f32   (v_mfma_f32_16x16x4_f32): 8 KiB chunks, 16 per update layer (4 k-steps
//        each, [h ; agg] input order) + 2 per readout output tile.
//  k32   (v_mfma_f32_16x16x32_{f16,bf16}): per update layer 8 chunks, then one
//        chunk per readout output tile, in the order the cores walk a layer:
//        output pair, then k-block.  f16x3: 16 KiB of (hi, lo) fp16 fragment
//        pairs; bf16: 8 KiB.  (A core may move two chunks at once.)
// Each chunk is [fragment j][lane 64][16 B], so one wave instruction moves 1 KiB.
enum ChainPrec { kPrecF32 = HF_WDTYPE_F32, kPrecBF16 = HF_WDTYPE_BF16, kPrecF16x3 = HF_WDTYPE_F16X3 };
constexpr int kMaxChainLayers = 8;

// Poisson by float64 FFT for power-of-two nx in [kFftMinNx, kFftMaxNx] (fv_poisson.hip).
constexpr int kFftMinNx = 256;
constexpr int kFftMaxNx = 2048;
__host__ __device__ inline bool poisson_uses_fft(int nx) {
  return nx >= kFftMinNx && nx <= kFftMaxNx && (nx & (nx - 1)) == 0;
}
__host__ __device__ inline int poisson_plan_len(int nx) { return poisson_uses_fft(nx) ? 3 * nx : nx; }
// Poisson mode of every FV/Poisson launcher below (pm): HF_POISSON_SPECTRAL
// (the reference's operator; its plan is hf_poisson_coeffs) or
// HF_POISSON_TRIDIAG (opt-in, not the reference's; plan = {dx/2}; one wave's
// cyclic reduction over an LDS row of nx doubles, so nx <= kTriMaxNx).
constexpr int kTriMaxNx = 16384;  // 128 KiB of LDS
bool poisson_mode_ok(int pm, int nx);

__host__ __device__ inline int chain_chunks(int layers, int prec) {
  return prec == kPrecF32 ? 16 * layers + 2 * kNT : 8 * layers + kNT;
}
__host__ __device__ inline int chain_chunk_bytes(int prec) { return prec == kPrecF16x3 ? 16384 : 8192; }
// bf16 streams end with a copy of their first kBF16StreamTail bytes (two 4 KiB units)
constexpr int kBF16StreamTail = 8192;

struct ChainW {
  const void *stream;   // [chain_chunks][chunk]
  const float *win;     // [2][64][4]   input layer A fragments (f32; bf16-rounded in bf16 mode)
  const float *bin;     // [kH]
  const float *bl;      // [L][kH]
  const float *be;      // [kH]
  const float *w2;      // [kH]
  float b2;
  int layers;
  int prec;             // ChainPrec
};

// Natural-layout float32 weights (device) for the generic-graph path.
struct GraphW {
  const float *w_in, *b_in;        // [H][in], [H]
  const float *w_l, *b_l;          // layer l: w_l + l*lsw [H][2H], b_l + l*lsb [H]
  const float *w_e, *b_e;          // [H][2H], [H]
  const float *w_2, *b_2;          // [H], [1]
  int in_dim, hidden, layers;
  int64_t lsw, lsb;                // per-layer strides (grouped or state-dict order)
};
// Strided weight view for the generic MFMA GEMM (graph.hip):
// weight(o, k) = k < K1 ? w1[o*so + k*si] : w2[o*so + (k-K1)*si].
struct WView {
  const float *w1, *w2;
  int64_t so, si;
};
inline WView wv_rows(const float *W, int K1, int K) { return {W, W + K1, K, 1}; }  // nn.Linear [O][K]
inline WView wv_t(const float *W, int Kf) { return {W, W, 1, Kf}; }              // W^T of [Kf'][Kf]
enum { kActNone = 0, kActRelu = 1, kActTanh = 2 };
// out[m][o] = resid[m][o] + act(b[o] + sum_k weight(o,k) in(m,k)), in(m,k) = [A1[i1(m)] ; A2[i2(m)]][k].
hipError_t gemm_linear(const float *A1, int K1, const int64_t *i1, const float *A2, int K2, const int64_t *i2,
                       WView W, const float *b, float *out, int64_t M, int O, int act, const float *resid,
                       hipStream_t s);
// Edges bucketed by key (row or col), ascending edge id per bucket; chain_nx > 0: arithmetic buckets.
int64_t edge_buckets_bytes(int64_t N, int64_t E);
hipError_t edge_buckets(const int64_t *key, int64_t E, int64_t N, int chain_nx, bool by_col, void *ws, int **off,
                        int **perm, hipStream_t s);

// PureGNN / PINN inference (baselines.hip).
int64_t pure_gnn_ws_bytes(int H, int64_t N, int64_t E);
hipError_t launch_pure_gnn_forward(const float *params, int in_dim, int H, int L, const float *nf, int64_t N,
                                   const int64_t *ei, int64_t E, int chain_nx, float *delta, void *ws, hipStream_t s);
hipError_t launch_pure_gnn_run(const float *params, int H, int L, const float *state0, float *final_state,
                               const float *x, int B, int nx, int T, float *traj, void *ws, hipStream_t s);
int64_t pinn_ws_bytes(int D, int H, int64_t B);
// scratch the rollouts actually use: the packed weights on their one-launch paths (baselines.hip)
int64_t pure_gnn_run_ws_bytes(int H, int B, int nx, int T);
// the one-launch PureGNN rollout also runs with no workspace (on nn.Linear's rows, unpacked)
bool pure_gnn_run_ws_optional(int H, int nx, int T);
int64_t pinn_run_ws_bytes(int D, int H, int64_t B);
hipError_t launch_pinn_forward(const float *params, int D, int H, int L, const float *state, float *out, int64_t B,
                               void *ws, hipStream_t s);
hipError_t launch_pinn_run(const float *params, int D, int H, int L, const float *state0, float *final_state,
                           int64_t B, int T, float *traj, void *ws, hipStream_t s);

// View of a flat float32 parameter buffer in state-dict order (the host_params
// order of hf_model_create): update layers interleave weight and bias.
GraphW graph_view_state_dict(const float *p, int in_dim, int hidden, int layers);

// Per-precision launchers (chain_f32.hip, chain_k32.hip = f16x3, chain_bf16.hip); the generic entry
// points below dispatch on ChainW::prec.
hipError_t launch_chain_flux_f32(const ChainW &, const float *, const float *, int64_t, const float *, int, int,
                                 float *, float *, hipStream_t);
hipError_t launch_chain_flux_k32(const ChainW &, const float *, const float *, int64_t, const float *, int, int,
                                 float *, float *, hipStream_t);
hipError_t launch_chain_flux_bf16(const ChainW &, const float *, const float *, int64_t, const float *, int, int,
                                  float *, float *, hipStream_t);
// Extra outputs of the persistent rollout: a classical twin of every IC
// stepped in the same wave (hf_run_compare), all optional.
struct RolloutExtras {
  float nu = 0.f, dx2 = 1.f;        // classical viscosity and f32(dx*dx)
  float *mse = nullptr;             // [B][T+1][3]; non-null enables the twin
  float *metrics_cl = nullptr;      // [B][T+1][HF_NUM_METRICS]
  int poisson = HF_POISSON_SPECTRAL;  // Poisson mode (pm) of the hybrid step and the twin
};
hipError_t launch_chain_rollout_f32(const ChainW &, const float *, float *, const float *, const double *, int, int,
                                    int, float, float, float *, float *, float *, const RolloutExtras &,
                                    hipStream_t);
// Cell-split rollout for small batches (chain_f32.hip; f32, nx in {32,48,64}, no classical twin).
bool chain_rollout_prefers_cells(const ChainW &, int B, int nx);
hipError_t launch_chain_rollout_cells(const ChainW &, const float *, float *, const float *, const double *, int,
                                      int, int, float, float, float *, float *, float *, int pm, hipStream_t);
hipError_t launch_chain_rollout_k32(const ChainW &, const float *, float *, const float *, const double *, int, int,
                                    int, float, float, float *, float *, float *, const RolloutExtras &,
                                    hipStream_t);
hipError_t launch_chain_rollout_bf16(const ChainW &, const float *, float *, const float *, const double *, int, int,
                                     int, float, float, float *, float *, float *, const RolloutExtras &,
                                     hipStream_t);

// Chain flux.  Feature source: AoS node features [B*nx][4] (nf != nullptr)
// or SoA state [B][3][nx] with IC stride ld_state floats + x[nx].
inline hipError_t launch_chain_flux(const ChainW &w, const float *nf, const float *state, int64_t ld_state,
                                    const float *x, int B, int nx, float *flux_edge, float *flux_face,
                                    hipStream_t s) {
  return w.prec == kPrecF32 ? launch_chain_flux_f32(w, nf, state, ld_state, x, B, nx, flux_edge, flux_face, s)
                            : launch_chain_flux_k32(w, nf, state, ld_state, x, B, nx, flux_edge, flux_face, s);
}

// Work of one step of the per-step flux kernel for B ICs of nx cells, in the
// persistent kernel's own units, and how many units one round of its resident
// workgroups takes (hf_run's lanes cut the batch at whole rounds).  Known for
// the bf16 super-window kernel (chain_bf16.hip); per_round = 0 otherwise.
struct FluxWork {
  int64_t units = 0, per_round = 0;
};
FluxWork chain_flux_work(const ChainW &w, int64_t B, int nx);

// Persistent fused rollout for nx in {16,32,48,64}.
inline hipError_t launch_chain_rollout(const ChainW &w, const float *state0, float *state_final,
                                       const float *x, const double *pc, int B, int nx, int T, float c,
                                       float dt, float *traj, float *flux_traj, float *metrics,
                                       hipStream_t s, const RolloutExtras &ex = RolloutExtras()) {
  return w.prec == kPrecF32
             ? launch_chain_rollout_f32(w, state0, state_final, x, pc, B, nx, T, c, dt, traj, flux_traj, metrics,
                                        ex, s)
             : launch_chain_rollout_k32(w, state0, state_final, x, pc, B, nx, T, c, dt, traj, flux_traj, metrics,
                                        ex, s);
}

// Per-step channel MSE between two trajectories [B][T+1][3][nx] -> [B][T+1][3].
hipError_t launch_traj_mse(const float *a, const float *b, int B, int T1, int nx, float *mse, hipStream_t s);
hipError_t launch_rollout_summary(const float *met, const float *mse, const float *met_ref, int B, int T,
                                  float *summary, float *drift, hipStream_t s);

// One FV + Poisson update (any nx).  face_flux != nullptr => hybrid update
// with that F; nullptr => classical (F = n*u, viscosity).  IC strides in floats.
hipError_t launch_fv_step(const float *in, int64_t ld_in, float *out, int64_t ld_out,
                          const float *face_flux, const double *pc, int B, int nx, float c,
                          float dt, float nu, float dx2, float *flux_out, int64_t ld_flux,
                          float *metrics, int64_t ld_metrics, int pm, hipStream_t s);

// The whole classical rollout (T steps of launch_fv_step's classical update)
// in one launch, states held in registers: FFT nx up to 1024 (fv_run_fused).
// state0 [B] x IC stride ld_s0 floats, state_final [B][3][nx] (may alias
// state0, may be NULL); traj [B][T+1][3][nx] rows 1..T, flux_traj [B][T][nx],
// metrics [B][T+1][4] rows 1..T, each optional; ref + mse (both or neither):
// per-step channel MSE [B][T+1][3] of ref [B][T+1][3][nx] minus this rollout,
// rows 0..T, bit-identical to launch_traj_mse on the recorded trajectory.
bool fv_run_fused(int nx);
hipError_t launch_fv_run(const float *state0, int64_t ld_s0, float *state_final, float *traj, const double *pc, int B,
                         int nx, int T, float c, float dt, float nu, float dx2, float *flux_traj, float *metrics,
                         const float *ref, float *mse, int pm, hipStream_t s);

// Metrics of a state batch (used for t=0 of non-fused rollouts).
hipError_t launch_state_metrics(const float *st, int64_t ld, int B, int nx, float *metrics,
                                int64_t ld_metrics, hipStream_t s);

hipError_t launch_poisson(const float *n, int ld_n, float *E, int ld_E, const double *pc, int B,
                          int nx, int pm, hipStream_t s);

int64_t graph_workspace_bytes(const GraphW &w, int64_t N, int64_t E);
// Training forward (activation tape) and backward, graph_train section of graph.hip.
int64_t graph_tape_bytes(const GraphW &w, int64_t N, int64_t E);
int64_t graph_backward_ws_bytes(const GraphW &w, int64_t N, int64_t E);
hipError_t launch_graph_forward_train(const GraphW &w, const float *nf, int64_t N, const int64_t *ei, int64_t E,
                                      int chain_nx, float *flux, void *tape, hipStream_t s);
hipError_t launch_graph_backward(const GraphW &w, const float *nf, int64_t N, const int64_t *ei, int64_t E,
                                 int chain_nx, const void *tape, const float *grad_flux, float *grad_params, float *grad_nf,
                                 void *ws, hipStream_t s);
// Chain-specialised training path (train_chain.hip): tagged chain graphs
// (chain_nx > 0) with hidden a power of two in [32, 256], in_dim <= 8 and
// N * 2 * hidden + 2 * hidden < 2^31; other graphs and widths take the
// generic CSR path.
bool chain_train_ok(const GraphW &w, int chain_nx, int64_t N);
int64_t chain_tape_bytes(const GraphW &w, int64_t N);
int64_t chain_backward_ws_bytes(const GraphW &w, int64_t N);
hipError_t launch_chain_forward_train(const GraphW &w, const float *nf, int64_t N, int nx, float *flux, void *tape,
                                      hipStream_t s);
hipError_t launch_chain_backward(const GraphW &w, const float *nf, int64_t N, int nx, const void *tape,
                                 const float *grad_flux, float *grad_params, float *grad_nf, void *ws, hipStream_t s);
// Fused training path (chain_f32.hip): FluxGNN(4, 128, L <= 8) on chains of
// nx in {16, 32, 48, 64}.  Forward: the flux kernel's IC-per-wave pass,
// storing the tape (h[l] at h0 + l * hstride, pq) and the ReLU' bits of
// h[0..L-1] (chain_train_mask_bytes); `pack` holds chain_train_pack_bytes(L)
// of device-packed weights.  Backward: the update layers' data gradients
// g[L-1..0] from g[L] (g[l] at g0 + l * gstride), or (dPQ non-NULL) from the
// readout's dP / dQ, g[L] included; `pack` holds chain_train_bwd_pack_bytes(L)
// of transposed weights.
bool chain_train_fused_ok(const GraphW &w, int nx);
int64_t chain_train_pack_bytes(int layers);
int64_t chain_train_mask_bytes(int layers, int64_t N);
int64_t chain_train_bwd_pack_bytes(int layers);
// bpack (forward): also pack the backward's stream there (chain_train_bwd_pack_bytes(L);
// ro: with the readout's [W_a^T | W_b^T] first, as the backward's dPQ form needs),
// in the same launch; the backward then takes it with prepacked.
hipError_t launch_chain_train_fwd_fused(const GraphW &w, const float *nf, int64_t B, int nx, float *fe, float *h0,
                                        int64_t hstride, float *pq, unsigned *mbits, void *pack, hipStream_t s,
                                        void *bpack = nullptr, int ro = 0);
hipError_t launch_chain_train_bwd_fused(const GraphW &w, int64_t B, int nx, float *g0, int64_t gstride,
                                        const unsigned *mbits, void *pack, const float *dPQ, hipStream_t s,
                                        const float *pq = nullptr, const float *gflux = nullptr,
                                        const float *w2 = nullptr, float *epart = nullptr, bool prepacked = false);
// The ablation loss's single-step terms and d loss / d flux_edge (train_chain.hip).
int64_t ablation_loss_ws_bytes(int B, int nx);
hipError_t launch_ablation_loss(const float *fe, const float *st, const float *ft, const float *sn, int B, int nx,
                                float c, float dx, const float *lam, int roll, float dt, const double *pc, float *loss,
                                float *flux_loss, float *dfe, void *ws, hipStream_t s);
constexpr int kLossMaxRollout = 3;  // rollout energy term in the loss kernels: rollout_steps <= 3
// The trainer's batch gather + chain node features (train_chain.hip).
hipError_t launch_chain_batch_gather(const int64_t *idx, int B, const float *st_all, const float *ft_all,
                                     const float *sn_all, int64_t N, int nx, const float *x, float *st, float *ft,
                                     float *sn, float *nf, hipStream_t s);
// Adam over one flat parameter buffer, step count on the device (train_chain.hip).
hipError_t launch_adam_flat(float *p, const float *g, float *m, float *v, int64_t n, float *step, unsigned *done,
                            float lr, float b1, float b2, float eps, hipStream_t s);
hipError_t launch_graph_flux(const GraphW &w, const float *nf, int64_t N, const int64_t *ei,
                             int64_t E, float *flux, void *ws, hipStream_t s);

}  // namespace hf
