/*
 * hybridflux.h — C ABI of the MI355X hybrid-rollout engine (libhybridflux.so).
 *
 * Drop-in boundary for the hot path of shanedirksen/gnn-plasma-flux: the
 * per-timestep loop  FluxGNN message passing on the periodic 1-D chain
 * -> flux symmetrisation -> finite-volume continuity + Burgers update ->
 * spectral Poisson solve.  The reference has no FFI of its own (it is pure
 * Python); each entry point below names the reference function it replaces
 * (paths relative to the reference root).  The Python host layer
 * (gnn-plasma-flux_amd/hybridflux) binds these through ctypes; INTEGRATION.md
 * shows the binding.
 *
 * Conventions
 *  - Every pointer named dev_* is a device (HBM) pointer; host_* are host.
 *  - Layouts: state [B][3][nx] float32 (n,u,E per IC, channel-major, the
 *    reference's [3,nx] per IC); node features [N][in_dim] float32 (AoS, as
 *    FluxGNN.forward receives them); edge fluxes [B][2*nx] in the reference
 *    edge order (edges i->i+1 first, then i+1->i).
 *  - Work is enqueued on `stream` (a hipStream_t, NULL = default stream) and
 *    is asynchronous: nothing here synchronises the host.
 *  - Return 0 on success, a negative HF_E* code on failure; the message is
 *    available from hf_last_error() (thread-local).  Nothing throws across
 *    the ABI.  There is NO CPU fallback: without a usable gfx950 device every
 *    compute entry point fails with HF_EHIP.
 *  - Ownership: the caller owns every state/flux/trajectory/metric buffer.
 *    A model handle owns only its packed, read-only device weights, so
 *    concurrent calls on one handle from different streams are safe.
 */
#ifndef HYBRIDFLUX_H
#define HYBRIDFLUX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HF_OK 0
#define HF_EINVAL (-1)      /* bad argument (shape, NULL pointer, size)        */
#define HF_EUNSUPPORTED (-2)/* configuration this build does not implement    */
#define HF_EHIP (-3)        /* HIP runtime error (no device, launch failure)  */
#define HF_ENOMEM (-4)      /* device allocation failed                       */

#define HF_WDTYPE_F32 0     /* weights and arithmetic in float32 (parity mode) */
#define HF_WDTYPE_BF16 1    /* bf16 MLP weights/activations, f32 accumulate    */
#define HF_WDTYPE_F16X3 2   /* fp32-accurate: fp16 hi+lo split of weights and
                               activations, 3 MFMA products, f32 accumulate   */

/* Number of per-(IC, step) rollout metrics written by hf_run / hf_step /
 * hf_run_compare / hf_traj_metrics:
 * [0] energy 0.5*mean(u^2+E^2)   (scripts/evaluation/evaluate_all.py:135,
 *                                  evaluate_long_rollout.py:38-42)
 * [1] charge mean(n)              (evaluate_all.py:141)
 * [2] 1.0 if every state value is finite else 0.0
 *                                 (evaluate_long_rollout.py:57-60)
 * [3] max |n-1| over the chain (NaN when [2] is 0; no reference counterpart).
 * Sums are float64, rounded to float32 once. */
#define HF_NUM_METRICS 4

/* Per-IC rollout summary written by hf_rollout_summary:
 * [0] exploded_at: first step t >= 1 whose state is not finite, -1 if none
 *     (evaluate_long_rollout.py:53-66)
 * [1] actual_steps: exploded_at - 1, or T (evaluate_long_rollout.py:74)
 * [2] final energy drift |e[a] - e[0]|, a = actual_steps
 *     (evaluate_long_rollout.py:72; evaluate_all.py:137,157)
 * [3] final charge drift |q[a] - q[0]| (evaluate_all.py:143,158)
 * [4] final_mse = mse_total[T], mse_total = mse_n + mse_u + mse_E
 *     (evaluate_all.py:132,155); NaN without an MSE series
 * [5] mean_mse = mean over t = 0..T of mse_total (evaluate_all.py:156,
 *     evaluate_multi_ic.py:91-94); NaN without an MSE series
 * [6], [7] final energy / charge drift of the reference (classical) series
 *     at T (energy_drift_true, charge_drift_true); NaN without one. */
#define HF_NUM_SUMMARY 8

typedef struct hf_model *hf_model_t;

/* Library version string, "hybridflux <ver> gfx950 src:<16 hex>": the hex is a
 * sha256 prefix of the sources, headers and Makefile the library was built
 * from, so a record that prints it names the exact sources that ran. */
const char *hf_version(void);

/* Thread-local message describing the last failure on this thread. */
const char *hf_last_error(void);

/* Number of visible HIP devices (0 when none); never fails. */
int hf_device_count(void);

/*
 * Replaces: FluxGNN.__init__ + load_state_dict (src/flux_gnn.py:11-38,
 * src/hybrid_solver.py:22-28).
 * host_params: every parameter of the reference state dict, float32,
 * concatenated in this order (row-major, shapes as nn.Linear stores them):
 *   input_mlp.0.weight [H][in_dim], input_mlp.0.bias [H],
 *   for l in 0..layers-1: update_mlps.l.0.weight [H][2H], update_mlps.l.0.bias [H],
 *   edge_mlp.0.weight [H][2H], edge_mlp.0.bias [H],
 *   edge_mlp.2.weight [1][H], edge_mlp.2.bias [1].
 * The handle packs them into the MFMA fragment order of the fused chain
 * kernels (when in_dim==4 && H==128) and keeps the natural layout for the
 * generic-graph path (always float32).  wdtype selects the chain kernels'
 * MFMA arithmetic: HF_WDTYPE_F32 (v_mfma_f32_16x16x4_f32, exact f32),
 * HF_WDTYPE_F16X3 (v_mfma_f32_16x16x32_f16 on a two-term fp16 split of both
 * operands, 3 products: fp32-level accuracy at ~5x the f32 MFMA rate) or
 * HF_WDTYPE_BF16 (bf16 weights and activations, config 4).
 */
int hf_model_create(const float *host_params, int in_dim, int hidden, int layers,
                    int wdtype, hf_model_t *out);
void hf_model_destroy(hf_model_t model);
/* Total float count host_params must hold for these dimensions. */
int64_t hf_model_param_count(int in_dim, int hidden, int layers);

/*
 * Replaces: FluxGNN.forward (src/flux_gnn.py:40-67) applied to the batched
 * chain graph of build_chain_graph (src/graph_constructor.py:6-39).
 * dev_node_features [B*nx][4]; dev_flux_edge [B][2nx] (may be NULL);
 * dev_flux_face [B][nx] = 0.5*(edge i + edge nx+i) (may be NULL;
 * src/hybrid_solver.py:45-48).  Any nx >= 1.
 */
int hf_chain_flux(hf_model_t model, const float *dev_node_features, int B, int nx,
                  float *dev_flux_edge, float *dev_flux_face, void *stream);

/*
 * Replaces: FluxGNN.forward on an ARBITRARY graph (examples/smoke_test.py:45-56
 * calls it with a random edge_index).  dev_edge_index [2][E] int64.
 * dev_workspace must hold hf_graph_workspace_bytes(model, N, E) bytes.
 */
int64_t hf_graph_workspace_bytes(hf_model_t model, int64_t N, int64_t E);
int hf_graph_flux(hf_model_t model, const float *dev_node_features, int64_t N,
                  const int64_t *dev_edge_index, int64_t E, float *dev_flux,
                  void *dev_workspace, void *stream);

/*
 * Training: FluxGNN.forward + autograd backward on any
 * graph (src/flux_gnn.py:40-67 under loss.backward() in
 * scripts/training/train_ablation.py:120-206).  Weights are read from a DEVICE
 * float32 buffer dev_params in the host_params order of hf_model_create
 * (state-dict order), so an optimizer can update them in place between steps.
 *
 * hf_graph_forward_train writes dev_flux[E] (as hf_graph_flux) and an
 * activation tape (hf_graph_tape_bytes) that hf_graph_backward consumes.
 * hf_graph_backward writes dL/dparams (overwriting, same layout as
 * dev_params, hf_model_param_count floats) and, when dev_grad_node_features
 * is not NULL, dL/dnode_features [N][in_dim].  dev_grad_flux is dL/dflux [E].
 * Weight gradients are split-K sums reduced in a fixed order: bitwise
 * deterministic for a given N, E.  chain_nx > 0 declares that edge_index is
 * N/chain_nx disjoint periodic chains of chain_nx cells in build_chain_graph
 * order (src/graph_constructor.py:34-38, E == 2N): with hidden a power of two
 * in [32, 256], in_dim <= 8 and N * 2 * hidden + 2 * hidden < 2^31 the chain
 * training path runs (the aggregation as
 * a stencil inside the GEMM operand loads, the edge readout split into
 * per-node P/Q GEMMs, f32 MFMA GEMMs throughout); otherwise the edge buckets
 * are formed arithmetically instead of by the count/scan/fill CSR build.  0
 * for any other graph.
 */
int64_t hf_graph_tape_bytes(int in_dim, int hidden, int layers, int64_t N, int64_t E);
int64_t hf_graph_backward_workspace_bytes(int in_dim, int hidden, int layers, int64_t N, int64_t E);
int hf_graph_forward_train(const float *dev_params, int in_dim, int hidden, int layers,
                           const float *dev_node_features, int64_t N, const int64_t *dev_edge_index,
                           int64_t E, int chain_nx, float *dev_flux, void *dev_tape, void *stream);
int hf_graph_backward(const float *dev_params, int in_dim, int hidden, int layers,
                      const float *dev_node_features, int64_t N, const int64_t *dev_edge_index, int64_t E,
                      int chain_nx, const void *dev_tape, const float *dev_grad_flux, float *dev_grad_params,
                      float *dev_grad_node_features, void *dev_workspace, void *stream);

/*
 * Replaces: the single-step terms of the reference trainer's ablation loss
 * (scripts/training/train_ablation.py:120-170: flux MSE, state MSE of the
 * finite-volume continuity update, Poisson MSE, charge and one-step energy
 * terms), batched over B samples as hybridflux.training.ablation_loss does.
 * dev_flux_edge [B][2nx] (FluxGNN output), dev_state_t / dev_state_next
 * [B][3][nx], dev_flux_t [B][nx]; c = f32(dt/dx), dx = f32(dx); lam[4] =
 * lambda_state, lambda_poisson, lambda_charge, lambda_energy_one; dev_c the
 * Poisson plan.  Writes dev_loss[0] = loss, dev_flux_loss[0] = the flux MSE
 * term and dev_dflux_edge
 * [B][2nx] = d loss / d flux_edge (the Poisson and energy terms go through a
 * detached solve, as in the reference, and the charge term's gradient is
 * identically 0).  dev_workspace: hf_ablation_loss_workspace_bytes(B, nx).
 */
int64_t hf_ablation_loss_workspace_bytes(int B, int nx);
int hf_ablation_loss(const float *dev_flux_edge, const float *dev_state_t, const float *dev_flux_t,
                     const float *dev_state_next, int B, int nx, float c, float dx, const float *lam,
                     const double *dev_c, float *dev_loss, float *dev_flux_loss, float *dev_dflux_edge,
                     void *dev_workspace, int64_t workspace_bytes, void *stream);

/*
 * Replaces: the whole per-sample loss of the reference trainer, the
 * multi-step rollout energy term included (scripts/training/
 * train_ablation.py:120-206, the 'full' and 'rollout_only' configs).
 * hf_ablation_loss plus lam[4] = lambda_energy_multi and rollout_steps = K,
 * dt = f32(dt): adds lam[4] * mean_{k<K, b} (e_k - e_0)^2, e_k = 0.5 mean(u_k^2)
 * (:172-206), when K > 0 and lam[4] > 0.  The energies use u_0..u_{K-1} only,
 * and u is advanced with the sample's E (k = 0) and then the detached Poisson
 * E of the previous n (:193-200); for K <= 3 that is u_0, u_1 and u_2 with E_1
 * = E(n') of the main forward's n' (the rollout's first forward is the same
 * model on the same state), so no further model forward reaches the loss and
 * the term is formed here from the inputs alone.  It carries no gradient (u
 * does not depend on the parameters), so dev_dflux_edge is hf_ablation_loss's.
 * K > 3 with lam[4] > 0 is HF_EUNSUPPORTED (later energies need forwards on
 * later states: pass lam[4] = 0 and add the term from them).  hf_ablation_loss
 * is this call with lam[4] = 0, K = 0.  Same workspace.
 */
int hf_ablation_loss_ex(const float *dev_flux_edge, const float *dev_state_t, const float *dev_flux_t,
                        const float *dev_state_next, int B, int nx, float c, float dx, const float *lam,
                        int rollout_steps, float dt, const double *dev_c, float *dev_loss, float *dev_flux_loss,
                        float *dev_dflux_edge, void *dev_workspace, int64_t workspace_bytes, void *stream);

/*
 * Replaces: one training batch of the reference trainer (its dataset of
 * (state_t, flux_t, state_next) triples indexed by a DataLoader batch,
 * scripts/training/train_ablation.py:27-44) and the batch's chain node
 * features (src/graph_constructor.py:6-39 build_chain_graph: [n, u, E, x] per
 * cell, batched), in one pass.  dev_idx [B] int64 sample indices (negative
 * ones wrap once, as torch indexing; beyond [-N, N) they are clamped);
 * dataset dev_state_t_all / dev_state_next_all [N][3][nx], dev_flux_t_all
 * [N][nx]; dev_x [nx].  Writes dev_state_t / dev_state_next [B][3][nx],
 * dev_flux_t [B][nx], dev_node_features [B*nx][4].
 */
int hf_chain_batch_gather(const int64_t *dev_idx, int B, const float *dev_state_t_all,
                          const float *dev_flux_t_all, const float *dev_state_next_all, int64_t N, int nx,
                          const float *dev_x, float *dev_state_t, float *dev_flux_t, float *dev_state_next,
                          float *dev_node_features, void *stream);

/*
 * Replaces: the reference trainer's optimizer step (torch.optim.Adam,
 * scripts/training/train_ablation.py:208-209; weight decay 0, no amsgrad) on
 * one flat float32 parameter buffer of n values, in one launch.  dev_step: the
 * step count (float, on the device; read, then incremented by the call, so a
 * captured graph replays it); dev_done: one unsigned, 0 before the first call
 * (the call leaves it 0).  Update per value: m = b1 m + (1 - b1) g, v = b2 v +
 * (1 - b2) g^2, p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps).
 */
int hf_adam_flat(float *dev_params, const float *dev_grads, float *dev_exp_avg, float *dev_exp_avg_sq, int64_t n,
                 float *dev_step, unsigned *dev_done, float lr, float beta1, float beta2, float eps, void *stream);

/*
 * The reference's other rollout models, inference.
 * dev_params: every parameter, float32, state-dict order, on the device.
 *
 * PureGNN (scripts/training/train_pure_gnn.py:35-76): input_mlp.0 [H][in],
 * update_mlps.l.0 [H][2H] (+bias) for each layer, output_mlp.0 [H][H],
 * output_mlp.2 [3][H] (+biases); tanh activations, residual message passing.
 * hf_pure_gnn_forward = PureGNN.forward(node_features [N][in], edge_index
 * [2][E]) -> delta [N][3]; chain_nx as for hf_graph_forward_train.
 * hf_pure_gnn_run = the rollout of scripts/evaluation/evaluate_multi_ic.py:45-66
 * (state <- state + delta, node features [n,u,E,x]) for B ICs on chains of nx
 * cells: state0/final [B][3][nx], traj [B][T+1][3][nx] or NULL; x [nx].
 * Workspace: hf_pure_gnn_workspace_bytes(H, N, E) for hf_pure_gnn_forward;
 * hf_pure_gnn_run_workspace_bytes(H, B, nx, T) for hf_pure_gnn_run.  The
 * rollout is ONE launch for all T steps for nx in {16, 32, 48, 64} with H in
 * {64, 128} (one IC per workgroup, activations in LDS); its workspace holds a
 * packed copy of the message/output weights made at the start of the call (the
 * copy for up to 8 layers; with more layers, or with dev_workspace == NULL, the
 * launch reads nn.Linear's rows in place, slower).  Otherwise, on chains whose nx divides 128 with H a multiple of 64,
 * each message layer is one f32 MFMA GEMM that forms the messages and the
 * residual in its epilogue (csrc/tgemm.h EpiMsg); other shapes run the generic
 * linear + gather kernels.
 *
 * PINN (scripts/training/train_pinn.py:36-61): net.0 [H][D], (layers-2) x
 * [H][H], net.last [D][H] (+biases), tanh between; out = state + net(state)
 * on states flattened to D = 3*nx.  hf_pinn_run = evaluate_multi_ic.py:70-83
 * for B ICs: state0/final [B][D], traj [B][T+1][D] or NULL.  The reference's
 * shape (D = 192, H = 256, 2 <= layers <= 8) runs as ONE launch for all T steps
 * (16 ICs per workgroup, activations in LDS; hf_pinn_forward is its T = 1),
 * whose workspace holds a packed copy of the weights made at the start of the
 * call (hf_pinn_workspace_bytes: the copy for the largest layer count, 8);
 * other shapes run per-layer GEMMs through the workspace.  B = 0 or T = 0
 * needs none.  ABI note (round 4): hf_pinn_run / hf_pinn_forward require the
 * workspace whenever hf_pinn_workspace_bytes > 0 (a NULL workspace is
 * HF_EINVAL; it used to be accepted); hf_pure_gnn_run accepts NULL on its
 * one-launch shapes.
 */
int64_t hf_pure_gnn_param_count(int in_dim, int hidden, int layers);
int64_t hf_pure_gnn_workspace_bytes(int hidden, int64_t N, int64_t E);
int64_t hf_pure_gnn_run_workspace_bytes(int hidden, int B, int nx, int T);
int hf_pure_gnn_forward(const float *dev_params, int in_dim, int hidden, int layers,
                        const float *dev_node_features, int64_t N, const int64_t *dev_edge_index, int64_t E,
                        int chain_nx, float *dev_delta, void *dev_workspace, void *stream);
int hf_pure_gnn_run(const float *dev_params, int hidden, int layers, const float *dev_state0,
                    float *dev_final, const float *dev_x, int B, int nx, int T, float *dev_traj,
                    void *dev_workspace, void *stream);
int64_t hf_pinn_param_count(int dim, int hidden, int layers);
int64_t hf_pinn_workspace_bytes(int dim, int hidden, int64_t B);
int hf_pinn_forward(const float *dev_params, int dim, int hidden, int layers, const float *dev_state,
                    float *dev_out, int64_t B, void *dev_workspace, void *stream);
int hf_pinn_run(const float *dev_params, int dim, int hidden, int layers, const float *dev_state0,
                float *dev_final, int64_t B, int T, float *dev_traj, void *dev_workspace, void *stream);

/*
 * Host helper (no device work): the Poisson "plan" for nx cells, length
 * hf_poisson_plan_len(nx) doubles.  plan[0..nx) is the first column c of the
 * real circulant matrix equal to the reference's spectral Poisson operator
 * E = Re(ifft(1j*fft(n-1)/k)), k=0 mode zeroed (src/baseline_solver.py:26,59-68):
 * E[i] = sum_j c[(i-j) mod nx] * (n[j]-1), computed in float64.  For power-of-two
 * nx in [256, 2048] the kernels apply the operator by float64 FFT instead and
 * the plan continues with the twiddles exp(-2 pi i m/nx), m < nx/2, as (re, im)
 * pairs, then 1/k_q (0 for q = 0 and, for even nx, q = nx/2: that term is imaginary for real rho, dropped by the reference's Re()).  Every dev_c argument below is a device copy
 * of this plan.
 */
int hf_poisson_plan_len(int nx);
int hf_poisson_coeffs(int nx, double length, double *host_c);

/* Replaces: BaselineSolver.solve_poisson (src/baseline_solver.py:59-68), batched.
 * dev_n, dev_E: [B][nx] float32 (row stride ld_n / ld_E floats);
 * dev_c: device copy of hf_poisson_coeffs. */
int hf_poisson(const float *dev_n, int ld_n, float *dev_E, int ld_E,
               const double *dev_c, int B, int nx, void *stream);

/*
 * Poisson modes.  Every entry point without a mode argument, and every *_ex
 * call given HF_POISSON_SPECTRAL, applies the reference's spectral operator
 * (src/baseline_solver.py:59-68) with the plan of hf_poisson_coeffs: the
 * parity mode and the default.
 *
 * HF_POISSON_TRIDIAG is an OPT-IN mode that is NOT the reference's operator
 * (no parity with the reference is claimed for it): the cyclic-reduction
 * tridiagonal solve the north star names, of the same equation dE/dx =
 * -(rho - mean rho), rho = n - 1, in second-order potential form on the
 * periodic grid:
 *   (phi[i-1] - 2 phi[i] + phi[i+1]) / dx^2 = rho[i] - mean(rho),
 *   E[i] = -(phi[i+1] - phi[i-1]) / (2 dx),
 * solved in float64 by one wave per IC (or IC pair) with phi[0] = 0 (E does not
 * depend on the gauge) and rounded to float32 once.  It differs from the
 * spectral E by ~1e-3 at nx = 64 (the symbol (dx/2) cot(k dx/2) vs 1/k).
 * Fused into the same kernels as the spectral solve (the persistent rollouts
 * at nx <= 64, the FV kernels at every other nx); nx <= 16384.  The training
 * loss (hf_ablation_loss) always uses the spectral operator.
 */
#define HF_POISSON_SPECTRAL 0
#define HF_POISSON_TRIDIAG 1
/* Length in doubles of the plan of `mode` for nx cells (-1: unsupported):
 * hf_poisson_plan_len(nx) for SPECTRAL, 1 for TRIDIAG (plan[0] = dx/2). */
int hf_poisson_plan_size(int mode, int nx);
/* Host helper (no device work): the plan of `mode` (SPECTRAL: hf_poisson_coeffs). */
int hf_poisson_plan(int mode, int nx, double length, double *host_plan);
/* hf_poisson with a Poisson mode; dev_plan is a device copy of hf_poisson_plan(mode, ...). */
int hf_poisson_ex(const float *dev_n, int ld_n, float *dev_E, int ld_E, const double *dev_plan,
                  int poisson_mode, int B, int nx, void *stream);

/*
 * Scratch of the generic (non-fused) sequencing.  hf_step, hf_run and
 * hf_run_compare take (dev_workspace, workspace_bytes): a device buffer of at
 * least hf_workspace_need(model, op, B, nx, T, flags) bytes (or the upper
 * bound hf_run_workspace_bytes(op, B, nx, T)) that the call may use as
 * scratch until the work it enqueued has run; the caller keeps it alive and
 * unshared until then.  dev_workspace == NULL makes the call allocate its
 * scratch stream-ordered (hipMallocAsync / hipFreeAsync on `stream`).  The
 * fused paths (nx in {16,32,48,64} with a model) use no scratch.
 */
#define HF_OP_STEP 0
#define HF_OP_RUN 1
#define HF_OP_COMPARE 2
/* An upper bound over every model, nx path and output choice of `op`. */
int64_t hf_run_workspace_bytes(int op, int B, int nx, int T);
/* The exact scratch the call will carve for this model (NULL = classical;
 * HF_OP_COMPARE needs a model), nx path and outputs: flags HF_WS_TRAJ when the
 * call is given dev_traj (hf_run), HF_WS_FLUX_FACE when given dev_flux_face
 * (hf_step).  0 on every path that needs no scratch (the fused rollouts, the
 * one-launch classical rollouts); -1 on bad arguments.  A dev_workspace of at
 * least this many bytes is accepted by the call; a smaller one is HF_EINVAL. */
#define HF_WS_TRAJ 1
#define HF_WS_FLUX_FACE 2
int64_t hf_workspace_need(hf_model_t model, int op, int B, int nx, int T, int flags);

/*
 * One timestep for B ICs (state_in -> state_out, may not alias).
 * model != NULL: HybridSolver.step (src/hybrid_solver.py:34-64):
 *   GNN flux -> symmetrise -> FV continuity -> Burgers u (no viscosity) -> Poisson.
 * model == NULL: BaselineSolver.step (src/baseline_solver.py:80-101):
 *   F=n*u -> FV continuity -> Burgers u + dt*(E + nu*lap u) -> Poisson.
 * Scalars are the reference's Python floats rounded to float32 on the host:
 *   c = f32(dt/dx), dt = f32(dt), nu = f32(nu), dx2 = f32(dx*dx).
 * dev_x [nx]: float32 cell centres (node feature x); dev_c: Poisson coeffs.
 * dev_flux_face [B][nx] (may be NULL): the F used this step (F_n classically).
 * dev_metrics [B][HF_NUM_METRICS] (may be NULL) for state_out.
 * Any nx >= 1: nx <= 6144 keeps the chain in LDS; larger nx (not an FFT size)
 * runs the update and a tiled Poisson sum over global memory, same values.
 */
int hf_step(hf_model_t model, const float *dev_state_in, float *dev_state_out,
            const float *dev_x, const double *dev_c, int B, int nx,
            float c, float dt, float nu, float dx2,
            float *dev_flux_face, float *dev_metrics,
            void *dev_workspace, int64_t workspace_bytes, void *stream);
/* hf_step with a Poisson mode (dev_plan: hf_poisson_plan(poisson_mode, ...));
 * hf_step == hf_step_ex(..., dev_c, HF_POISSON_SPECTRAL, ...). */
int hf_step_ex(hf_model_t model, const float *dev_state_in, float *dev_state_out,
               const float *dev_x, const double *dev_plan, int poisson_mode, int B, int nx,
               float c, float dt, float nu, float dx2,
               float *dev_flux_face, float *dev_metrics,
               void *dev_workspace, int64_t workspace_bytes, void *stream);

/*
 * T-step rollout (HybridSolver.run src/hybrid_solver.py:66-73 when model !=
 * NULL, BaselineSolver.run src/baseline_solver.py:103-118 when NULL), batched.
 * dev_state0 [B][3][nx] -> dev_state_final [B][3][nx]; the two may alias
 * (the same buffer holds the initial and, after the call, the final states).
 * dev_traj [B][T+1][3][nx] (may be NULL) receives every state incl. t=0.
 * dev_flux_traj [B][T][nx] (may be NULL) receives the face flux of each step
 *   (the classical run's `fluxes`).
 * dev_metrics [B][T+1][HF_NUM_METRICS] (may be NULL).
 * For nx in {16,32,48,64} with model != NULL the whole rollout is ONE
 * persistent kernel (state resident on-chip across steps); so is the classical
 * rollout (model == NULL) at nx <= 64 and nx in {256, 512, 1024}, bit-identical to T
 * hf_step calls (HF_FV_PERSIST=0 in the environment selects the per-step
 * launches, for A/B timing).  Otherwise, with
 * model != NULL and B*nx >= 2^21 cells, slices of the batch step on up to 3
 * library-owned lane streams forked from and joined back into `stream` with
 * events (HF_RUN_LANES=1..4 in the environment overrides the count): the call
 * stays ordered on `stream` (and capturable), and every IC's result is
 * bit-identical to the one-stream sequencing.  The lane streams belong to
 * (device, `stream`): calls on different streams or threads never share a
 * lane, and capturing `stream` draws in only its own lanes.
 */
int hf_run(hf_model_t model, const float *dev_state0, float *dev_state_final,
           const float *dev_x, const double *dev_c, int B, int nx, int T,
           float c, float dt, float nu, float dx2,
           float *dev_traj, float *dev_flux_traj, float *dev_metrics,
           void *dev_workspace, int64_t workspace_bytes, void *stream);
/* hf_run with a Poisson mode; same paths, workspace and aliasing rules. */
int hf_run_ex(hf_model_t model, const float *dev_state0, float *dev_state_final,
              const float *dev_x, const double *dev_plan, int poisson_mode, int B, int nx, int T,
              float c, float dt, float nu, float dx2,
              float *dev_traj, float *dev_flux_traj, float *dev_metrics,
              void *dev_workspace, int64_t workspace_bytes, void *stream);

/*
 * Hybrid rollout scored against the classical solver from the same ICs, in
 * one pass (replaces the serial per-IC loop of
 * scripts/evaluation/evaluate_multi_ic.py:21-94: BaselineSolver.step from
 * state0, HybridSolver.run from state0, per-step channel MSE; and the
 * energy/charge series of scripts/evaluation/evaluate_all.py:118-159).
 * The classical twin uses the same dt/dx and viscosity `nu`.
 * dev_mse [B][T+1][3] float32 (required): mean over cells of
 *   (hybrid - classical)^2 for n, u, E at every step (step 0 is 0), summed in
 *   float64 and rounded once.
 * dev_metrics / dev_metrics_classical [B][T+1][HF_NUM_METRICS] (may be NULL).
 * dev_state_final receives the hybrid final state; it may alias dev_state0.
 * For nx in {16,32,48,64} both solvers advance inside the one persistent kernel.
 * For nx in {256, 512, 1024} (model not fused) the hybrid rollout runs first and
 * the classical twin is one launch that scores each step against the hybrid
 * trajectory as it goes; the results equal the recorded-trajectory path bit
 * for bit.  dev_workspace, if given, is sized by hf_workspace_need(model,
 * HF_OP_COMPARE, ...): 0 at the fused nx, one hybrid trajectory plus the face
 * flux at nx in {256, 512, 1024}, two trajectories, a state and the flux
 * otherwise.
 */
int hf_run_compare(hf_model_t model, const float *dev_state0, float *dev_state_final,
                   const float *dev_x, const double *dev_c, int B, int nx, int T,
                   float c, float dt, float nu, float dx2, float *dev_mse,
                   float *dev_metrics, float *dev_metrics_classical,
                   void *dev_workspace, int64_t workspace_bytes, void *stream);
/* hf_run_compare with a Poisson mode: the hybrid rollout AND its classical
 * twin both use it. */
int hf_run_compare_ex(hf_model_t model, const float *dev_state0, float *dev_state_final,
                      const float *dev_x, const double *dev_plan, int poisson_mode, int B, int nx, int T,
                      float c, float dt, float nu, float dx2, float *dev_mse,
                      float *dev_metrics, float *dev_metrics_classical,
                      void *dev_workspace, int64_t workspace_bytes, void *stream);

/*
 * Metric series of recorded trajectories (the host-side scoring of
 * scripts/evaluation/evaluate_all.py:118-159 and evaluate_multi_ic.py:88-94,
 * on the device):
 * hf_traj_metrics: dev_traj [B][T1][3][nx] -> dev_metrics [B][T1][HF_NUM_METRICS].
 * hf_traj_mse: per-step channel MSE of two trajectories [B][T1][3][nx] ->
 *   dev_mse [B][T1][3] (n, u, E), float64 sums rounded once.
 */
int hf_traj_metrics(const float *dev_traj, int B, int T1, int nx, float *dev_metrics, void *stream);
int hf_traj_mse(const float *dev_traj_a, const float *dev_traj_b, int B, int T1, int nx, float *dev_mse,
                void *stream);

/*
 * Per-IC summary of a T-step rollout from its metric series (SURVEY.md 8f
 * rank 1; fields at HF_NUM_SUMMARY).  dev_metrics [B][T+1][HF_NUM_METRICS]
 * (required), dev_mse [B][T+1][3] (may be NULL), dev_metrics_ref
 * [B][T+1][HF_NUM_METRICS] (may be NULL: the classical twin's series).
 * dev_summary [B][HF_NUM_SUMMARY] (required); dev_drift [B][T+1][4] (may be
 * NULL): |energy_t - energy_0|, |charge_t - charge_0| of the rollout, then
 * of the reference series (NaN without one).
 */
int hf_rollout_summary(const float *dev_metrics, const float *dev_mse, const float *dev_metrics_ref, int B,
                       int T, float *dev_summary, float *dev_drift, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* HYBRIDFLUX_H */
