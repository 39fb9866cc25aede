// The reference's other rollout models, inference on the
// MI355X: PureGNN (scripts/training/train_pure_gnn.py:35-76) and PINN
// (scripts/training/train_pinn.py:36-61), batched over ICs, with the rollout
// loops of scripts/evaluation/evaluate_multi_ic.py:45-83 and
// benchmark_timing.py:100-203 (state <- state + model(state)).
//
// Both are built on the generic MFMA GEMM of graph.hip (gemm_linear: fused
// bias, tanh and residual epilogues).  PureGNN's edge message
// tanh(W [h_src ; h_dst] + b) is evaluated through the split
// W_a h_src + W_b h_dst: two per-node GEMMs (P = W_a h, Q = W_b h) and one
// fused gather kernel that forms every incoming message of a node, sums them
// in edge order (index_add_, :64-66) and adds the residual (:67) — half the
// FLOPs of an edge-wise GEMM and no [E][H] message tensor in HBM.
#include "hf_device.h"
#include "hf_internal.h"
#include "tgemm.h"

namespace hf {
namespace {

inline size_t a256(size_t v) { return (v + 255) & ~size_t(255); }
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float message(const float *P, int64_t s, int H, int f, float q, float b) {
  return tanhf(__fadd_rn(__fadd_rn(P[s * H + f], q), b));
}

// h_out[d] = h[d] + sum_{e: dst[e] = d, ascending e} tanh(P[src[e]] + Q[d] + b).
// chain_nx > 0: B periodic chains in build_chain_graph order, where the
// messages into cell i come from i-1 (edge i-1) then i+1 (edge nx+i).
__global__ void message_sum_kernel(const float *__restrict__ h, const float *__restrict__ P,
                                   const float *__restrict__ Q, const float *__restrict__ b,
                                   const int64_t *__restrict__ src, const int *__restrict__ off,
                                   const int *__restrict__ perm, int chain_nx, int64_t N, int H,
                                   float *__restrict__ h_out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N * H) return;
  const int64_t d = t / H;
  const int f = (int)(t - d * H);
  const float q = Q[t], bf = b[f];
  float acc = 0.f;
  if (chain_nx > 0) {
    const int64_t c0 = d / chain_nx * chain_nx;
    const int i = (int)(d - c0);
    acc = __fadd_rn(acc, message(P, c0 + (i + chain_nx - 1) % chain_nx, H, f, q, bf));
    acc = __fadd_rn(acc, message(P, c0 + (i + 1) % chain_nx, H, f, q, bf));
  } else {
    for (int p = off[d]; p < off[d + 1]; ++p) acc = __fadd_rn(acc, message(P, src[perm[p]], H, f, q, bf));
  }
  h_out[t] = __fadd_rn(h[t], acc);
}

// node features [n, u, E, x] of every cell (benchmark_timing.py:121-125)
__global__ void chain_features_kernel(const float *__restrict__ state, const float *__restrict__ x, int64_t B, int nx,
                                      float *__restrict__ nf) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * nx) return;
  const int64_t b = t / nx;
  const int i = (int)(t - b * nx);
  const float *s = state + b * 3 * nx;
  reinterpret_cast<float4 *>(nf)[t] = make_float4(s[i], s[nx + i], s[2 * nx + i], x[i]);
}

// state' = state + delta^T  (delta [B*nx][3], benchmark_timing.py:128-130), written to
// out (contiguous [B][3][nx]) and, when given, to a trajectory slot of per-IC stride ld2.
__global__ void add_delta_kernel(const float *__restrict__ state, const float *__restrict__ delta, int64_t B, int nx,
                                 float *__restrict__ out, float *__restrict__ out2, int64_t ld2) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= B * 3 * nx) return;
  const int64_t b = t / (3 * nx);
  const int r = (int)(t - b * 3 * nx), c = r / nx, i = r - c * nx;
  const float v = __fadd_rn(state[t], delta[(b * nx + i) * 3 + c]);
  out[t] = v;
  if (out2) out2[b * ld2 + r] = v;
}

struct PureW {
  const float *w_in, *b_in;  // [H][in], [H]
  const float *w_l, *b_l;    // layer l at + l*(2H*H + H): [H][2H], [H]
  const float *w_o1, *b_o1;  // [H][H], [H]
  const float *w_o2, *b_o2;  // [3][H], [3]
  int in_dim, H, L;
  int64_t ls;
  const float *w_lp, *w_o1p;  // the one-launch rollout's packed copies: [l][u][P|Q][kb][lane][4], [u][kb][lane][4]
};

PureW pure_view(const float *p, int in_dim, int H, int L) {
  PureW w{};
  int64_t o = 0;
  w.in_dim = in_dim;
  w.H = H;
  w.L = L;
  w.w_in = p + o; o += (int64_t)H * in_dim;
  w.b_in = p + o; o += H;
  w.w_l = p + o;
  w.b_l = p + o + 2LL * H * H;
  w.ls = 2LL * H * H + H;
  o += L * w.ls;
  w.w_o1 = p + o; o += (int64_t)H * H;
  w.b_o1 = p + o; o += H;
  w.w_o2 = p + o; o += 3LL * H;
  w.b_o2 = p + o;
  return w;
}

struct PureWs {
  float *h0, *h1, *P, *Q, *nf, *delta;
  void *buckets;
};

PureWs carve_pure(void *ws, int H, int64_t N) {
  char *p = static_cast<char *>(ws);
  auto take = [&](size_t bytes) {
    char *r = p;
    p += a256(bytes);
    return r;
  };
  PureWs w{};
  w.h0 = reinterpret_cast<float *>(take(sizeof(float) * N * H));
  w.h1 = reinterpret_cast<float *>(take(sizeof(float) * N * H));
  w.P = reinterpret_cast<float *>(take(sizeof(float) * N * H));
  w.Q = reinterpret_cast<float *>(take(sizeof(float) * N * H));
  w.nf = reinterpret_cast<float *>(take(sizeof(float) * N * 4));
  w.delta = reinterpret_cast<float *>(take(sizeof(float) * N * 3));
  w.buckets = p;
  return w;
}

// The chain form of PureGNN's layers (tgemm.h): on chains whose length
// divides the 128-cell row tile and hidden widths in multiples of 64, a message
// layer is ONE f32 MFMA GEMM h [N][H] x [W_a ; W_b]^T whose block epilogue
// forms the messages and the residual (EpiMsg), and output_mlp.0 is a GEMM
// with a tanh epilogue.  Otherwise: the generic linear + gather kernels.
bool pure_chain_ok(int H, int chain_nx, int64_t N) {
  return chain_nx > 0 && 128 % chain_nx == 0 && H % 64 == 0 && H <= 1024 && N * H < (int64_t(1) << 31);
}

// PureGNN.forward (train_pure_gnn.py:57-76) over buckets already built.
hipError_t pure_forward(const PureW &w, const float *nf, int64_t N, const int64_t *src, const int *off,
                        const int *perm, int chain_nx, PureWs &b, float *delta, hipStream_t s) {
  const int H = w.H;
  hipError_t e;
  if ((e = gemm_linear(nf, w.in_dim, nullptr, nullptr, 0, nullptr, wv_rows(w.w_in, w.in_dim, w.in_dim), w.b_in, b.h0,
                       N, H, kActTanh, nullptr, s)))
    return e;
  float *h = b.h0, *hn = b.h1;
  if (pure_chain_ok(H, chain_nx, N)) {
    using namespace tg;
    for (int l = 0; l < w.L; ++l) {
      const float *W = w.w_l + l * w.ls;
      if ((e = tgemm<VPlain, false, VPQ, false, EpiMsg>(VPlain{h, H, N, kNoSplit, 0, H}, VPQ{W, H},
                                                         EpiMsg{h, hn, w.b_l + l * w.ls, H, chain_nx}, N, 2LL * H, H, 1,
                                                         s)))
        return e;
      float *t = h;
      h = hn;
      hn = t;
    }
    if ((e = tgemm<VPlain, false, VPlain, false, EpiTanh>(VPlain{h, H, N, kNoSplit, 0, H},
                                                           VPlain{w.w_o1, H, H, kNoSplit, 0, H},
                                                           EpiTanh{hn, H, w.b_o1}, N, H, H, 1, s)))
      return e;
    return gemm_linear(hn, H, nullptr, nullptr, 0, nullptr, wv_rows(w.w_o2, H, H), w.b_o2, delta, N, 3, kActNone,
                       nullptr, s);
  }
  const unsigned nb = (unsigned)((N * H + 255) / 256);
  for (int l = 0; l < w.L; ++l) {
    const float *W = w.w_l + l * w.ls;
    if ((e = gemm_linear(h, H, nullptr, nullptr, 0, nullptr, WView{W, W, 2LL * H, 1}, nullptr, b.P, N, H, kActNone,
                         nullptr, s)))
      return e;
    if ((e = gemm_linear(h, H, nullptr, nullptr, 0, nullptr, WView{W + H, W + H, 2LL * H, 1}, nullptr, b.Q, N, H,
                         kActNone, nullptr, s)))
      return e;
    hipLaunchKernelGGL(message_sum_kernel, dim3(nb), dim3(256), 0, s, h, b.P, b.Q, w.b_l + l * w.ls, src, off, perm,
                       chain_nx, N, H, hn);
    float *t = h;
    h = hn;
    hn = t;
  }
  if ((e = gemm_linear(h, H, nullptr, nullptr, 0, nullptr, wv_rows(w.w_o1, H, H), w.b_o1, hn, N, H, kActTanh, nullptr,
                       s)))
    return e;
  return gemm_linear(hn, H, nullptr, nullptr, 0, nullptr, wv_rows(w.w_o2, H, H), w.b_o2, delta, N, 3, kActNone,
                     nullptr, s);
}

// PINN: layers 0..L-1 are net.{0,2,4,..}: D->H tanh, (L-2) x H->H tanh, H->D (+ state)
struct PinnW {
  const float *w[kMaxChainLayers], *b[kMaxChainLayers];
  int D, H, L;
  const float *wp[kMaxChainLayers];  // the one-launch rollout's packed copies of w (pinn_pack_kernel)
};
PinnW pinn_view(const float *p, int D, int H, int L) {
  PinnW w{};
  w.D = D;
  w.H = H;
  w.L = L;
  int64_t o = 0;
  for (int l = 0; l < L; ++l) {
    const int64_t in = l == 0 ? D : H, out = l == L - 1 ? D : H;
    w.w[l] = p + o; o += in * out;
    w.b[l] = p + o; o += out;
  }
  return w;
}

// ---------------------------------------------------------------------------
// PINN rollout in one launch (train_pinn.py:48-61 iterated as
// evaluate_multi_ic.py:75-81): a workgroup owns 16 ICs for all T steps, with
// their state and the hidden activations in LDS, and runs every layer as
// v_mfma_f32_16x16x4_f32 tiles (16 output features x 16 ICs) whose weight
// operand is read from a packed copy of nn.Linear's rows in the caller's
// workspace (pinn_pack_kernel: each wave's k-block one contiguous 1 KiB;
// L2-resident: 0.9 MB), kPinnAhead k-blocks in flight.  The k order inside a
// 16-block is permuted so that a lane's four MFMA steps read one float4 of its
// weight row (k = 16 kb + 4 (lane >> 4) + step); the activations use the same
// order, so LDS holds them as [k-block][lane][4]: an MFMA output tile is
// written back with one ds_write_b128 per lane and read as the next layer's B
// operand with one ds_read_b128.  No activation and no intermediate state
// reaches HBM; the ICs never exchange anything, so no step needs a grid sync.
constexpr int kPinnIcs = 16;

#ifndef HF_PINN_WAVES
#define HF_PINN_WAVES 8
#endif
// waves per workgroup: 8 (two per SIMD, two output tiles each, sharing each B
// fragment read).  With the loads serialised (round 3) 16 waves of one tile
// measured 3 % faster than 8 (profiles/r03_pinn_ab.txt); with the weight
// stream pipelined 8 waves measure 1.5-2.5 % faster than 16
// (profiles/r04_pinn_waves_ab.jsonl).
constexpr int kPinnWaves = HF_PINN_WAVES;
#ifndef HF_PINN_AHEAD
#define HF_PINN_AHEAD 4
#endif
// weight k-blocks in flight per wave (pinn_layer's software pipeline)
constexpr int kPinnAhead = HF_PINN_AHEAD;

// This wave's packed weight rows of one layer: output tiles wave + kPinnWaves j
// (j < NT; a spare tile past the layer's last is clamped to it and not stored)
template <int NT>
struct PinnRows {
  const float *p[NT];
};

// One layer on this wave's NT output tiles: out = act(W in + b) (ACT 0: tanh;
// 1: the last layer, state += W in + b).  wrow / nrow: this wave's packed
// weight rows of this layer / of the layer after it (KBN k-blocks; the next
// step's layer 0 after the last layer).
//
// The weight stream of a step is one software pipeline over all its layers:
// wq holds k-blocks c .. c+P-1 of the stream, the last P-1 iterations of a
// layer load the next layer's first P-1 k-blocks (so no layer starts on an L2
// round trip; loads stay in flight across the workgroup barrier, which waits
// on LDS only), and each iteration ends in a scheduling barrier, so the
// compiler cannot sink a load down to its use (left to itself it issued each
// load right before its MFMAs and waited for it there).  The B fragment of
// k-block c+1 is read from LDS under c's MFMAs (and feeds all NT tiles); the
// bias comes from LDS too (copied there once: a global bias load would be sunk
// into the store's branch and waited for there behind the next layer's
// k-blocks, vmcnt being in order).
// SPLIT (the last layer when its NTILES = 1.5 kPinnWaves tiles, the reference's
// PINN(192, 256): 12 tiles over 8 waves): instead of a second, clamped tile
// that waves 4-7 computed and dropped (a third of their MFMAs), wave w takes
// its own tile w whole (j = 0) and half the k-blocks of remainder tile
// kPinnWaves + w % R (j = 1, R = NTILES - kPinnWaves): waves R.. the first
// half, waves 0..R-1 the second, so every wave issues 1.5 tiles of MFMAs.  A
// first-half wave publishes its partial sums in LDS (sp) as soon as its half is
// done, then a flag word (release, workgroup scope); the second-half wave adds
// them (acquire on the flag, tag = step + 1) in its epilogue:
// out = state + ((lo + hi) + b).
struct PinnSplit {
  f4v *sp;     // [R][64] partial sums of the first halves
  int *flag;   // [R] step tag of the partial in sp
  int tag;     // this step's tag (t + 1)
};
// Barrier-free layer hand-off (HF_PINN_FLAGS): each output tile carries a
// flag word in LDS that its wave sets (release, workgroup scope) to the
// layer's tag (step * L + layer + 1, increasing) once the tile is stored; a
// wave reads input k-block c only after flag c holds the producing layer's tag
// (acquire).  Tiles are owned by one wave each, the activations cycle through
// three buffers (a writer of layer l has consumed every tile of layer l-1, so
// every wave is past layer l-2, the last reader of the buffer layer l
// overwrites), so no workgroup barrier orders a step: a wave starts a layer on
// the k-blocks that are ready while the slower waves finish theirs.  The last
// layer's owner waves also store their new state rows to the trajectory.
struct PinnSync {
  const int *in_flag = nullptr;  // flags of the input tiles (nullptr: a barrier ordered them)
  int in_tag = 0;
  int *out_flag = nullptr;
  int out_tag = 0;
  float *traj = nullptr;  // ACT 1: row step + 1 of IC b0 (ICs ldt apart), or nullptr
  int64_t ldt = 0;
  int nic = 0;  // ICs of the workgroup that exist
};
__device__ __forceinline__ void pinn_wait(const int *f, int tag) {
  // bounded: never reached in a correct run, but a lost producer ends in wrong values, not a hang
  for (int it = 0; __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < tag && it < (1 << 20); ++it)
    __builtin_amdgcn_s_sleep(1);
}
template <int K, int NTILES, int ACT, int KBN, int NT, bool SPLIT = false>
__device__ __forceinline__ void pinn_layer(const PinnRows<NT> &wrow, const float *bias, const float *in, float *out,
                                           int wave, int lane, f4v (&wq)[kPinnAhead][NT],
                                           const PinnRows<NT> &nrow, const PinnSplit &spl = PinnSplit{},
                                           const PinnSync &sy = PinnSync{}) {
  constexpr int KB = K / 16, P = kPinnAhead;
  static_assert(KB % P == 0 && KBN >= P - 1, "a layer's k-blocks fill whole rounds of the ring");
  static_assert(!SPLIT || (ACT == 1 && NT == 2 && 2 * (NTILES - kPinnWaves) == kPinnWaves && KB % 2 == 0),
                "split last layer: 1.5 tiles per wave");
  constexpr int R = NTILES - kPinnWaves;
  // SPLIT: j = 1 runs k-blocks [k1lo, k1lo + KB/2) of this wave (wave-uniform)
  const int k1lo = SPLIT ? (wave >= R ? 0 : KB / 2) : 0;
  auto on1 = [&](int kb) { return !SPLIT || (kb >= k1lo && kb < k1lo + KB / 2); };
  f4v acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = f4v{0.f, 0.f, 0.f, 0.f};
  // flags: one read of all the input tiles' flags; only if some are not yet
  // set does the wave wait per k-block
  bool ready = true;
  if (sy.in_flag) {
    const int f = lane < KB ? __hip_atomic_load(sy.in_flag + lane, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)
                            : sy.in_tag;
    ready = __all(f >= sy.in_tag);
    if (!ready) pinn_wait(sy.in_flag, sy.in_tag);
  }
  f4v bv = *reinterpret_cast<const f4v *>(in + lane * 4);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int c = 0; c < KB; ++c) {
    constexpr int kAhead = P - 1;
    const int s = c + kAhead;  // slot s % P held k-block c - 1, consumed last iteration
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      if (s < KB) {
        if (j == 0 || on1(s)) wq[s % P][j] = *reinterpret_cast<const f4v *>(wrow.p[j] + 256 * s);
      } else {
        wq[s % P][j] = *reinterpret_cast<const f4v *>(nrow.p[j] + 256 * (s - KB));
      }
    }
    f4v bn = bv;
    if (c + 1 < KB) {
      if (!ready) pinn_wait(sy.in_flag + c + 1, sy.in_tag);
      bn = *reinterpret_cast<const f4v *>(in + (c + 1) * 256 + lane * 4);
    }
    const bool use1 = on1(c);
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int j = 0; j < NT; ++j)
        if (j == 0 || use1) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(wq[c % P][j][e], bv[e], acc[j], 0, 0, 0);
    bv = bn;
    if constexpr (SPLIT) {
      if (c == KB / 2 - 1 && wave >= R) {  // the first half of remainder tile kPinnWaves + wave % R is done
        spl.sp[(wave - R) * 64 + lane] = acc[1];
        __hip_atomic_store(spl.flag + (wave - R), spl.tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (SPLIT) {
    if (wave < R) {  // remainder tile kPinnWaves + wave: lo (published) + hi (acc[1])
      while (__hip_atomic_load(spl.flag + wave, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != spl.tag)
        __builtin_amdgcn_s_sleep(1);
      const f4v lo = spl.sp[wave * 64 + lane];
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[1][i] = __fadd_rn(lo[i], acc[1][i]);
    }
  }
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int t = SPLIT && j == 1 ? kPinnWaves + wave % R : wave + kPinnWaves * j;
    if (SPLIT && j == 1 && wave >= R) break;  // (its half went to the second-half wave)
    if (NTILES % kPinnWaves != 0 && t >= NTILES) break;
    float *o = out + t * 256 + lane * 4;
    const f4v bq = *reinterpret_cast<const f4v *>(bias + 16 * t + 4 * (lane >> 4));
    f4v v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = __fadd_rn(acc[j][i], bq[i]);
    if (ACT == 0) {
#pragma unroll
      for (int i = 0; i < 4; i += 2) {  // packed pairs (bit-identical to tanh_fast)
        const hf_f2 t = tanh_fast2(hf_f2{v[i], v[i + 1]});
        v[i] = t.x, v[i + 1] = t.y;
      }
    } else {
      const f4v st = *reinterpret_cast<const f4v *>(o);
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = __fadd_rn(st[i], v[i]);
      // the new state's features 16t + 4 (lane >> 4) .. +3 of IC lane & 15
      if (sy.traj && (lane & 15) < sy.nic)
        *reinterpret_cast<f4v *>(sy.traj + (lane & 15) * sy.ldt + 16 * t + 4 * (lane >> 4)) = v;
    }
    *reinterpret_cast<f4v *>(o) = v;
    if (sy.out_flag) __hip_atomic_store(sy.out_flag + t, sy.out_tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

// LDS index of feature k of IC n in the [k-block][lane][4] order above
__device__ __forceinline__ int pinn_at(int k, int n) { return (k >> 4) * 256 + (((k >> 2) & 3) * 16 + n) * 4 + (k & 3); }

template <int D, int H>
__global__ __launch_bounds__(64 * kPinnWaves, 1) void pinn_run_kernel(PinnW w, const float *__restrict__ state0,
                                                          float *__restrict__ final_state, float *__restrict__ traj,
                                                          int64_t B, int T) {
  static_assert(D % 16 == 0 && H % 16 == 0, "16-feature tiles");
  constexpr int NT = (H / 16 + kPinnWaves - 1) / kPinnWaves;  // output tiles per wave (H >= D)
  static_assert(H >= D, "the widest layer sets the tiles per wave");
  constexpr int NTH = 64 * kPinnWaves;
  __shared__ f4v s_state4[D * kPinnIcs / 4];
// HF_PINN_FLAGS=1: the barrier-free hand-off (PinnSync).  Measured and not
// kept: correct (tests/test_gpu_baselines.py) but 12 % slower than the
// barriers (profiles/r06_models_ab.txt, run 3): without a barrier the older
// wave of each SIMD pair runs ahead and then waits on the younger one's tiles.
#ifndef HF_PINN_FLAGS
#define HF_PINN_FLAGS 0
#endif
  constexpr bool kFlags = HF_PINN_FLAGS;
  __shared__ f4v s_act4[kFlags ? 3 : 2][H * kPinnIcs / 4];
  __shared__ int s_fh[3][H / 16];  // PinnSync flags of the three activation buffers' tiles
  __shared__ int s_fs[D / 16];     // ... and of the state's
  __shared__ f4v s_bias4[kMaxChainLayers * H / 4];  // layer l's bias at l * H
  // the split last layer's partial sums and flags (PinnSplit)
#ifdef HF_EXP_PINN_NOSPLIT  // A/B: the clamped spare tile of round 5
  constexpr bool kSplit = false;
#else
  constexpr bool kSplit = 2 * (D / 16 - kPinnWaves) == kPinnWaves && NT == 2 && (H / 16) % 2 == 0;
#endif
  __shared__ f4v s_part[kSplit ? (D / 16 - kPinnWaves) * 64 : 1];
  __shared__ int s_flag[kSplit ? D / 16 - kPinnWaves : 1];
  float *s_state = reinterpret_cast<float *>(s_state4);
  float *const act0 = reinterpret_cast<float *>(s_act4[0]), *const act1 = reinterpret_cast<float *>(s_act4[1]);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t b0 = (int64_t)blockIdx.x * kPinnIcs;
  static_assert(NTH == 256 || NTH == 512 || NTH == 1024, "4, 8 or 16 waves");
  const int64_t ldt = (int64_t)(T + 1) * D;
  for (int idx = tid; idx < kPinnIcs * D; idx += NTH) {
    const int n = idx / D, d = idx - n * D;
    const int64_t b = b0 + n < B ? b0 + n : B - 1;  // missing ICs mirror the last one and write nothing
    const float v = state0[b * D + d];
    s_state[pinn_at(d, n)] = v;
    if (traj && b0 + n < B) traj[b * ldt + d] = v;
  }
  const int L = w.L;
#ifdef HF_EXP_PINN_PRIO  // experiment: static issue priority 1 for the second-dispatched half (waves 4-7)
  if (wave >= kPinnWaves / 2) __builtin_amdgcn_s_setprio(1);
#endif
  if (kSplit && tid < D / 16 - kPinnWaves) s_flag[tid] = 0;
  if (tid < 3 * (H / 16)) s_fh[tid / (H / 16)][tid % (H / 16)] = 0;
  if (tid < D / 16) s_fs[tid] = 0;
  float *const s_bias = reinterpret_cast<float *>(s_bias4);
  for (int l = 0; l < L; ++l)
    for (int i = tid; i < (l == L - 1 ? D : H); i += NTH) s_bias[l * H + i] = w.b[l][i];
  __syncthreads();
  // this wave's packed weight rows of layer l: output tiles min(wave + kPinnWaves j, tiles - 1), k-block 0
  auto row = [&](int l) {
    const int tiles = l == L - 1 ? D / 16 : H / 16, kb = l == 0 ? D / 16 : H / 16;
    PinnRows<NT> r;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      int t = wave + kPinnWaves * j;
      if (kSplit && j == 1 && l == L - 1 && l > 0) t = kPinnWaves + wave % (D / 16 - kPinnWaves);  // PinnSplit
      r.p[j] = w.wp[l] + ((int64_t)(t < tiles ? t : tiles - 1) * kb * 64 + lane) * 4;
    }
    return r;
  };
  f4v wq[kPinnAhead][NT];
  {
    const PinnRows<NT> r0 = row(0);
#pragma unroll
    for (int kb = 0; kb < kPinnAhead - 1; ++kb)
#pragma unroll
      for (int j = 0; j < NT; ++j) wq[kb][j] = *reinterpret_cast<const f4v *>(r0.p[j] + 256 * kb);
  }
  if constexpr (kFlags) {
    float *const act2 = reinterpret_cast<float *>(s_act4[kFlags ? 2 : 0]);
    auto hb = [&](int i) { return i == 0 ? act0 : (i == 1 ? act1 : act2); };
    const int nic = B - b0 < kPinnIcs ? (int)(B - b0) : kPinnIcs;
    for (int t = 0; t < T; ++t) {
      const int G = t * L;  // tags: layer l of step t publishes G + l + 1
      pinn_layer<D, H / 16, 0, H / 16, NT>(row(0), s_bias, s_state, hb(0), wave, lane, wq, row(1), PinnSplit{},
                                           PinnSync{s_fs, G, s_fh[0], G + 1});
      for (int l = 1; l < L - 1; ++l)
        pinn_layer<H, H / 16, 0, H / 16, NT>(row(l), s_bias + l * H, hb((l - 1) % 3), hb(l % 3), wave, lane, wq,
                                             row(l + 1), PinnSplit{},
                                             PinnSync{s_fh[(l - 1) % 3], G + l, s_fh[l % 3], G + l + 1});
      PinnSync sl{s_fh[(L - 2) % 3], G + L - 1, s_fs, G + L,
                  traj ? traj + b0 * ldt + (int64_t)(t + 1) * D : nullptr, ldt, nic};
      if constexpr (kSplit)
        pinn_layer<H, D / 16, 1, D / 16, NT, true>(row(L - 1), s_bias + (L - 1) * H, hb((L - 2) % 3), s_state, wave,
                                                   lane, wq, row(0), PinnSplit{s_part, s_flag, t + 1}, sl);
      else
        pinn_layer<H, D / 16, 1, D / 16, NT>(row(L - 1), s_bias + (L - 1) * H, hb((L - 2) % 3), s_state, wave, lane,
                                             wq, row(0), PinnSplit{}, sl);
    }
    __syncthreads();  // every wave's last state tiles stored
  }
  for (int t = 0; t < (kFlags ? 0 : T); ++t) {
    pinn_layer<D, H / 16, 0, H / 16, NT>(row(0), s_bias, s_state, act0, wave, lane, wq, row(1));
    __syncthreads();
    for (int l = 1; l < L - 1; ++l) {
      pinn_layer<H, H / 16, 0, H / 16, NT>(row(l), s_bias + l * H, (l & 1) ? act0 : act1, (l & 1) ? act1 : act0, wave, lane, wq,
                                       row(l + 1));
      __syncthreads();
    }
    if constexpr (kSplit)
      pinn_layer<H, D / 16, 1, D / 16, NT, true>(row(L - 1), s_bias + (L - 1) * H, (L & 1) ? act1 : act0, s_state, wave,
                                                 lane, wq, row(0), PinnSplit{s_part, s_flag, t + 1});
    else
      pinn_layer<H, D / 16, 1, D / 16, NT>(row(L - 1), s_bias + (L - 1) * H, (L & 1) ? act1 : act0, s_state, wave, lane,
                                           wq, row(0));
    __syncthreads();
    if (traj) {
      for (int idx = tid; idx < kPinnIcs * D; idx += NTH) {
        const int n = idx / D, d = idx - n * D;
        if (b0 + n < B) traj[(b0 + n) * ldt + (int64_t)(t + 1) * D + d] = s_state[pinn_at(d, n)];
      }
    }
  }
  for (int idx = tid; idx < kPinnIcs * D; idx += NTH) {
    const int n = idx / D, d = idx - n * D;
    if (b0 + n < B) final_state[(b0 + n) * D + d] = s_state[pinn_at(d, n)];
  }
}

// ---------------------------------------------------------------------------
// PureGNN rollout in one launch (train_pure_gnn.py:57-76 iterated as
// evaluate_multi_ic.py:45-66): a workgroup owns ONE IC for all T steps, its
// state and hidden activations in LDS; node features [n, u, E, x] are formed
// there each step.  Every GEMM runs as v_mfma_f32_16x16x4_f32 tiles (16 output
// features x 16 cells) with the weight operand read straight from nn.Linear's
// rows (float4 per lane: the PINN kernel's permuted k order) and the
// activations held in LDS as [k-block][cell group g][lane][4], cell group g
// holding cells NC c + g (c = lane & 15): the chain kernels' interleaved layout,
// so a cell's neighbours are in the same lane of the next group, or one DPP row
// rotation away at the group ends (periodic: row_ror wraps lane 15 to lane 0).
//  * message layer: wave u computes P and Q (W_a h and W_b h, rows of
//    update_mlps.l.0) for features 16u .. 16u + 15 over all cells; after a
//    barrier (every read of h done) it finishes those features in registers:
//    h += tanh(P[i-1] + Q[i] + b) + tanh(P[i+1] + Q[i] + b), messages in edge
//    order (from i-1, then i+1, as index_add_), and writes them back in place;
//  * output_mlp: o = tanh(W_o1 h + b) as tiles into LDS, then the 3 x nx
//    outputs as dot products; state += delta (benchmark_timing.py:128-130).
// A workgroup is H/16 waves; two share a CU, so one's epilogue runs beside
// the other's MFMAs.  Shapes: nx = 16 NC (NC <= 4), H in {64, 128}.
template <int NC>
__device__ __forceinline__ int pure_act_idx(int f, int cell) {
  const int g = cell % NC, c = cell / NC;
  return (((f >> 4) * NC + g) * 64 + ((f >> 2) & 3) * 16 + c) * 4 + (f & 3);
}
__device__ __forceinline__ float dpp_ror(float v, int ctrl_is_15) {
  const int iv = __builtin_bit_cast(int, v);
  return __builtin_bit_cast(float, ctrl_is_15 ? __builtin_amdgcn_mov_dpp(iv, 0x12F, 0xf, 0xf, false)
                                              : __builtin_amdgcn_mov_dpp(iv, 0x121, 0xf, 0xf, false));
}

// acc[j][g] (j < NR row tiles) = rows of W X over cell group g; row tile j's
// weight row for lane row m (0..15) is rowptr(j, m), K floats each.
template <int K, int NC, int NR, class RowPtr>
__device__ __forceinline__ void pure_tiles(const RowPtr &rowptr, const float *act, int lane, f4v (&acc)[NR][NC]) {
  constexpr int KB = K / 16, P = 3;
  const float *wr[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    wr[j] = rowptr(j, lane & 15) + 4 * (lane >> 4);
#pragma unroll
    for (int g = 0; g < NC; ++g) acc[j][g] = f4v{0.f, 0.f, 0.f, 0.f};
  }
  f4v wq[P][NR];
#pragma unroll
  for (int kb = 0; kb < KB + P - 1; ++kb) {
    if (kb < KB) {
#pragma unroll
      for (int j = 0; j < NR; ++j) wq[kb % P][j] = *reinterpret_cast<const f4v *>(wr[j] + 16 * kb);
    }
    if (kb >= P - 1) {
      const int c = kb - (P - 1);
#pragma unroll
      for (int g = 0; g < NC; ++g) {
        const f4v bv = *reinterpret_cast<const f4v *>(act + ((c * NC + g) * 64 + lane) * 4);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int j = 0; j < NR; ++j)
            acc[j][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(wq[c % P][j][e], bv[e], acc[j][g], 0, 0, 0);
      }
    }
  }
}

// pure_tiles on packed weights (pure_pack_kernel): row tile j's k-block kb is
// the contiguous 1 KiB at base + (j * KB + kb) * 256 — whole 128-B lines per
// load, where nn.Linear's rows give a load 16 rows x 64 B (half lines)
template <int K, int NC, int NR>
__device__ __forceinline__ void pure_tiles_packed(const float *base, const float *act, int lane, f4v (&acc)[NR][NC]) {
  constexpr int KB = K / 16, P = 3;
  const float *wr[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    wr[j] = base + (int64_t)j * KB * 256 + lane * 4;
#pragma unroll
    for (int g = 0; g < NC; ++g) acc[j][g] = f4v{0.f, 0.f, 0.f, 0.f};
  }
  // explicit software pipeline, as pinn_layer: k-blocks c+1 .. c+P-1 in flight
  // while c is multiplied, one scheduling region per k-block
  f4v wq[P][NR];
#pragma unroll
  for (int kb = 0; kb < P - 1; ++kb)
#pragma unroll
    for (int j = 0; j < NR; ++j) wq[kb][j] = *reinterpret_cast<const f4v *>(wr[j] + 256 * kb);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int c = 0; c < KB; ++c) {
    if (c + P - 1 < KB) {
#pragma unroll
      for (int j = 0; j < NR; ++j) wq[(c + P - 1) % P][j] = *reinterpret_cast<const f4v *>(wr[j] + 256 * (c + P - 1));
    }
#pragma unroll
    for (int g = 0; g < NC; ++g) {
      const f4v bv = *reinterpret_cast<const f4v *>(act + ((c * NC + g) * 64 + lane) * 4);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int j = 0; j < NR; ++j)
          acc[j][g] = __builtin_amdgcn_mfma_f32_16x16x4f32(wq[c % P][j][e], bv[e], acc[j][g], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}
// rows r0 + 16 u + (lane & 15), columns c0 + 16 kb + 4 (lane >> 4) + e of a row-major [*][ld] matrix
__global__ void pure_pack_kernel(const float *__restrict__ W, int64_t ld, int rows, int K, int nj, int64_t jcol,
                                 float *__restrict__ P) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int KB = K / 16;
  if (i >= (int64_t)rows * K * nj) return;
  const int e = (int)(i & 3), lane = (int)((i >> 2) & 63);
  int64_t r = i >> 8;  // ((u * nj + j) * KB + kb)
  const int kb = (int)(r % KB);
  r /= KB;
  const int j = (int)(r % nj), u = (int)(r / nj);
  P[i] = W[(int64_t)(16 * u + (lane & 15)) * ld + j * jcol + 16 * kb + 4 * (lane >> 4) + e];
}

#ifndef HF_PURE_WG
#define HF_PURE_WG 2
#endif
template <int H, int NC, bool PACKED>
__global__ __launch_bounds__(64 * (H / 16), HF_PURE_WG) void pure_run_kernel(PureW w, const float *__restrict__ state0,
                                                                    float *__restrict__ final_state,
                                                                    const float *__restrict__ x,
                                                                    float *__restrict__ traj, int B, int T) {
  constexpr int NX = 16 * NC, NTH = 64 * (H / 16);
  __shared__ float s_st[3 * NX];
  __shared__ float s_x[NX];
  // two activation buffers: a layer reads h from one and writes h' to the
  // other, so no barrier has to separate every wave's reads of h from the
  // in-place rewrite (one barrier per layer instead of two)
  __shared__ f4v s_act4[2][H * NX / 4];
  float *act = reinterpret_cast<float *>(s_act4[0]), *act2 = reinterpret_cast<float *>(s_act4[1]);
  const int tid = threadIdx.x, u = tid >> 6, lane = tid & 63, q4 = 4 * (lane >> 4);
  const int64_t b = blockIdx.x;
  const int64_t ldt = (int64_t)(T + 1) * 3 * NX;
  for (int i = tid; i < 3 * NX; i += NTH) {
    const float v = state0[b * 3 * NX + i];
    s_st[i] = v;
    if (traj) traj[b * ldt + i] = v;
  }
  for (int i = tid; i < NX; i += NTH) s_x[i] = x[i];
#ifdef HF_EXP_PURE_PRIO  // experiment: static issue priority 1 for the second-dispatched half
  if (u >= H / 32) __builtin_amdgcn_s_setprio(1);
#endif
  __syncthreads();
#ifndef HF_PURE_MFMA_IO
#define HF_PURE_MFMA_IO 1
#endif
  for (int t = 0; t < T; ++t) {
    // input_mlp: h = tanh(W_in [n, u, E, x] + b_in)
    if (HF_PURE_MFMA_IO) {
      // on the matrix core: one v_mfma_f32_16x16x4f32 per cell group, A = rows
      // 16u .. 16u+15 of W_in (lane: row lane & 15, input lane >> 4), B = the
      // group's [n, u, E, x] (lane: input lane >> 4 of cell NC (lane & 15) + g);
      // its output tile is the activation layout's (feature 16u + 4 (lane >> 4)
      // + i of cell column lane & 15).  The f32 MFMA's sum is an fmaf chain over
      // the 4 inputs (MI355X_MICROARCH.md), as the VALU form's; + b_in, tanh pairs.
      const float a = w.w_in[(16 * u + (lane & 15)) * 4 + (lane >> 4)];
      f4v bi;
#pragma unroll
      for (int i = 0; i < 4; ++i) bi[i] = w.b_in[16 * u + q4 + i];
#pragma unroll
      for (int g = 0; g < NC; ++g) {
        const int cell = NC * (lane & 15) + g, k = lane >> 4;
        const float bf = k < 3 ? s_st[k * NX + cell] : s_x[cell];
        const f4v z = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bf, f4v{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        f4v h;
#pragma unroll
        for (int i = 0; i < 4; i += 2) {
          const hf_f2 th = tanh_fast2(hf_f2{__fadd_rn(z[i], bi[i]), __fadd_rn(z[i + 1], bi[i + 1])});
          h[i] = th.x, h[i + 1] = th.y;
        }
        *reinterpret_cast<f4v *>(act + ((u * NC + g) * 64 + lane) * 4) = h;
      }
    } else {
      for (int idx = tid; idx < H * NX; idx += NTH) {
        const int f = idx / NX, c = idx - f * NX;
        const float *wi = w.w_in + f * 4;
        float v = __fmul_rn(wi[0], s_st[c]);
        v = __fmaf_rn(wi[1], s_st[NX + c], v);
        v = __fmaf_rn(wi[2], s_st[2 * NX + c], v);
        v = __fmaf_rn(wi[3], s_x[c], v);
        act[pure_act_idx<NC>(f, c)] = tanh_fast(__fadd_rn(v, w.b_in[f]));
      }
    }
    __syncthreads();
    for (int l = 0; l < w.L; ++l) {
      const float *W = w.w_l + l * w.ls, *bl = w.b_l + l * w.ls;
      f4v acc[2][NC];  // [P | Q][cell group]
      if constexpr (PACKED)
        pure_tiles_packed<H, NC, 2>(w.w_lp + ((int64_t)l * (H / 16) + u) * 2 * (H / 16) * 256, act, lane, acc);
      else
        pure_tiles<H, NC, 2>([&](int j, int m) { return W + (int64_t)(16 * u + m) * 2 * H + j * H; }, act, lane, acc);
      f4v bq;
#pragma unroll
      for (int i = 0; i < 4; ++i) bq[i] = bl[16 * u + q4 + i];
#pragma unroll
      for (int g = 0; g < NC; ++g) {
        const int o = ((u * NC + g) * 64 + lane) * 4;
        f4v h = *reinterpret_cast<const f4v *>(act + o);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          // cell NC c + g: left (g - 1, c) or, at g = 0, (NC - 1, c - 1); right (g + 1, c) or (0, c + 1)
          const float pl = g > 0 ? acc[0][g - 1][i] : dpp_ror(acc[0][NC - 1][i], 0);
          const float pr = g < NC - 1 ? acc[0][g + 1][i] : dpp_ror(acc[0][0][i], 1);
          const float qv = acc[1][g][i];
#ifndef HF_PURE_TANH2
#define HF_PURE_TANH2 1
#endif
          if (HF_PURE_TANH2) {  // the two messages' tanh as packed f32 (bit-identical)
            const hf_f2 t = tanh_fast2((hf_f2{pl, pr} + qv) + bq[i]);
            h[i] = __fadd_rn(h[i], __fadd_rn(t.x, t.y));
          } else {
            float m = tanh_fast(__fadd_rn(__fadd_rn(pl, qv), bq[i]));
            m = __fadd_rn(m, tanh_fast(__fadd_rn(__fadd_rn(pr, qv), bq[i])));
            h[i] = __fadd_rn(h[i], m);
          }
        }
        *reinterpret_cast<f4v *>(act2 + o) = h;
      }
      __syncthreads();
      float *tmp = act;
      act = act2;
      act2 = tmp;
    }
    // output_mlp.0: o = tanh(W_o1 h + b_o1), written over h once every wave has read it
    {
      f4v acc[1][NC];
      if constexpr (PACKED)
        pure_tiles_packed<H, NC, 1>(w.w_o1p + (int64_t)u * (H / 16) * 256, act, lane, acc);
      else
        pure_tiles<H, NC, 1>([&](int, int m) { return w.w_o1 + (int64_t)(16 * u + m) * H; }, act, lane, acc);
      f4v bo;
#pragma unroll
      for (int i = 0; i < 4; ++i) bo[i] = w.b_o1[16 * u + q4 + i];
#pragma unroll
      for (int g = 0; g < NC; ++g) {
        f4v o;
#pragma unroll
        for (int i = 0; i < 4; i += 2) {  // packed pairs (bit-identical to tanh_fast)
          const hf_f2 t = tanh_fast2(hf_f2{acc[0][g][i], acc[0][g][i + 1]} + hf_f2{bo[i], bo[i + 1]});
          o[i] = t.x, o[i + 1] = t.y;
        }
        *reinterpret_cast<f4v *>(act2 + ((u * NC + g) * 64 + lane) * 4) = o;
      }
    }
    __syncthreads();
    {
      float *tmp = act;
      act = act2;
      act2 = tmp;
    }
    // output_mlp.2 and the update: state += W_o2 o + b_o2
    if (HF_PURE_MFMA_IO) {
      // on the matrix core: wave g < NC takes cell group g, A = the 3 rows of
      // W_o2 (rows 3..15 zero; the packed weights' k order), B = o as stored:
      // H/16 k-blocks x 4 MFMA steps; channel ch of cell NC c + g lands in lane
      // c, element ch
      if (u < NC) {
        const int g = u, row = lane & 15;
        f4v acc = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kb = 0; kb < H / 16; ++kb) {
          const f4v av = row < 3 ? *reinterpret_cast<const f4v *>(w.w_o2 + row * H + 16 * kb + q4)
                                 : f4v{0.f, 0.f, 0.f, 0.f};
          const f4v bv = *reinterpret_cast<const f4v *>(act + ((kb * NC + g) * 64 + lane) * 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[e], bv[e], acc, 0, 0, 0);
        }
        if (lane < 16) {
          const int cell = NC * lane + g;
#pragma unroll
          for (int ch = 0; ch < 3; ++ch)
            s_st[ch * NX + cell] = __fadd_rn(s_st[ch * NX + cell], __fadd_rn(acc[ch], w.b_o2[ch]));
        }
      }
    } else if (tid < 3 * NX) {
      const int ch = tid / NX, c = tid - ch * NX;
      const float *wo = w.w_o2 + ch * H;
      float v = 0.f;
      for (int f = 0; f < H; ++f) v = __fmaf_rn(wo[f], act[pure_act_idx<NC>(f, c)], v);
      s_st[tid] = __fadd_rn(s_st[tid], __fadd_rn(v, w.b_o2[ch]));
    }
    __syncthreads();
    if (traj)
      for (int i = tid; i < 3 * NX; i += NTH) traj[b * ldt + (int64_t)(t + 1) * 3 * NX + i] = s_st[i];
  }
  for (int i = tid; i < 3 * NX; i += NTH) final_state[b * 3 * NX + i] = s_st[i];
}

#ifndef HF_PURE_FUSED
#define HF_PURE_FUSED 1
#endif
bool pure_fused_ok(int H, int nx) { return (H == 64 || H == 128) && nx % 16 == 0 && nx >= 16 && nx <= 64; }

// floats of the one-launch PureGNN rollout's packed weights (L layers, width H)
int64_t pure_packed_floats(int H, int L) { return (int64_t)L * 2 * H * H + (int64_t)H * H; }

template <int H, bool PACKED>
void pure_fused_launch(const PureW &w, const float *state0, float *final_state, const float *x, int B, int nx, int T,
                       float *traj, hipStream_t s) {
  switch (nx / 16) {
    case 1: hipLaunchKernelGGL((pure_run_kernel<H, 1, PACKED>), dim3(B), dim3(64 * (H / 16)), 0, s, w, state0, final_state, x, traj, B, T); break;
    case 2: hipLaunchKernelGGL((pure_run_kernel<H, 2, PACKED>), dim3(B), dim3(64 * (H / 16)), 0, s, w, state0, final_state, x, traj, B, T); break;
    case 3: hipLaunchKernelGGL((pure_run_kernel<H, 3, PACKED>), dim3(B), dim3(64 * (H / 16)), 0, s, w, state0, final_state, x, traj, B, T); break;
    default: hipLaunchKernelGGL((pure_run_kernel<H, 4, PACKED>), dim3(B), dim3(64 * (H / 16)), 0, s, w, state0, final_state, x, traj, B, T); break;
  }
}

// ws: the packed copy (pure_packed_floats(H, kMaxChainLayers) floats, hf_pure_gnn_run_workspace_bytes),
// made here from the state-dict-order weights; more layers than that run on nn.Linear's rows
template <int H>
hipError_t pure_fused_h(const PureW &w0, const float *state0, float *final_state, const float *x, int B, int nx, int T,
                        float *traj, void *ws, hipStream_t s) {
  PureW w = w0;
  if (ws && w.L <= kMaxChainLayers) {
    float *packed = static_cast<float *>(ws);
    const int64_t nl = (int64_t)w.L * 2 * H * H, no = (int64_t)H * H;
    for (int l = 0; l < w.L; ++l)
      hipLaunchKernelGGL(pure_pack_kernel, dim3((unsigned)((2LL * H * H + 255) / 256)), dim3(256), 0, s,
                         w.w_l + l * w.ls, (int64_t)2 * H, H, H, 2, (int64_t)H, packed + (int64_t)l * 2 * H * H);
    hipLaunchKernelGGL(pure_pack_kernel, dim3((unsigned)((no + 255) / 256)), dim3(256), 0, s, w.w_o1, (int64_t)H, H, H,
                       1, (int64_t)0, packed + nl);
    w.w_lp = packed;
    w.w_o1p = packed + nl;
    pure_fused_launch<H, true>(w, state0, final_state, x, B, nx, T, traj, s);
  } else {
    pure_fused_launch<H, false>(w, state0, final_state, x, B, nx, T, traj, s);
  }
  return hipGetLastError();
}

// the one-launch rollout's shapes: the reference's PINN(3 * 64, 256, L)
bool pinn_fused_ok(int D, int H, int L) { return D == 192 && H == 256 && L >= 2 && L <= kMaxChainLayers; }

// The one-launch rollout's weight layout.  nn.Linear's [out][in] rows give a
// wave's float4-per-lane k-block 16 rows x 64 B: half of each 128-B line per
// load, the other half re-requested by the next k-block's load.  Packed as
// [tile][k-block][lane][4] (element (t, kb, lane, e) = W[16t + (lane & 15)][16kb
// + 4(lane >> 4) + e]) a k-block is one contiguous 1 KiB: 8 whole lines.  One
// launch packs every layer (thread i of the concatenated packed arrays finds
// its layer in the table); the packed copy lives in the caller's workspace.
struct PinnPack {
  const float *w[kMaxChainLayers];
  int64_t off[kMaxChainLayers + 1];  // packed float offsets, off[L] = total
  int in[kMaxChainLayers];
  int L;
};
__global__ void pinn_pack_kernel(PinnPack pk, float *__restrict__ P) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= pk.off[pk.L]) return;
  int l = 0;
  while (l + 1 < pk.L && i >= pk.off[l + 1]) ++l;
  const int64_t q = i - pk.off[l];
  const int in = pk.in[l], KB = in / 16;
  const int e = (int)(q & 3), lane = (int)((q >> 2) & 63);
  const int64_t r = q >> 8;  // t * KB + kb
  const int kb = (int)(r % KB), t = (int)(r / KB);
  P[i] = pk.w[l][(int64_t)(16 * t + (lane & 15)) * in + 16 * kb + 4 * (lane >> 4) + e];
}

// floats of the packed copy for L layers (pinn_fused_ok shapes)
int64_t pinn_packed_floats(int D, int H, int L) {
  int64_t n = 0;
  for (int l = 0; l < L; ++l) n += (int64_t)(l == 0 ? D : H) * (l == L - 1 ? D : H);
  return n;
}

hipError_t pinn_fused(const PinnW &w0, const float *state0, float *final_state, int64_t B, int T, float *traj,
                      void *ws, hipStream_t s) {
  const int64_t blocks = (B + kPinnIcs - 1) / kPinnIcs;
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  PinnW w = w0;
  PinnPack pk{};
  pk.L = w.L;
  float *packed = static_cast<float *>(ws);  // >= pinn_packed_floats(D, H, kMaxChainLayers) floats (caller-checked)
  for (int l = 0; l < w.L; ++l) {
    pk.w[l] = w.w[l];
    pk.in[l] = l == 0 ? w.D : w.H;
    pk.off[l + 1] = pk.off[l] + (int64_t)pk.in[l] * (l == w.L - 1 ? w.D : w.H);
    w.wp[l] = packed + pk.off[l];
  }
  hipLaunchKernelGGL(pinn_pack_kernel, dim3((unsigned)((pk.off[w.L] + 255) / 256)), dim3(256), 0, s, pk, packed);
  hipLaunchKernelGGL((pinn_run_kernel<192, 256>), dim3((unsigned)blocks), dim3(64 * kPinnWaves), 0, s, w, state0, final_state,
                     traj, B, T);
  return hipGetLastError();
}

}  // namespace

int64_t pure_gnn_ws_bytes(int H, int64_t N, int64_t E) {
  return (int64_t)(4 * a256(sizeof(float) * N * H) + a256(sizeof(float) * N * 4) + a256(sizeof(float) * N * 3) +
                   2 * a256(sizeof(float) * N * 3)) +
         edge_buckets_bytes(N, E);
}

hipError_t launch_pure_gnn_forward(const float *params, int in_dim, int H, int L, const float *nf, int64_t N,
                                   const int64_t *ei, int64_t E, int chain_nx, float *delta, void *ws, hipStream_t s) {
  const PureW w = pure_view(params, in_dim, H, L);
  PureWs b = carve_pure(ws, H, N);
  int *off = nullptr, *perm = nullptr;
  hipError_t e;
  if (!chain_nx && (e = edge_buckets(ei + E, E, N, 0, true, b.buckets, &off, &perm, s))) return e;  // by dst (:65)
  return pure_forward(w, nf, N, ei, off, perm, chain_nx, b, delta, s);
}

// evaluate_multi_ic.py:45-66 for B ICs at once: traj [B][T+1][3][nx] (optional).
hipError_t launch_pure_gnn_run(const float *params, int H, int L, const float *state0, float *final_state,
                               const float *x, int B, int nx, int T, float *traj, void *ws, hipStream_t s) {
  const PureW w = pure_view(params, 4, H, L);
  const int64_t N = (int64_t)B * nx, S = 3LL * nx;
  const int64_t ldt = (T + 1) * S;
  hipError_t e;
  if (HF_PURE_FUSED && T > 0 && pure_fused_ok(H, nx))  // one launch (it writes trajectory row 0 itself; ws: packed weights)
    return H == 64 ? pure_fused_h<64>(w, state0, final_state, x, B, nx, T, traj, ws, s)
                   : pure_fused_h<128>(w, state0, final_state, x, B, nx, T, traj, ws, s);
  if (traj && (e = hipMemcpy2DAsync(traj, sizeof(float) * ldt, state0, sizeof(float) * S, sizeof(float) * S, B,
                                    hipMemcpyDeviceToDevice, s)))
    return e;
  if (T == 0) return hipMemcpyAsync(final_state, state0, sizeof(float) * N * 3, hipMemcpyDeviceToDevice, s);
  PureWs b = carve_pure(ws, H, N);  // (the workspace is non-NULL on this path: hf_pure_gnn_run checks)
  float *st[2] = {reinterpret_cast<float *>(b.buckets),
                  reinterpret_cast<float *>(static_cast<char *>(b.buckets) + a256(sizeof(float) * N * 3))};
  const unsigned nb = (unsigned)((N + 255) / 256), sb = (unsigned)((N * 3 + 255) / 256);
  const float *cur = state0;
  for (int t = 0; t < T; ++t) {
    hipLaunchKernelGGL(chain_features_kernel, dim3(nb), dim3(256), 0, s, cur, x, (int64_t)B, nx, b.nf);
    if ((e = pure_forward(w, b.nf, N, nullptr, nullptr, nullptr, nx, b, b.delta, s))) return e;
    float *nxt = t == T - 1 ? final_state : st[t & 1];
    hipLaunchKernelGGL(add_delta_kernel, dim3(sb), dim3(256), 0, s, cur, b.delta, (int64_t)B, nx, nxt,
                       traj ? traj + (t + 1) * S : nullptr, ldt);
    cur = nxt;
  }
  return hipGetLastError();
}

int64_t pinn_ws_bytes(int D, int H, int64_t B) {
  return (int64_t)(2 * a256(sizeof(float) * B * H) + 2 * a256(sizeof(float) * B * D));
}

int64_t pure_gnn_run_ws_bytes(int H, int B, int nx, int T) {
  if (B == 0 || T == 0) return 0;
  if (HF_PURE_FUSED && pure_fused_ok(H, nx))  // the packed weights, for up to kMaxChainLayers layers
    return (int64_t)a256(sizeof(float) * pure_packed_floats(H, kMaxChainLayers));
  return pure_gnn_ws_bytes(H, (int64_t)B * nx, 2LL * B * nx);
}

bool pure_gnn_run_ws_optional(int H, int nx, int T) { return HF_PURE_FUSED && T > 0 && pure_fused_ok(H, nx); }

int64_t pinn_run_ws_bytes(int D, int H, int64_t B) {
  // the one-launch shape: the packed weight copy, sized for the most layers the ABI admits
  if (B == 0) return 0;
  return pinn_fused_ok(D, H, 2) ? (int64_t)a256(sizeof(float) * pinn_packed_floats(D, H, kMaxChainLayers))
                                : pinn_ws_bytes(D, H, B);
}

hipError_t launch_pinn_forward(const float *params, int D, int H, int L, const float *state, float *out, int64_t B,
                               void *ws, hipStream_t s) {
  const PinnW w = pinn_view(params, D, H, L);
  if (pinn_fused_ok(D, H, L)) return B > 0 ? pinn_fused(w, state, out, B, 1, nullptr, ws, s) : hipSuccess;
  float *buf[2] = {static_cast<float *>(ws),
                   reinterpret_cast<float *>(static_cast<char *>(ws) + a256(sizeof(float) * B * H))};
  const float *in = state;
  hipError_t e;
  for (int l = 0; l < L; ++l) {
    const int K = l == 0 ? D : H;
    const bool last = l == L - 1;
    float *o = last ? out : buf[l & 1];
    if ((e = gemm_linear(in, K, nullptr, nullptr, 0, nullptr, wv_rows(w.w[l], K, K), w.b[l], o, B, last ? D : H,
                         last ? kActNone : kActTanh, last ? state : nullptr, s)))
      return e;
    in = o;
  }
  return hipSuccess;
}

// evaluate_multi_ic.py:70-83 for B ICs at once: traj [B][T+1][D] (optional).
hipError_t launch_pinn_run(const float *params, int D, int H, int L, const float *state0, float *final_state,
                           int64_t B, int T, float *traj, void *ws, hipStream_t s) {
  const size_t row = sizeof(float) * D, ldt = row * (T + 1);
  hipError_t e;
  // one launch (the kernel writes trajectory row 0 itself; the workspace holds the packed weights)
  if (T > 0 && pinn_fused_ok(D, H, L))
    return B > 0 ? pinn_fused(pinn_view(params, D, H, L), state0, final_state, B, T, traj, ws, s) : hipSuccess;
  if (traj && (e = hipMemcpy2DAsync(traj, ldt, state0, row, row, B, hipMemcpyDeviceToDevice, s))) return e;
  if (T == 0) return hipMemcpyAsync(final_state, state0, row * B, hipMemcpyDeviceToDevice, s);
  char *p = static_cast<char *>(ws) + 2 * a256(sizeof(float) * B * H);  // non-NULL here: hf_pinn_run checks
  float *st[2] = {reinterpret_cast<float *>(p), reinterpret_cast<float *>(p + a256(sizeof(float) * B * D))};
  const float *cur = state0;
  for (int t = 0; t < T; ++t) {
    float *nxt = t == T - 1 ? final_state : st[t & 1];
    if ((e = launch_pinn_forward(params, D, H, L, cur, nxt, B, ws, s))) return e;
    if (traj && (e = hipMemcpy2DAsync(reinterpret_cast<char *>(traj) + (t + 1) * row, ldt, nxt, row, row, B,
                                      hipMemcpyDeviceToDevice, s)))
      return e;
    cur = nxt;
  }
  return hipSuccess;
}

}  // namespace hf
