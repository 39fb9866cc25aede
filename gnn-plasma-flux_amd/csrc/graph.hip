// FluxGNN on an arbitrary graph (src/flux_gnn.py:40-67), float32: inference,
// and the training forward + backward that make FluxGNN differentiable.
//
// This is the path for edge_index tensors that are not the periodic chain
// (examples/smoke_test.py:53 feeds a random one) and for training on any
// graph (scripts/training/train_ablation.py:120-206 calls loss.backward()
// through FluxGNN).  Chain inference — the hot path — never comes here; it
// runs in chain_f32.hip / chain_k32.hip.
//
//  * Mean aggregation is deterministic and in reference order: edges are
//    bucketed by destination row into a CSR whose segments are sorted by edge
//    id, so node i sums h[col[e]] in increasing e exactly like the serial
//    index_add_ (src/flux_gnn.py:57), then divides by max(deg,1) (:58-59).
//  * Linear layers are one LDS-tiled kernel computing
//    act(b + W [A1[r1(m)] ; A2[r2(m)]]) with optional row gathers, so the
//    concatenations of :60 and :62-64 are never materialised.  The weight is
//    read through a strided view, so the same kernel multiplies by W^T in
//    the backward pass without a transposed copy.
//  * Weight gradients dW = sum_m delta[m] (x) X[m] are a split-K reduction
//    over rows: each split writes its partial tile, a second kernel sums the
//    splits in a fixed order (deterministic, no atomics).
#include <algorithm>

#include "hf_device.h"
#include "hf_internal.h"

namespace hf {
namespace {



// ------------------------------------------------------------ MFMA GEMM core
// C[i][j] = sum_{r in [rb, re)} A(i, r) * B(j, r) for a 64 x 64 tile, on
// v_mfma_f32_16x16x4_f32: 4 waves, each a 32 x 32 quadrant (2 x 2 MFMA tiles).
// The reduction is staged through LDS in chunks of kKC, reduction-major
// (s[r][i]), with the next chunk prefetched into registers while the current
// one feeds the MFMAs.  Operands are functors (gathers, transposed weight
// views, ones column for the bias gradient); kRowFast picks the thread
// mapping that makes the operand's global reads contiguous.
typedef float f4v __attribute__((ext_vector_type(4)));
constexpr int kT = 64, kKC = 32, kPad = 4;
constexpr int kPer = kT * kKC / 256;  // elements per thread per operand per chunk

// in(m,k) = k < K1 ? A1[r1(m)][k] : A2[r2(m)][k-K1]   (rows m, reduction k)
struct OpIn {
  const float *A1, *A2;
  const int64_t *i1, *i2;
  int K1, K2;
  int64_t M;
  static constexpr bool kRowFast = false;
  __device__ float operator()(int64_t m, int64_t k) const {
    if (m >= M || k >= K1 + K2) return 0.f;
    return k < K1 ? A1[(i1 ? i1[m] : m) * K1 + k] : A2[(i2 ? i2[m] : m) * K2 + (k - K1)];
  }
};
// weight(o,k) through a WView                        (rows o, reduction k)
template <bool RF>
struct OpW {
  WView W;
  int O, K, K1;
  static constexpr bool kRowFast = RF;
  __device__ float operator()(int64_t o, int64_t k) const {
    if (o >= O || k >= K) return 0.f;
    return k < K1 ? W.w1[o * W.so + k * W.si] : W.w2[o * W.so + (k - K1) * W.si];
  }
};
// D^T: A(o, m) = D[m][o]                              (rows o, reduction m)
struct OpDT {
  const float *D;
  int O;
  int64_t me;
  static constexpr bool kRowFast = true;
  __device__ float operator()(int64_t o, int64_t m) const { return (o < O && m < me) ? D[m * O + o] : 0.f; }
};
// X^T with a ones column: B(k, m) = in(m,k) for k < K, 1 for k == K   (rows k, reduction m)
struct OpXT {
  OpIn in;
  int64_t me;
  static constexpr bool kRowFast = true;
  __device__ float operator()(int64_t k, int64_t m) const {
    if (m >= me) return 0.f;
    const int K = in.K1 + in.K2;
    return k < K ? in(m, k) : (k == K ? 1.f : 0.f);
  }
};

template <class Op>
__device__ __forceinline__ void gload(const Op &op, int64_t i0, int64_t r0, float (&v)[kPer]) {
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int e = threadIdx.x + 256 * q;
    const int i = Op::kRowFast ? e % kT : e / kKC, r = Op::kRowFast ? e / kT : e % kKC;
    v[q] = op(i0 + i, r0 + r);
  }
}
template <class Op>
__device__ __forceinline__ void lstore(float (*sm)[kT + kPad], const float (&v)[kPer]) {
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int e = threadIdx.x + 256 * q;
    const int i = Op::kRowFast ? e % kT : e / kKC, r = Op::kRowFast ? e / kT : e % kKC;
    sm[r][i] = v[q];
  }
}

// acc[ti][tj][x] = C[i0 + 32*wi + 16*ti + 4*(l>>4) + x][j0 + 32*wj + 16*tj + (l&15)]
template <class OA, class OB>
__device__ __forceinline__ void gemm_tile(const OA &A, const OB &B, int64_t i0, int64_t j0, int64_t rb, int64_t re,
                                          f4v (&acc)[2][2]) {
  __shared__ float sA[kKC][kT + kPad];
  __shared__ float sB[kKC][kT + kPad];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wi = wave >> 1, wj = wave & 1;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f4v{0.f, 0.f, 0.f, 0.f};
  float va[kPer], vb[kPer];
  if (rb < re) {
    gload(A, i0, rb, va);
    gload(B, j0, rb, vb);
  }
  for (int64_t r0 = rb; r0 < re; r0 += kKC) {
    lstore<OA>(sA, va);
    lstore<OB>(sB, vb);
    __syncthreads();
    if (r0 + kKC < re) {
      gload(A, i0, r0 + kKC, va);
      gload(B, j0, r0 + kKC, vb);
    }
#pragma unroll
    for (int s = 0; s < kKC / 4; ++s) {
      const int rr = 4 * s + (lane >> 4);
      float a[2], b[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        a[t] = sA[rr][32 * wi + 16 * t + (lane & 15)];
        b[t] = sB[rr][32 * wj + 16 * t + (lane & 15)];
      }
#pragma unroll
      for (int ta = 0; ta < 2; ++ta)
#pragma unroll
        for (int tb = 0; tb < 2; ++tb)
          acc[ta][tb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[ta], b[tb], acc[ta][tb], 0, 0, 0);
    }
    __syncthreads();
  }
}

// out[m][o] = resid[m][o] + act(bias[o] + sum_k weight(o,k) * in(m,k)) [* (mask[m][o] > 0)].
template <bool WRF>
__global__ __launch_bounds__(256) void linear_kernel(OpIn in, OpW<WRF> w, const float *__restrict__ bias,
                                                     float *out, int act, const float *__restrict__ mask,
                                                     const float *__restrict__ resid) {
  const int64_t m0 = (int64_t)blockIdx.x * kT;
  const int o0 = blockIdx.y * kT;
  f4v acc[2][2];
  gemm_tile(in, w, m0, o0, 0, in.K1 + in.K2, acc);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int O = w.O;
#pragma unroll
  for (int ta = 0; ta < 2; ++ta)
#pragma unroll
    for (int tb = 0; tb < 2; ++tb) {
      const int o = o0 + 32 * (wave & 1) + 16 * tb + (lane & 15);
      if (o >= O) continue;
      const float bo = bias ? bias[o] : 0.f;
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const int64_t m = m0 + 32 * (wave >> 1) + 16 * ta + 4 * (lane >> 4) + x;
        if (m >= in.M) continue;
        float v = bias ? __fadd_rn(acc[ta][tb][x], bo) : acc[ta][tb][x];
        if (act == kActRelu) v = relu(v);
        else if (act == kActTanh) v = tanhf(v);
        if (mask && !(mask[m * O + o] > 0.f)) v = 0.f;
        if (resid) v = __fadd_rn(resid[m * O + o], v);
        out[m * O + o] = v;
      }
    }
}

// part[s][o][k] = sum_{m in split s} D[m][o] * X(m,k), k <= K (k == K: bias column).
__global__ __launch_bounds__(256) void wgrad_kernel(const float *__restrict__ D, int O, OpIn in, int64_t R,
                                                    float *__restrict__ part) {
  const int o0 = blockIdx.x * kT, k0 = blockIdx.y * kT;
  const int64_t mb = (int64_t)blockIdx.z * R;
  const int64_t me = mb + R < in.M ? mb + R : in.M;
  const int KB = in.K1 + in.K2 + 1;
  f4v acc[2][2];
  gemm_tile(OpDT{D, O, me}, OpXT{in, me}, o0, k0, mb, me, acc);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int ta = 0; ta < 2; ++ta)
#pragma unroll
    for (int tb = 0; tb < 2; ++tb) {
      const int k = k0 + 32 * (wave & 1) + 16 * tb + (lane & 15);
      if (k >= KB) continue;
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const int o = o0 + 32 * (wave >> 1) + 16 * ta + 4 * (lane >> 4) + x;
        if (o < O) part[((int64_t)blockIdx.z * O + o) * KB + k] = acc[ta][tb][x];
      }
    }
}

// gw[o][k] = sum_s part[s][o][k] (k < K), gb[o] = sum_s part[s][o][K], in a fixed order.
__global__ void wgrad_reduce_kernel(const float *__restrict__ part, int S, int O, int K, float *gw, float *gb) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int KB = K + 1;
  if (t >= (int64_t)O * KB) return;
  const int o = (int)(t / KB), k = (int)(t - (int64_t)o * KB);
  const int64_t st = (int64_t)O * KB;
  float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;  // fixed association: ((s%4 lanes) then 0+1+2+3)
  int s = 0;
  for (; s + 4 <= S; s += 4) {
    v0 = __fadd_rn(v0, part[(int64_t)s * st + t]);
    v1 = __fadd_rn(v1, part[(int64_t)(s + 1) * st + t]);
    v2 = __fadd_rn(v2, part[(int64_t)(s + 2) * st + t]);
    v3 = __fadd_rn(v3, part[(int64_t)(s + 3) * st + t]);
  }
  for (; s < S; ++s) v0 = __fadd_rn(v0, part[(int64_t)s * st + t]);
  const float v = __fadd_rn(__fadd_rn(v0, v1), __fadd_rn(v2, v3));
  if (k < K) gw[(int64_t)o * K + k] = v;
  else if (gb) gb[o] = v;
}

__global__ void count_deg_kernel(const int64_t *__restrict__ key, int64_t E, int *deg) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < E) atomicAdd(&deg[key[e]], 1);
}

// Exclusive scan of deg[N] into off[N+1] by one 1024-thread block.
__global__ __launch_bounds__(1024) void scan_kernel(const int *__restrict__ deg, int64_t N,
                                                    int *__restrict__ off, int *__restrict__ cur) {
  __shared__ int s[1024];
  __shared__ int carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < N; base += 1024) {
    const int64_t i = base + threadIdx.x;
    const int v = i < N ? deg[i] : 0;
    s[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
      const int t = threadIdx.x >= o ? s[threadIdx.x - o] : 0;
      __syncthreads();
      s[threadIdx.x] += t;
      __syncthreads();
    }
    if (i < N) {
      off[i] = carry + s[threadIdx.x] - v;
      cur[i] = off[i];
    }
    __syncthreads();
    if (threadIdx.x == 1023) carry += s[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) off[N] = carry;
}

__global__ void fill_kernel(const int64_t *__restrict__ key, int64_t E, int *cur, int *__restrict__ perm) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < E) perm[atomicAdd(&cur[key[e]], 1)] = (int)e;
}

// Restore edge order inside each segment (insertion sort by id).
__global__ void sort_segments_kernel(const int *__restrict__ off, int64_t N, int *perm) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const int a = off[i], z = off[i + 1];
  for (int p = a + 1; p < z; ++p) {
    const int v = perm[p];
    int q = p - 1;
    while (q >= a && perm[q] > v) {
      perm[q + 1] = perm[q];
      --q;
    }
    perm[q + 1] = v;
  }
}

__global__ void aggregate_kernel(const float *__restrict__ h, const int64_t *__restrict__ col,
                                 const int *__restrict__ off, const int *__restrict__ perm,
                                 int64_t N, int H, float *__restrict__ agg) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N * H) return;
  const int64_t i = t / H;
  const int f = (int)(t - i * H);
  const int a = off[i], z = off[i + 1];
  float s = 0.f;
  for (int p = a; p < z; ++p) s = __fadd_rn(s, h[col[perm[p]] * H + f]);
  const int deg = z - a;
  agg[t] = __fdiv_rn(s, (float)(deg > 0 ? deg : 1));
}

// ------------------------------------------------------------- backward pieces
// dz[e][f] = g[e] * w2[f] where relu(z)[e][f] > 0   (d of w2 . relu(z) + b2)
__global__ void readout_delta_kernel(const float *__restrict__ g, const float *__restrict__ r,
                                     const float *__restrict__ w2, int64_t E, int H, float *__restrict__ dz) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= E * H) return;
  const int64_t e = t / H;
  const int f = (int)(t - e * H);
  dz[t] = r[t] > 0.f ? __fmul_rn(g[e], w2[f]) : 0.f;
}

// S_row[j] = sum over edges e with row[e] = j of dz[e]; S_col likewise by col.
__global__ void edge_scatter_kernel(const float *__restrict__ dz, const int *__restrict__ off_r,
                                    const int *__restrict__ perm_r, const int *__restrict__ off_c,
                                    const int *__restrict__ perm_c, int64_t N, int H, float *__restrict__ s_row,
                                    float *__restrict__ s_col) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N * H) return;
  const int64_t j = t / H;
  const int f = (int)(t - j * H);
  float a = 0.f, b = 0.f;
  for (int p = off_r[j]; p < off_r[j + 1]; ++p) a = __fadd_rn(a, dz[(int64_t)perm_r[p] * H + f]);
  for (int p = off_c[j]; p < off_c[j + 1]; ++p) b = __fadd_rn(b, dz[(int64_t)perm_c[p] * H + f]);
  s_row[t] = a;
  s_col[t] = b;
}

// Backward of h' = mlp([h ; agg(h)]) into h, then through the ReLU that made h:
// dh[j] = dX[j][:H] + sum_{e: col[e]=j} dX[row[e]][H:] / max(deg(row[e]),1);
// delta[j] = dh[j] where h[j] > 0.
__global__ void agg_backward_kernel(const float *__restrict__ dX, const int64_t *__restrict__ row,
                                    const int *__restrict__ off_r, const int *__restrict__ off_c,
                                    const int *__restrict__ perm_c, const float *__restrict__ h, int64_t N, int H,
                                    float *__restrict__ delta) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N * H) return;
  const int64_t j = t / H;
  const int f = (int)(t - j * H);
  float v = dX[j * 2 * H + f];
  for (int p = off_c[j]; p < off_c[j + 1]; ++p) {
    const int64_t i = row[perm_c[p]];
    const int deg = off_r[i + 1] - off_r[i];
    v = __fadd_rn(v, __fdiv_rn(dX[i * 2 * H + H + f], (float)(deg > 0 ? deg : 1)));
  }
  delta[t] = h[t] > 0.f ? v : 0.f;
}

inline size_t align256(size_t v) { return (v + 255) & ~size_t(255); }

struct Carve {
  char *p;
  template <class T>
  T *take(size_t n) {
    T *r = reinterpret_cast<T *>(p);
    p += align256(sizeof(T) * n);
    return r;
  }
};

hipError_t linear(const float *A1, int K1, const int64_t *i1, const float *A2, int K2, const int64_t *i2,
                  WView W, const float *b, float *out, int64_t M, int O, int act, hipStream_t s,
                  const float *mask = nullptr, const float *resid = nullptr) {
  if (M <= 0) return hipSuccess;
  dim3 grid((unsigned)((M + kT - 1) / kT), (unsigned)((O + kT - 1) / kT));
  const OpIn in{A1, A2, i1, i2, K1, K2, M};
  if (W.si == 1)
    hipLaunchKernelGGL(linear_kernel<false>, grid, dim3(256), 0, s, in, OpW<false>{W, O, K1 + K2, K1}, b, out,
                       act, mask, resid);
  else
    hipLaunchKernelGGL(linear_kernel<true>, grid, dim3(256), 0, s, in, OpW<true>{W, O, K1 + K2, K1}, b, out,
                       act, mask, resid);
  return hipGetLastError();
}

constexpr int64_t kMaxSplits = 128;
inline int64_t split_rows(int64_t M) {  // >= 256 rows per split, <= 128 splits, multiple of the LDS chunk
  int64_t R = (M + kMaxSplits - 1) / kMaxSplits;
  R = R < 256 ? 256 : R;
  return (R + kKC - 1) / kKC * kKC;
}

// gw[O][K1+K2] = D^T X, gb[O] = column sums of D (gb may be NULL).
hipError_t wgrad(const float *D, int O, const float *A1, int K1, const int64_t *i1, const float *A2, int K2,
                 const int64_t *i2, int64_t M, float *gw, float *gb, float *part, hipStream_t s) {
  const int K = K1 + K2;
  if (M <= 0) {
    hipError_t e = hipMemsetAsync(gw, 0, sizeof(float) * O * K, s);
    if (e == hipSuccess && gb) e = hipMemsetAsync(gb, 0, sizeof(float) * O, s);
    return e;
  }
  const int64_t R = split_rows(M);
  const int S = (int)((M + R - 1) / R);
  dim3 grid((unsigned)((O + kT - 1) / kT), (unsigned)((K + 1 + kT - 1) / kT), (unsigned)S);
  hipLaunchKernelGGL(wgrad_kernel, grid, dim3(256), 0, s, D, O, OpIn{A1, A2, i1, i2, K1, K2, M}, R, part);
  const int64_t n = (int64_t)O * (K + 1);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, part, S, O, K, gw,
                     gb);
  return hipGetLastError();
}

inline int64_t wgrad_part_floats(const GraphW &w, int64_t N, int64_t E) {
  const int64_t H = w.hidden;
  auto need = [](int64_t M, int64_t O, int64_t K) {
    const int64_t R = split_rows(M > 0 ? M : 1);
    return ((M + R - 1) / R) * O * (K + 1);
  };
  int64_t m = need(N, H, 2 * H);
  m = std::max(m, need(E, H, 2 * H));
  m = std::max(m, need(E, 1, H));
  m = std::max(m, need(N, H, w.in_dim));
  return m;
}

// CSR of B = N/nx periodic chains in build_chain_graph's edge order
// (src/graph_constructor.py:34-38: edge i = (i -> i+1), edge nx+i = (i+1 -> i)
// per chain), bucketed by row (by_col = 0) or col; two edges per node, ascending.
__global__ void chain_csr_kernel(int64_t N, int nx, int by_col, int *__restrict__ off, int *__restrict__ perm) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j > N) return;
  off[j] = (int)(2 * j);
  if (j == N) return;
  const int64_t b = j / nx;
  const int i = (int)(j - b * nx), im = (i + nx - 1) % nx;
  const int64_t base = 2 * b * nx;
  perm[2 * j] = (int)(base + (by_col ? im : i));
  perm[2 * j + 1] = (int)(base + nx + (by_col ? i : im));
}

// CSR of edges bucketed by key[e] (row or col), segments sorted by edge id.
hipError_t build_csr(const int64_t *key, int64_t E, int64_t N, int *deg, int *off, int *cur, int *perm,
                     hipStream_t s, int chain_nx = 0, bool by_col = false) {
  hipError_t err;
  if (chain_nx > 0) {
    hipLaunchKernelGGL(chain_csr_kernel, dim3((unsigned)((N + 1 + 255) / 256)), dim3(256), 0, s, N, chain_nx,
                       by_col ? 1 : 0, off, perm);
    return hipGetLastError();
  }
  if ((err = hipMemsetAsync(deg, 0, sizeof(int) * N, s)) != hipSuccess) return err;
  const unsigned eb = (unsigned)((E + 255) / 256), nb = (unsigned)((N + 255) / 256);
  if (E > 0) hipLaunchKernelGGL(count_deg_kernel, dim3(eb), dim3(256), 0, s, key, E, deg);
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, s, deg, N, off, cur);
  if (E > 0) hipLaunchKernelGGL(fill_kernel, dim3(eb), dim3(256), 0, s, key, E, cur, perm);
  hipLaunchKernelGGL(sort_segments_kernel, dim3(nb), dim3(256), 0, s, off, N, perm);
  return hipGetLastError();
}

// Forward over a CSR already built; h[l] for l = 0..L are separate buffers
// when `keep` (training tape), or ping-pong h[0]/h[1] otherwise.
hipError_t forward_core(const GraphW &w, const float *nf, int64_t N, const int64_t *ei, int64_t E,
                        const int *off, const int *perm, float *const *h, float *const *agg, bool keep, float *z,
                        float *flux, hipStream_t s) {
  const int H = w.hidden;
  const int64_t *row = ei, *col = ei + E;
  hipError_t err;
  // input MLP (src/flux_gnn.py:49)
  if ((err = linear(nf, w.in_dim, nullptr, nullptr, 0, nullptr, wv_rows(w.w_in, w.in_dim, w.in_dim), w.b_in, h[0],
                    N, H, kActRelu, s)))
    return err;
  int cur = 0;
  for (int l = 0; l < w.layers; ++l) {  // :53-60
    const int nxt = keep ? l + 1 : 1 - cur;
    float *a = keep ? agg[l] : agg[0];
    const unsigned ab = (unsigned)((N * H + 255) / 256);
    hipLaunchKernelGGL(aggregate_kernel, dim3(ab), dim3(256), 0, s, h[cur], col, off, perm, N, H, a);
    if ((err = linear(h[cur], H, nullptr, a, H, nullptr, wv_rows(w.w_l + l * w.lsw, H, 2 * H), w.b_l + l * w.lsb,
                      h[nxt], N, H, kActRelu, s)))
      return err;
    cur = nxt;
  }
  // edge readout (:62-66): z = ReLU(W_e [h[row] ; h[col]] + b_e); flux = w2 z + b2
  if ((err = linear(h[cur], H, row, h[cur], H, col, wv_rows(w.w_e, H, 2 * H), w.b_e, z, E, H, kActRelu, s))) return err;
  return linear(z, H, nullptr, nullptr, 0, nullptr, wv_rows(w.w_2, H, H), w.b_2, flux, E, 1, kActNone, s);
}

inline int64_t param_count(const GraphW &w) {
  const int64_t H = w.hidden;
  return H * w.in_dim + H + w.layers * (2 * H * H + H) + 2 * H * H + H + H + 1;
}

struct Tape {
  int *deg, *off, *cur, *perm;  // CSR by row (forward aggregation)
  float *h[kMaxChainLayers + 1];
  float *agg[kMaxChainLayers];
  float *z;                     // relu(z) of the edge readout [E][H]
};

Tape carve_tape(const GraphW &w, int64_t N, int64_t E, void *base) {
  Carve c{static_cast<char *>(base)};
  Tape t{};
  t.deg = c.take<int>(N);
  t.off = c.take<int>(N + 1);
  t.cur = c.take<int>(N);
  t.perm = c.take<int>(E);
  for (int l = 0; l <= w.layers; ++l) t.h[l] = c.take<float>(N * w.hidden);
  for (int l = 0; l < w.layers; ++l) t.agg[l] = c.take<float>(N * w.hidden);
  t.z = c.take<float>(E * w.hidden);
  return t;
}

}  // namespace

hipError_t gemm_linear(const float *A1, int K1, const int64_t *i1, const float *A2, int K2, const int64_t *i2,
                       WView W, const float *b, float *out, int64_t M, int O, int act, const float *resid,
                       hipStream_t s) {
  return linear(A1, K1, i1, A2, K2, i2, W, b, out, M, O, act, s, nullptr, resid);
}

hipError_t edge_buckets(const int64_t *key, int64_t E, int64_t N, int chain_nx, bool by_col, void *ws,
                        int **off, int **perm, hipStream_t s) {
  Carve c{static_cast<char *>(ws)};
  int *deg = c.take<int>(N), *o = c.take<int>(N + 1), *cur = c.take<int>(N), *p = c.take<int>(E);
  *off = o;
  *perm = p;
  return build_csr(key, E, N, deg, o, cur, p, s, chain_nx, by_col);
}

int64_t edge_buckets_bytes(int64_t N, int64_t E) {
  return (int64_t)(2 * align256(sizeof(int) * N) + align256(sizeof(int) * (N + 1)) + align256(sizeof(int) * E));
}

GraphW graph_view_state_dict(const float *p, int in_dim, int hidden, int layers) {
  GraphW g{};
  const int64_t H = hidden;
  int64_t o = 0;
  g.in_dim = in_dim;
  g.hidden = hidden;
  g.layers = layers;
  g.w_in = p + o; o += H * in_dim;
  g.b_in = p + o; o += H;
  g.w_l = p + o;
  g.b_l = p + o + H * 2 * H;
  g.lsw = g.lsb = H * 2 * H + H;
  o += layers * (H * 2 * H + H);
  g.w_e = p + o; o += H * 2 * H;
  g.b_e = p + o; o += H;
  g.w_2 = p + o; o += H;
  g.b_2 = p + o;
  return g;
}

int64_t graph_workspace_bytes(const GraphW &w, int64_t N, int64_t E) {
  const int64_t H = w.hidden;
  size_t b = 0;
  b += align256(sizeof(int) * (size_t)N);              // deg
  b += align256(sizeof(int) * (size_t)(N + 1));        // off
  b += align256(sizeof(int) * (size_t)N);              // cursor
  b += align256(sizeof(int) * (size_t)E);              // perm
  b += 3 * align256(sizeof(float) * (size_t)(N * H));  // h, h', agg
  b += align256(sizeof(float) * (size_t)(E * H));      // z
  return (int64_t)b;
}

hipError_t launch_graph_flux(const GraphW &w, const float *nf, int64_t N, const int64_t *ei, int64_t E,
                             float *flux, void *ws, hipStream_t s) {
  if (E <= 0) return hipSuccess;
  const int H = w.hidden;
  Carve c{static_cast<char *>(ws)};
  int *deg = c.take<int>(N), *off = c.take<int>(N + 1), *cur = c.take<int>(N), *perm = c.take<int>(E);
  float *h[2] = {c.take<float>(N * H), c.take<float>(N * H)};
  float *agg[1] = {c.take<float>(N * H)};
  float *z = c.take<float>(E * H);
  hipError_t err;
  if ((err = build_csr(ei, E, N, deg, off, cur, perm, s))) return err;
  return forward_core(w, nf, N, ei, E, off, perm, h, agg, false, z, flux, s);
}

// ------------------------------------------------------------------ training
int64_t graph_tape_bytes(const GraphW &w, int64_t N, int64_t E) {
  const int64_t H = w.hidden;
  size_t b = align256(sizeof(int) * N) * 2 + align256(sizeof(int) * (N + 1)) + align256(sizeof(int) * E);
  b += (size_t)(2 * w.layers + 1) * align256(sizeof(float) * N * H);
  b += align256(sizeof(float) * E * H);
  return std::max((int64_t)b, chain_tape_bytes(w, N));  // either path (tagged chains: train_chain.hip)
}

int64_t graph_backward_ws_bytes(const GraphW &w, int64_t N, int64_t E) {
  const int64_t H = w.hidden;
  size_t b = align256(sizeof(float) * E * H);                    // dz
  b += 3 * align256(sizeof(float) * N * H);                      // S_row, S_col, deltas
  b += align256(sizeof(float) * N * 2 * H);                      // dX
  b += align256(sizeof(float) * wgrad_part_floats(w, N, E));     // split-K partials
  b += align256(sizeof(int) * N) * 2 + align256(sizeof(int) * (N + 1)) + align256(sizeof(int) * E);  // CSR by col
  return std::max((int64_t)b, chain_backward_ws_bytes(w, N));
}

hipError_t launch_graph_forward_train(const GraphW &w, const float *nf, int64_t N, const int64_t *ei, int64_t E,
                                      int chain_nx, float *flux, void *tape, hipStream_t s) {
  if (E <= 0) return hipSuccess;  // no flux to compute; the backward returns zeros
  if (chain_train_ok(w, chain_nx, N)) return launch_chain_forward_train(w, nf, N, chain_nx, flux, tape, s);
  Tape t = carve_tape(w, N, E, tape);
  hipError_t err;
  if ((err = build_csr(ei, E, N, t.deg, t.off, t.cur, t.perm, s, chain_nx, false))) return err;
  return forward_core(w, nf, N, ei, E, t.off, t.perm, t.h, t.agg, true, t.z, flux, s);
}

// Reverse of forward_core (autograd of src/flux_gnn.py:40-67).  grad_params
// is written in state-dict order (the layout of graph_view_state_dict).
hipError_t launch_graph_backward(const GraphW &w, const float *nf, int64_t N, const int64_t *ei, int64_t E,
                                 int chain_nx, const void *tape, const float *grad_flux, float *grad_params, float *grad_nf,
                                 void *ws, hipStream_t s) {
  const int H = w.hidden, L = w.layers;
  const Tape t = carve_tape(w, N, E, const_cast<void *>(tape));
  const GraphW g = graph_view_state_dict(grad_params, w.in_dim, H, L);
  float *gw_in = const_cast<float *>(g.w_in), *gb_in = const_cast<float *>(g.b_in);
  float *gw_e = const_cast<float *>(g.w_e), *gb_e = const_cast<float *>(g.b_e);
  float *gw_2 = const_cast<float *>(g.w_2), *gb_2 = const_cast<float *>(g.b_2);
  const int64_t *row = ei, *col = ei + E;

  hipError_t err;
  if (E <= 0) {  // no edges, no flux: every gradient is zero
    if ((err = hipMemsetAsync(grad_params, 0, sizeof(float) * param_count(w), s))) return err;
    if (grad_nf && (err = hipMemsetAsync(grad_nf, 0, sizeof(float) * N * w.in_dim, s))) return err;
    return hipSuccess;
  }
  if (chain_train_ok(w, chain_nx, N))
    return launch_chain_backward(w, nf, N, chain_nx, tape, grad_flux, grad_params, grad_nf, ws, s);
  Carve c{static_cast<char *>(ws)};
  float *dz = c.take<float>(E * H);
  float *buf[3] = {c.take<float>(N * H), c.take<float>(N * H), c.take<float>(N * H)};
  float *dX = c.take<float>(N * 2 * H);
  float *part = c.take<float>(wgrad_part_floats(w, N, E));
  int *deg_c = c.take<int>(N), *off_c = c.take<int>(N + 1), *cur_c = c.take<int>(N), *perm_c = c.take<int>(E);
  const unsigned nb = (unsigned)((N * H + 255) / 256);

  if ((err = build_csr(col, E, N, deg_c, off_c, cur_c, perm_c, s, chain_nx, true))) return err;
  // readout: flux = w2 . relu(z) + b2, z = W_e [h[row] ; h[col]] + b_e        (:62-66)
  if ((err = wgrad(grad_flux, 1, t.z, H, nullptr, nullptr, 0, nullptr, E, gw_2, gb_2, part, s))) return err;
  hipLaunchKernelGGL(readout_delta_kernel, dim3((unsigned)((E * H + 255) / 256)), dim3(256), 0, s, grad_flux, t.z,
                     w.w_2, E, H, dz);
  if ((err = wgrad(dz, H, t.h[L], H, row, t.h[L], H, col, E, gw_e, gb_e, part, s))) return err;
  hipLaunchKernelGGL(edge_scatter_kernel, dim3(nb), dim3(256), 0, s, dz, t.off, t.perm, off_c, perm_c, N, H, buf[0],
                     buf[1]);
  // dh_L = W_a^T S_row + W_b^T S_col, masked by relu'(h_L): the delta of layer L-1 (or of the input MLP)
  const WView wet{w.w_e, w.w_e + H, 1, 2 * H};
  if ((err = linear(buf[0], H, nullptr, buf[1], H, nullptr, wet, nullptr, buf[2], N, H, kActNone, s, t.h[L])))
    return err;
  int cur = 2;
  // update layers, last to first                                                 (:53-60)
  for (int l = L - 1; l >= 0; --l) {
    float *gw_l = const_cast<float *>(g.w_l + l * g.lsw), *gb_l = const_cast<float *>(g.b_l + l * g.lsb);
    if ((err = wgrad(buf[cur], H, t.h[l], H, nullptr, t.agg[l], H, nullptr, N, gw_l, gb_l, part, s))) return err;
    // [d h_l ; d agg_l] = W_l^T delta                                             ([N][2H])
    if ((err = linear(buf[cur], H, nullptr, nullptr, 0, nullptr, wv_t(w.w_l + l * w.lsw, 2 * H), nullptr, dX, N,
                      2 * H, kActNone, s)))
      return err;
    const int nxt = cur == 0 ? 1 : 0;
    hipLaunchKernelGGL(agg_backward_kernel, dim3(nb), dim3(256), 0, s, dX, row, t.off, off_c, perm_c, t.h[l], N, H,
                       buf[nxt]);
    cur = nxt;
  }
  const float *delta = buf[cur];
  // input MLP                                                                   (:49)
  if ((err = wgrad(delta, H, nf, w.in_dim, nullptr, nullptr, 0, nullptr, N, gw_in, gb_in, part, s))) return err;
  if (grad_nf &&
      (err = linear(delta, H, nullptr, nullptr, 0, nullptr, wv_t(w.w_in, w.in_dim), nullptr, grad_nf, N, w.in_dim,
                    kActNone, s)))
    return err;
  return hipGetLastError();
}

}  // namespace hf
