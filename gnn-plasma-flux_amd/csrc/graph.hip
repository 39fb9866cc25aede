// FluxGNN.forward on an arbitrary graph (src/flux_gnn.py:40-67), float32.
//
// This is the compatibility path for edge_index tensors that are not the
// periodic chain (examples/smoke_test.py:53 feeds a random one).  The chain
// — the hot path — never comes here; it runs in chain_gnn.hip.
//
//  * Mean aggregation is deterministic and in reference order: edges are
//    bucketed by destination row into a CSR whose segments are sorted by edge
//    id, so node i sums h[col[e]] in increasing e exactly like the serial
//    index_add_ (src/flux_gnn.py:57), then divides by max(deg,1) (:58-59).
//  * Linear layers are one LDS-tiled kernel computing
//    act(b + W [A1[r1(m)] ; A2[r2(m)]]) with optional row gathers, so the
//    concatenations of :60 and :62-64 are never materialised.
#include "hf_device.h"
#include "hf_internal.h"

namespace hf {
namespace {

constexpr int kBM = 64, kBO = 64, kBK = 16;

// out[m][o] = act(bias[o] + sum_k W[o][k] * in(m,k)),
// in(m,k) = k < K1 ? A1[r1(m)][k] : A2[r2(m)][k-K1],  r(m) = idx ? idx[m] : m.
__global__ __launch_bounds__(256) void linear_kernel(const float *__restrict__ A1, int K1,
                                                     const int64_t *__restrict__ idx1,
                                                     const float *__restrict__ A2, int K2,
                                                     const int64_t *__restrict__ idx2,
                                                     const float *__restrict__ W,
                                                     const float *__restrict__ bias, float *out,
                                                     int64_t M, int O, int relu_out) {
  __shared__ float sA[kBK][kBM + 1];
  __shared__ float sW[kBK][kBO + 1];
  const int K = K1 + K2;
  const int64_t m0 = (int64_t)blockIdx.x * kBM;
  const int o0 = blockIdx.y * kBO;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;  // 16 x 16 threads, 4x4 outputs each
  float acc[4][4] = {};
  for (int k0 = 0; k0 < K; k0 += kBK) {
    for (int e = threadIdx.x; e < kBK * kBM; e += 256) {
      const int kk = e % kBK, mm = e / kBK;
      const int64_t m = m0 + mm;
      const int k = k0 + kk;
      float v = 0.f;
      if (m < M && k < K) {
        if (k < K1) v = A1[(idx1 ? idx1[m] : m) * K1 + k];
        else v = A2[(idx2 ? idx2[m] : m) * K2 + (k - K1)];
      }
      sA[kk][mm] = v;
    }
    for (int e = threadIdx.x; e < kBK * kBO; e += 256) {
      const int kk = e % kBK, oo = e / kBK;
      const int o = o0 + oo, k = k0 + kk;
      sW[kk][oo] = (o < O && k < K) ? W[(int64_t)o * K + k] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < kBK; ++kk) {
      float a[4], w[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = sA[kk][ty + 16 * i];
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] = sW[kk][tx + 16 * i];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[i][q] = fmaf(a[i], w[q], acc[i][q]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t m = m0 + ty + 16 * i;
    if (m >= M) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int o = o0 + tx + 16 * q;
      if (o >= O) continue;
      float v = __fadd_rn(acc[i][q], bias[o]);
      out[m * O + o] = relu_out ? relu(v) : v;
    }
  }
}

__global__ void count_deg_kernel(const int64_t *__restrict__ row, int64_t E, int *deg) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < E) atomicAdd(&deg[row[e]], 1);
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

__global__ void fill_kernel(const int64_t *__restrict__ row, int64_t E, int *cur,
                            int *__restrict__ perm) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < E) perm[atomicAdd(&cur[row[e]], 1)] = (int)e;
}

// Restore edge order inside each destination segment (insertion sort by id).
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

inline size_t align256(size_t v) { return (v + 255) & ~size_t(255); }

hipError_t linear(const float *A1, int K1, const int64_t *i1, const float *A2, int K2,
                  const int64_t *i2, const float *W, const float *b, float *out, int64_t M, int O,
                  bool act, hipStream_t s) {
  if (M <= 0) return hipSuccess;
  dim3 grid((unsigned)((M + kBM - 1) / kBM), (unsigned)((O + kBO - 1) / kBO));
  hipLaunchKernelGGL(linear_kernel, grid, dim3(256), 0, s, A1, K1, i1, A2, K2, i2, W, b, out, M, O,
                     act ? 1 : 0);
  return hipGetLastError();
}

}  // namespace

int64_t graph_workspace_bytes(const GraphW &w, int64_t N, int64_t E) {
  const int64_t H = w.hidden;
  size_t b = 0;
  b += align256(sizeof(int) * (size_t)N);            // deg
  b += align256(sizeof(int) * (size_t)(N + 1));      // off
  b += align256(sizeof(int) * (size_t)N);            // cursor
  b += align256(sizeof(int) * (size_t)E);            // perm
  b += 3 * align256(sizeof(float) * (size_t)(N * H));  // h, h', agg
  b += align256(sizeof(float) * (size_t)(E * H));    // z
  return (int64_t)b;
}

hipError_t launch_graph_flux(const GraphW &w, const float *nf, int64_t N, const int64_t *ei,
                             int64_t E, float *flux, void *ws, hipStream_t s) {
  if (E <= 0) return hipSuccess;
  const int H = w.hidden;
  char *p = static_cast<char *>(ws);
  auto take = [&](size_t bytes) {
    char *r = p;
    p += align256(bytes);
    return r;
  };
  int *deg = reinterpret_cast<int *>(take(sizeof(int) * N));
  int *off = reinterpret_cast<int *>(take(sizeof(int) * (N + 1)));
  int *cur = reinterpret_cast<int *>(take(sizeof(int) * N));
  int *perm = reinterpret_cast<int *>(take(sizeof(int) * E));
  float *h0 = reinterpret_cast<float *>(take(sizeof(float) * N * H));
  float *h1 = reinterpret_cast<float *>(take(sizeof(float) * N * H));
  float *agg = reinterpret_cast<float *>(take(sizeof(float) * N * H));
  float *z = reinterpret_cast<float *>(take(sizeof(float) * E * H));
  const int64_t *row = ei, *col = ei + E;

  hipError_t err;
  if ((err = hipMemsetAsync(deg, 0, sizeof(int) * N, s)) != hipSuccess) return err;
  const unsigned eb = (unsigned)((E + 255) / 256), nb = (unsigned)((N + 255) / 256);
  hipLaunchKernelGGL(count_deg_kernel, dim3(eb), dim3(256), 0, s, row, E, deg);
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, s, deg, N, off, cur);
  hipLaunchKernelGGL(fill_kernel, dim3(eb), dim3(256), 0, s, row, E, cur, perm);
  hipLaunchKernelGGL(sort_segments_kernel, dim3(nb), dim3(256), 0, s, off, N, perm);
  if ((err = hipGetLastError()) != hipSuccess) return err;

  // input MLP (src/flux_gnn.py:49)
  if ((err = linear(nf, w.in_dim, nullptr, nullptr, 0, nullptr, w.w_in, w.b_in, h0, N, H, true, s)))
    return err;
  for (int l = 0; l < w.layers; ++l) {  // :53-60
    const unsigned ab = (unsigned)((N * H + 255) / 256);
    hipLaunchKernelGGL(aggregate_kernel, dim3(ab), dim3(256), 0, s, h0, col, off, perm, N, H, agg);
    if ((err = linear(h0, H, nullptr, agg, H, nullptr, w.w_l + (size_t)l * H * 2 * H,
                      w.b_l + (size_t)l * H, h1, N, H, true, s)))
      return err;
    float *t = h0;
    h0 = h1;
    h1 = t;
  }
  // edge readout (:62-66): z = ReLU(W_e [h[row] ; h[col]] + b_e); flux = w2 z + b2
  if ((err = linear(h0, H, row, h0, H, col, w.w_e, w.b_e, z, E, H, true, s))) return err;
  return linear(z, H, nullptr, nullptr, 0, nullptr, w.w_2, w.b_2, flux, E, 1, false, s);
}

}  // namespace hf
