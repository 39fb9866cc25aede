// The f32 MFMA GEMM of the chain training path (train_chain.hip) and of the
// PureGNN chain layers (baselines.hip): operand views, epilogues, tgemm_kernel.
//
// C[i][j] = sum_r A(i, r) B(r, j) on 128 x 128 output tiles, 4 waves of
// 64 x 64 (2 x 2 v_mfma_f32_32x32x2_f32 tiles), the reduction staged through
// double-buffered LDS in chunks of 32.  Operands are views (a plain row-major
// matrix, a split weight, the chain stencil [X ; agg X]); the epilogue is a
// functor per output element, or (kBlock) a workgroup-wide pass over the tile
// through LDS.
#pragma once
#include <cstdint>
#include <type_traits>

#include <hip/hip_runtime.h>

namespace hf {
namespace tg {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16 __attribute__((ext_vector_type(16)));

#ifndef HF_TG_KC
#define HF_TG_KC 32
#endif
#ifndef HF_TG_WG
#define HF_TG_WG 2
#endif
// timing diagnostics (CXXFLAGS_EXTRA=-DHF_DIAG_TG_*; results wrong): no stage
// loads (NOGL), LDS stores (NOLS), stage barriers (NOBAR), partial-tile stores (NOEPI)
#ifdef HF_DIAG_TG_NOGL
constexpr bool kDiagNoGl = true;
#else
constexpr bool kDiagNoGl = false;
#endif
#ifdef HF_DIAG_TG_NOLS
constexpr bool kDiagNoLs = true;
#else
constexpr bool kDiagNoLs = false;
#endif
#ifdef HF_DIAG_TG_NOBAR
constexpr bool kDiagNoBar = true;
#else
constexpr bool kDiagNoBar = false;
#endif
#ifdef HF_DIAG_TG_NOEPI
constexpr bool kDiagNoEpi = true;
#else
constexpr bool kDiagNoEpi = false;
#endif
#ifndef HF_TG_FRAG_AHEAD
#define HF_TG_FRAG_AHEAD 1
#endif
#ifndef HF_TG_PAIR_LOOP
#define HF_TG_PAIR_LOOP 1
#endif
constexpr bool kFragAhead = HF_TG_FRAG_AHEAD, kPairLoop = HF_TG_PAIR_LOOP;
constexpr int kBM = 128, kBN = 128, kKC = HF_TG_KC;  // reduction chunk per stage (32; 16: a build knob)
constexpr int kNQ = kBM * kKC / 4 / 256;             // float4 per thread per operand per stage
constexpr int kIMSh = kKC == 32 ? 3 : 2;             // log2(float4 per [i][r] row)
static_assert(kKC == 32 || kKC == 16, "stage depth");
constexpr int kStrIM = kKC + 4;   // [i][r] tile rows: 36 floats (conflict-free b128 reads of 16 lanes)
constexpr int kStrRM = kBM + 8;   // [r][i] tile rows: 136 floats (the two lane halves 4 rows apart land on disjoint banks)
constexpr int kTileF = (kBM * kStrIM > kKC * kStrRM) ? kBM * kStrIM : kKC * kStrRM;

__device__ __forceinline__ int64_t chain_prev(int64_t m, int nx) {
  const int i = (int)((unsigned)m % (unsigned)nx);
  return m + (i == 0 ? nx - 1 : -1);
}
__device__ __forceinline__ int64_t chain_next(int64_t m, int nx) {
  const int i = (int)((unsigned)m % (unsigned)nx);
  return m + (i == nx - 1 ? 1 - nx : 1);
}

// Row-major matrix views (element (row, col) of a logical [rows][cols] matrix).
// Plain: rows in blocks of 2^hshift; row r at p + (r & (2^hshift - 1)) * ld +
// (r >> hshift) * hoff (a split weight like [W_a ; W_b] read out of
// nn.Linear's [H][2H]; hshift = 62 for an ordinary matrix).  No 64-bit
// division on the load path.
struct VPlain {
  const float *p;
  int64_t ld, rows;
  int hshift;
  int64_t hoff;
  int cols;
  struct Row {
    int off;  // float offset of the row from p (< 2^31, host-checked)
  };
  // Rows past the end are clamped to the last one, columns past the end to the
  // last float4: the GEMM either discards what such loads feed (output rows /
  // columns past I / J) or zeroes it (reduction rows past the split's end).
  __device__ Row row(int64_t r) const {
    r = r < rows ? r : rows - 1;
    const int64_t lo = r & ((int64_t(1) << hshift) - 1), hi = r >> hshift;
    return Row{(int)(lo * ld + hi * hoff)};
  }
  __device__ f4 load4(const Row &w, int c) const {
    c = c < cols ? c : cols - 4;
    return *reinterpret_cast<const f4 *>(p + (unsigned)(w.off + c));
  }
  // two-phase form (tgemm_kernel): load2 issues the loads, combine forms the value
  static constexpr bool kTwo = false;
  __device__ void load2(const Row &w, int c, f4 &a, f4 &) const { a = load4(w, c); }
  __device__ f4 combine(int, const f4 &a, const f4 &) const { return a; }
  bool fits32() const { return rows * ld + cols + (rows >> hshift) * hoff < (int64_t(1) << 31); }
  // exact GEMMs (tgemm_kernel EX): the row kKC further on, unsplit views only
  __device__ void adv(Row &w) const { w.off += kKC * (int)ld; }
  __device__ void load2x(const Row &w, int c, f4 &a, f4 &) const {
    a = *reinterpret_cast<const f4 *>(p + (unsigned)(w.off + c));
  }
  bool exact_ok(int64_t R) const { return hshift >= 62 && R <= rows; }
};
constexpr int kNoSplit = 62;
// [X ; agg X] of X [rows][C] on chains of nx rows: cols [0, C) are X, [C, 2C)
// are (X[prev] + X[next]) * 0.5 (src/flux_gnn.py:53-59 on the chain).  The
// row handle holds the three row offsets (one 32-bit remainder per row, rows
// < 2^31, offsets < 2^31), computed once per row rather than per load.
struct VStencil {
  const float *X;
  int64_t rows;
  int C, nx;
  struct Row {
    int self, nxt, prv;  // float offsets of the rows (nxt, prv less C)
    int i;               // the row's cell on its chain
  };
  __device__ Row row(int64_t r) const {
    r = r < rows ? r : rows - 1;
    const int i = (int)((unsigned)r % (unsigned)nx);
    const int64_t nr = r + (i == nx - 1 ? 1 - nx : 1), pr = r + (i == 0 ? nx - 1 : -1);
    return Row{(int)(r * C), (int)(nr * C - C), (int)(pr * C - C), i};
  }
  // exact GEMMs: the row kKC further on, its cell stepped instead of divided out
  __device__ void adv(Row &w) const {
    const int d = kKC % nx;
    w.self += kKC * C;
    w.i += d;
    w.i -= w.i >= nx ? nx : 0;
    w.nxt = w.self + (w.i == nx - 1 ? -nx * C : 0);
    w.prv = w.self + (w.i == 0 ? (nx - 2) * C : -2 * C);
  }
  __device__ void load2x(const Row &w, int c, f4 &a, f4 &b) const {
    const bool self = c < C;
    a = *reinterpret_cast<const f4 *>(X + (unsigned)((self ? w.self : w.nxt) + c));
    b = *reinterpret_cast<const f4 *>(X + (unsigned)((self ? w.self : w.prv) + c));
  }
  bool exact_ok(int64_t R) const { return R <= rows; }
  // Two-phase: load2 issues two loads (the two neighbour rows, or the row
  // itself twice for c < C: branch-free, the second is an L1 hit), combine forms
  // (a + b) * 0.5 later, when the stage is written to LDS.  The one-call form
  // made the compiler wait for both loads right where they were issued, at the
  // start of the stage, before its MFMAs; a branch on c < C (uniform only when
  // C is a multiple of the stage depth) spilled the pair to scratch.
  static constexpr bool kTwo = true;
  __device__ void load2(const Row &w, int c, f4 &a, f4 &b) const {
    c = c < 2 * C ? c : 2 * C - 4;
    const bool self = c < C;
    a = *reinterpret_cast<const f4 *>(X + (unsigned)((self ? w.self : w.nxt) + c));
    b = *reinterpret_cast<const f4 *>(X + (unsigned)((self ? w.self : w.prv) + c));
  }
  __device__ f4 combine(int c, const f4 &a, const f4 &b) const {
    c = c < 2 * C ? c : 2 * C - 4;
    return c < C ? a : (a + b) * 0.5f;
  }
  bool fits32() const { return rows * C + C < (int64_t(1) << 31); }
};

// Epilogues: out[i][j] = act(v + bias[j]) (bias on j < nbias), or v masked by mask[i][j] > 0,
// or the split's partial tile.
template <bool RELU>
struct EpiAct {
  float *out;
  int64_t ld;
  const float *bias;
  int nbias;
  __device__ float bias_of(int64_t j) const { return (bias && j < nbias) ? bias[j] : 0.f; }
  static constexpr bool kPre = false, kBlock = false;
  __device__ float pre(int64_t, int64_t) const { return 0.f; }
  __device__ void operator()(int64_t i, int64_t j, float v, float bj, float) const {
    v = __fadd_rn(v, bj);  // + 0 where there is no bias
    if (RELU) v = v > 0.f ? v : (v == v ? 0.f : v);  // NaN stays NaN, as torch.relu
    out[i * ld + j] = v;
  }
};
struct EpiMask {
  float *out;
  int64_t ld;
  const float *mask;
  int64_t ldm;
  __device__ float bias_of(int64_t) const { return 0.f; }
  // the mask of the whole tile is loaded before any store: out may alias
  // nothing, but the compiler cannot know, and would otherwise wait out one
  // load latency per element
  static constexpr bool kPre = true, kBlock = false;
  __device__ float pre(int64_t i, int64_t j) const { return mask[i * ldm + j]; }
  __device__ void operator()(int64_t i, int64_t j, float v, float, float m) const { out[i * ld + j] = m > 0.f ? v : 0.f; }
};
struct EpiPart {
  float *part;
  int64_t I, J;
  int64_t z = 0;  // the split (set by tgemm_kernel)
  __device__ float bias_of(int64_t) const { return 0.f; }
  static constexpr bool kPre = false, kBlock = false;
  __device__ float pre(int64_t, int64_t) const { return 0.f; }
  __device__ void operator()(int64_t i, int64_t j, float v, float, float) const {
    if (!kDiagNoEpi || v == 1.2345e-30f) part[(z * I + i) * J + j] = v;
  }
};
// out[i][j] = tanh(v + bias[j]) (PureGNN's output_mlp.0, train_pure_gnn.py:74-75)
struct EpiTanh {
  float *out;
  int64_t ld;
  const float *bias;
  __device__ float bias_of(int64_t j) const { return bias[j]; }
  static constexpr bool kPre = false, kBlock = false;
  __device__ float pre(int64_t, int64_t) const { return 0.f; }
  __device__ void operator()(int64_t i, int64_t j, float v, float bj, float) const { out[i * ld + j] = tanhf(__fadd_rn(v, bj)); }
};

// [W_a ; W_b] of a PureGNN message layer (nn.Linear [H][2H]) as the B operand
// of its P/Q GEMM, in 64-feature blocks so that one 128-column tile holds P
// and Q of the same 64 features: output column j is feature
// f = 64 (j >> 7) + (j & 63) of P (bit 6 of j clear) or of Q (set), i.e. row f
// of W, columns [0, H) or [H, 2H).  H % 64 == 0 (host-checked).
struct VPQ {
  const float *W;
  int H;
  struct Row {
    int off;
  };
  __device__ Row row(int64_t j) const {
    j = j < 2 * H ? j : 2 * H - 1;
    const int f = (int)((j >> 7) * 64 + (j & 63)), q = (int)((j >> 6) & 1);
    return Row{f * 2 * H + q * H};
  }
  __device__ f4 load4(const Row &w, int c) const {
    c = c < H ? c : H - 4;
    return *reinterpret_cast<const f4 *>(W + (unsigned)(w.off + c));
  }
  static constexpr bool kTwo = false;
  __device__ void load2(const Row &w, int c, f4 &a, f4 &) const { a = load4(w, c); }
  __device__ f4 combine(int, const f4 &a, const f4 &) const { return a; }
  bool fits32() const { return 2LL * H * H < (int64_t(1) << 31); }
};

// PureGNN message layer on tile-aligned chains (train_pure_gnn.py:60-67 on
// build_chain_graph): h'[i] = h[i] + tanh(P[i-1] + Q[i] + b) + tanh(P[i+1] + Q[i] + b)
// with the messages summed in edge order (from i-1, then from i+1, as
// index_add_), P = W_a h, Q = W_b h the tile's accumulators (VPQ columns).
// Block epilogue: the waves park P and Q of the tile's 128 cells x 64
// features in LDS, then every thread finishes 32 (cell, feature) outputs, so
// neither P nor Q reaches HBM.  Needs nx | 128 (whole chains per row tile).
struct EpiMsg {
  const float *h;  // layer input [N][H]
  float *out;      // layer output [N][H]
  const float *b;  // message bias [H]
  int H, nx;
  static constexpr bool kPre = false, kBlock = true;
  __device__ float bias_of(int64_t) const { return 0.f; }
  __device__ float pre(int64_t, int64_t) const { return 0.f; }
  __device__ void operator()(int64_t, int64_t, float, float, float) const {}
  static constexpr int kS = 65;  // LDS row stride of the parked tiles
  __device__ void block(const f16 (&acc)[2][2], float *sP, float *sQ, int64_t i0, int64_t j0, int64_t I, int wi, int wj,
                        int lane, int t) const {
    float *dst = wj == 0 ? sP : sQ;
    const int hl = lane >> 5;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int bb = 0; bb < 2; ++bb)
#pragma unroll
        for (int v = 0; v < 16; ++v)
          dst[(64 * wi + 32 * a + 8 * (v >> 2) + 4 * hl + (v & 3)) * kS + 32 * bb + (lane & 31)] = acc[a][bb][v];
    __syncthreads();
    const int f = t & 63;
    const int64_t fg = (j0 >> 7) * 64 + f;
    const float bf = b[fg];
#pragma unroll 4
    for (int k = 0; k < 32; ++k) {
      const int r = (t >> 6) + 4 * k;
      const int64_t i = i0 + r;
      if (i >= I) break;
      const int ci = (int)((unsigned)i % (unsigned)nx);
      const int rp = r + (ci == 0 ? nx - 1 : -1), rn = r + (ci == nx - 1 ? 1 - nx : 1);
      const float q = sQ[r * kS + f];
      float m = tanhf(__fadd_rn(__fadd_rn(sP[rp * kS + f], q), bf));
      m = __fadd_rn(m, tanhf(__fadd_rn(__fadd_rn(sP[rn * kS + f], q), bf)));
      out[i * H + fg] = __fadd_rn(h[i * H + fg], m);
    }
  }
};

// C[i][j] = sum_{r in split} A(i, r) B(r, j) over I x J, R.  A(i, r) = GA(r, i)
// when ARM (the operand's global rows run along the reduction), else GA(i, r);
// B(r, j) = GB(r, j) when BRM, else GB(j, r).  Both LDS tiles copy the global
// rows as they are; the MFMA reads adapt: an [i][r] tile gives each lane four
// consecutive r in one ds_read_b128 (MFMA step s of lane half h uses
// r = 8g + 4h + s), an [r][i] tile one ds_read_b32 per MFMA at the same r.
// COLSUM (ARM A only): the split's column sums of GA over its rows (the bias
// gradient), written to bias_part[split][i] by the blocks of column tile 0.
// EX (both operands RM; host-checked: whole tiles, R % kKC == 0, R within both
// views, unsplit views): no clamps or zeroed rows, and each thread's row
// handles are stepped by kKC per stage instead of recomputed (the stencil's
// cell index without a division).
#ifndef HF_TG_XCD
#define HF_TG_XCD 1
#endif
// HF_TG_XCD (measured +0.8 % on the training step, profiles/r05_train_tgemm_xcd_prio_ab.txt):
// pairs of consecutive tiles (x fastest) on one XCD.  Blocks b and
// b + 8 share an XCD (MI355X_MICROARCH.md, workgroup dispatch); consecutive
// tiles of a weight-gradient split read the same rows (the two column tiles
// of [h ; agg h], or the P and Q halves against h[L]).
__device__ __forceinline__ void tg_block(unsigned &bx, unsigned &by, unsigned &bz) {
  bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (HF_TG_XCD) {
    const unsigned gx = gridDim.x, gy = gridDim.y, T = gx * gy * gridDim.z;
    unsigned L = bx + gx * (by + gy * bz);
    if (L < T - T % 16) L = 2 * (8 * (L >> 4) + (L & 7)) + ((L >> 3) & 1);
    bx = L % gx;
    by = (L / gx) % gy;
    bz = L / (gx * gy);
  }
}

// HF_TG_STAGGER > 0 (a build knob): a workgroup whose waves hold an odd wave
// slot on their SIMDs (the second workgroup of a CU, HW_REG_HW_ID.WAVE_ID)
// starts s_sleep(HF_TG_STAGGER) x 64 cycles late, so that the two workgroups
// sharing each SIMD reach their LDS stores and barriers at different times
// (MI355X_MICROARCH.md, "two waves that run the same program")
#ifndef HF_TG_STAGGER
#define HF_TG_STAGGER 0
#endif
__device__ __forceinline__ void tg_stagger() {
  if constexpr (HF_TG_STAGGER > 0) {
    const unsigned slot = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 4);  // HW_ID[3:0]
    if (slot & 1) __builtin_amdgcn_s_sleep(HF_TG_STAGGER);
  }
}

// One output tile (bx, by) of split bz: the body of tgemm_kernel and of
// tgemm_batch_kernel.
template <class LA, bool ARM, class LB, bool BRM, class Epi, bool COLSUM, bool EX = false>
__device__ __forceinline__ void tgemm_tile(LA ga, LB gb, Epi epi, int64_t I, int64_t J, int64_t R, int64_t rsplit,
                                           float *bias_part, unsigned bx, unsigned by, unsigned bz) {
  static_assert(!EX || (ARM && BRM), "exact form: both operands run along the reduction");
  // (a block epilogue parks a 128 x 65 tile in each operand's two buffers)
  constexpr int kBufF = (Epi::kBlock && 2 * kTileF < kBM * 65) ? (kBM * 65 + 1) / 2 : kTileF;
  __shared__ float sA[2][kBufF];
  __shared__ float sB[2][kBufF];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, wi = wave >> 1, wj = wave & 1, h = lane >> 5;
  const int64_t i0 = (int64_t)bx * kBM, j0 = (int64_t)by * kBN;
  const int64_t rb = (int64_t)bz * rsplit;
  if constexpr (std::is_same<Epi, EpiPart>::value) epi.z = bz;
  const int64_t re = rb + rsplit < R ? rb + rsplit : R;
  f16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[a][b][v] = 0.f;
  // Two register sets of 4 float4 per operand: the loads of stage s+2 are
  // issued while stage s computes and land in LDS at the end of stage s+1, so
  // each load has two stages (~2 x 4096 MFMA cycles per wave) to arrive.
#ifndef HF_TG_DEPTH
#define HF_TG_DEPTH 1
#endif
  constexpr int kDepth = HF_TG_DEPTH;  // stages of loads in flight: 1 (double buffer) and 2 measured equal
  // (profiles/r03_train_gemm_depth_ab.txt); 1 holds ~30 fewer registers
  f4 ra[kDepth][kNQ], rbv[kDepth][kNQ], csum = f4{0.f, 0.f, 0.f, 0.f};
  // second loads of two-phase views (the stencil's neighbour rows)
  f4 ra2[LA::kTwo ? kDepth : 1][kNQ], rb2[LB::kTwo ? kDepth : 1][kNQ];
  // thread -> (global row, col) of its 4 float4 per operand per stage.  The
  // rows of an [i][r] operand are the same every stage: their handles are made once.
  typename LA::Row rowa[kNQ];
  typename LB::Row rowb[kNQ];
  if (!ARM) {
#pragma unroll
    for (int q = 0; q < kNQ; ++q) rowa[q] = ga.row(i0 + ((t + 256 * q) >> kIMSh));
  }
  if (!BRM) {
#pragma unroll
    for (int q = 0; q < kNQ; ++q) rowb[q] = gb.row(j0 + ((t + 256 * q) >> kIMSh));
  }
  if (EX) {  // the first stage's rows; gload steps them
#pragma unroll
    for (int q = 0; q < kNQ; ++q) {
      rowa[q] = ga.row(rb + ((t + 256 * q) >> 5));
      rowb[q] = gb.row(rb + ((t + 256 * q) >> 5));
    }
  }
  // Branch-free loads: addresses clamped by the views; only reduction rows
  // past the split's end (RM operands) are zeroed, by select.  [i][r]
  // operands need R % kKC == 0 (host-checked), so their r never runs past re.
  // operand column of load q of the stage at r0 (the view's c)
  auto col_a = [&](int q, int64_t r0) {
    const int idx = t + 256 * q;
    return ARM ? (int)(i0 + 4 * (idx & 31)) : (int)(r0 + 4 * (idx & ((1 << kIMSh) - 1)));
  };
  auto col_b = [&](int q, int64_t r0) {
    const int idx = t + 256 * q;
    return BRM ? (int)(j0 + 4 * (idx & 31)) : (int)(r0 + 4 * (idx & ((1 << kIMSh) - 1)));
  };
  // issues the stage's loads only; lstore forms the values (view combine, the
  // zeroed reduction rows past the split's end) when it writes them to LDS
  auto gload = [&](int set, int64_t r0) {
#pragma unroll
    for (int q = 0; q < kNQ; ++q) {
      const int idx = t + 256 * q;
      if constexpr (EX) {
        ga.load2x(rowa[q], col_a(q, r0), ra[set][q], ra2[LA::kTwo ? set : 0][q]);
        gb.load2x(rowb[q], col_b(q, r0), rbv[set][q], rb2[LB::kTwo ? set : 0][q]);
        ga.adv(rowa[q]);
        gb.adv(rowb[q]);
      } else {
        ga.load2(ARM ? ga.row(r0 + (idx >> 5)) : rowa[q], col_a(q, r0), ra[set][q], ra2[LA::kTwo ? set : 0][q]);
        gb.load2(BRM ? gb.row(r0 + (idx >> 5)) : rowb[q], col_b(q, r0), rbv[set][q], rb2[LB::kTwo ? set : 0][q]);
      }
    }
  };
  auto lstore = [&](int buf, int set, int64_t r0) {
#pragma unroll
    for (int q = 0; q < kNQ; ++q) {
      const int idx = t + 256 * q, im = (1 << kIMSh) - 1;
      f4 va = ga.combine(col_a(q, r0), ra[set][q], ra2[LA::kTwo ? set : 0][q]);
      f4 vb = gb.combine(col_b(q, r0), rbv[set][q], rb2[LB::kTwo ? set : 0][q]);
      const bool in = EX || r0 + (idx >> 5) < re;
      if (ARM) va = f4{in ? va[0] : 0.f, in ? va[1] : 0.f, in ? va[2] : 0.f, in ? va[3] : 0.f};
      if (BRM) vb = f4{in ? vb[0] : 0.f, in ? vb[1] : 0.f, in ? vb[2] : 0.f, in ? vb[3] : 0.f};
      float *pa = ARM ? &sA[buf][(idx >> 5) * kStrRM + 4 * (idx & 31)] : &sA[buf][(idx >> kIMSh) * kStrIM + 4 * (idx & im)];
      float *pb = BRM ? &sB[buf][(idx >> 5) * kStrRM + 4 * (idx & 31)] : &sB[buf][(idx >> kIMSh) * kStrIM + 4 * (idx & im)];
      *reinterpret_cast<f4 *>(pa) = va;
      *reinterpret_cast<f4 *>(pb) = vb;
      if (COLSUM) csum += va;
    }
  };
  if (rb < re) {
    gload(0, rb);
    lstore(0, 0, rb);
    if (kDepth == 2 && rb + kKC < re) gload(kDepth - 1, rb + kKC);
  }
  __syncthreads();
  // one stage; register sets and LDS buffers indexed by the compile-time parity
  auto stage = [&](auto parity, int64_t r0) {
    constexpr int cur = decltype(parity)::value;
    // LDS[cur] holds stage r0; depth 2: register set cur^1 holds (in flight) stage r0 + kKC
    if (kDiagNoGl) {
    } else if (kDepth == 2) {
      if (r0 + 2 * kKC < re) gload(cur % kDepth, r0 + 2 * kKC);
    } else if (r0 + kKC < re) {
      gload(0, r0 + kKC);
    }
    const float *A = sA[cur], *B = sB[cur];
    // fragments of group g (8 reduction rows): av[x][s] / bv[x][s] for MFMA step s
    auto frag = [&](int g, float (&av)[2][4], float (&bv)[2][4]) {
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const int il = 64 * wi + 32 * x + (lane & 31), jl = 64 * wj + 32 * x + (lane & 31);
        if (ARM) {
#pragma unroll
          for (int s = 0; s < 4; ++s) av[x][s] = A[(8 * g + 4 * h + s) * kStrRM + il];
        } else {
          const f4 v = *reinterpret_cast<const f4 *>(&A[il * kStrIM + 8 * g + 4 * h]);
#pragma unroll
          for (int s = 0; s < 4; ++s) av[x][s] = v[s];
        }
        if (BRM) {
#pragma unroll
          for (int s = 0; s < 4; ++s) bv[x][s] = B[(8 * g + 4 * h + s) * kStrRM + jl];
        } else {
          const f4 v = *reinterpret_cast<const f4 *>(&B[jl * kStrIM + 8 * g + 4 * h]);
#pragma unroll
          for (int s = 0; s < 4; ++s) bv[x][s] = v[s];
        }
      }
    };
    auto mfma16 = [&](const float (&av)[2][4], const float (&bv)[2][4]) {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[a][s], bv[b][s], acc[a][b], 0, 0, 0);
    };
    if constexpr (kFragAhead) {
      // group g + 1's fragments are read while group g's 16 MFMAs run: the
      // wave keeps its own MFMA pipe fed instead of waiting one LDS latency
      // per MFMA step for the other wave of its SIMD to cover it
      float av[2][2][4], bv[2][2][4];
      frag(0, av[0], bv[0]);
#pragma unroll
      for (int g = 0; g < kKC / 8; ++g) {
        if (g + 1 < kKC / 8) frag(g + 1, av[(g + 1) & 1], bv[(g + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);  // the next group's ds_reads stay ahead of this group's MFMAs
        mfma16(av[g & 1], bv[g & 1]);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int g = 0; g < kKC / 8; ++g) {
        float av[2][4], bv[2][4];
        frag(g, av, bv);
        mfma16(av, bv);
      }
    }
    if (!kDiagNoLs && r0 + kKC < re) lstore(cur ^ 1, (cur ^ 1) % kDepth, r0 + kKC);
    if (!kDiagNoBar) __syncthreads();
  };
  if (kPairLoop) {
    // stage pairs, then an odd last stage: no exit from between the two
    // parities, whose accumulators the compiler otherwise copied to the exit's
    // registers every pair (64 VGPRs and 32 moves behind an MFMA drain)
    const int nst = rb < re ? (int)((re - rb + kKC - 1) / kKC) : 0;
    int k = 0;
    for (; k + 2 <= nst; k += 2) {
      stage(std::integral_constant<int, 0>{}, rb + (int64_t)k * kKC);
      stage(std::integral_constant<int, 1>{}, rb + (int64_t)(k + 1) * kKC);
    }
    if (k < nst) stage(std::integral_constant<int, 0>{}, rb + (int64_t)k * kKC);
  } else {
    for (int64_t r0 = rb; r0 < re;) {
      stage(std::integral_constant<int, 0>{}, r0);
      r0 += kKC;
      if (r0 >= re) break;
      stage(std::integral_constant<int, 1>{}, r0);
      r0 += kKC;
    }
  }
  if constexpr (Epi::kBlock) {
    static_assert(kBM * EpiMsg::kS <= 2 * kBufF, "a parked P or Q tile fits one operand's two buffers");
    epi.block(acc, sA[0], sB[0], i0, j0, I, wi, wj, lane, t);
    return;
  }
  if (i0 + kBM <= I && j0 + kBN <= J) {  // workgroup-uniform: interior tiles store unchecked
    f16 pm[2][2];
    if (Epi::kPre) {
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int v = 0; v < 16; ++v)
            pm[a][b][v] = epi.pre(i0 + 64 * wi + 32 * a + 8 * (v >> 2) + 4 * h + (v & 3), j0 + 64 * wj + 32 * b + (lane & 31));
    }
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int64_t j = j0 + 64 * wj + 32 * b + (lane & 31);
      const float bj = epi.bias_of(j);
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int v = 0; v < 16; ++v)
          epi(i0 + 64 * wi + 32 * a + 8 * (v >> 2) + 4 * h + (v & 3), j, acc[a][b][v], bj, Epi::kPre ? pm[a][b][v] : 0.f);
    }
  } else {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int64_t j = j0 + 64 * wj + 32 * b + (lane & 31);
      const float bj = j < J ? epi.bias_of(j) : 0.f;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int64_t i = i0 + 64 * wi + 32 * a + 8 * (v >> 2) + 4 * h + (v & 3);
          if (i < I && j < J) epi(i, j, acc[a][b][v], bj, Epi::kPre ? epi.pre(i, j) : 0.f);
        }
    }
  }
  if (COLSUM && by == 0) {
    // thread t summed the rows t>>5 (+8q) of columns 4(t&31)..+3: fold the 8 row groups in order
    __shared__ f4 s_cs[256];
    s_cs[t] = csum;
    __syncthreads();
    if (t < 32) {
      f4 v = s_cs[t];
#pragma unroll
      for (int g = 1; g < 8; ++g) v += s_cs[t + 32 * g];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t i = i0 + 4 * t + e;
        if (i < I) bias_part[(int64_t)bz * I + i] = v[e];
      }
    }
  }
}

template <class LA, bool ARM, class LB, bool BRM, class Epi, bool COLSUM, bool EX = false>
__global__ __launch_bounds__(256, HF_TG_WG) void tgemm_kernel(LA ga, LB gb, Epi epi, int64_t I, int64_t J, int64_t R,
                                                       int64_t rsplit, float *bias_part) {
  unsigned bx, by, bz;
  tg_block(bx, by, bz);
  tg_stagger();
  tgemm_tile<LA, ARM, LB, BRM, Epi, COLSUM, EX>(ga, gb, epi, I, J, R, rsplit, bias_part, bx, by, bz);
}

// NB independent GEMMs of one shape in ONE launch (the layers' weight
// gradients, each from its own operands into its own partials): grid z =
// problem * S + split.  One launch keeps the machine full across the
// problems' tails, which a launch per problem drains (each is about one wave
// of workgroups).  Every tile's arithmetic is tgemm_kernel's.
constexpr int kTgMaxBatch = 8;
template <class LA, class LB, class Epi>
struct TgBatch {
  LA a[kTgMaxBatch];
  LB b[kTgMaxBatch];
  Epi e[kTgMaxBatch];
  float *bias_part[kTgMaxBatch];
  int n;      // problems
  int64_t S;  // splits per problem
};
template <class LA, bool ARM, class LB, bool BRM, class Epi, bool COLSUM, bool EX = false>
__global__ __launch_bounds__(256, HF_TG_WG) void tgemm_batch_kernel(TgBatch<LA, LB, Epi> bt, int64_t I, int64_t J,
                                                             int64_t R, int64_t rsplit) {
  unsigned bx, by, bz;
  tg_block(bx, by, bz);
  tg_stagger();
  const unsigned pb = bz / (unsigned)bt.S, sz = bz - pb * (unsigned)bt.S;
  tgemm_tile<LA, ARM, LB, BRM, Epi, COLSUM, EX>(bt.a[pb], bt.b[pb], bt.e[pb], I, J, R, rsplit, bt.bias_part[pb], bx, by,
                                                sz);
}

#ifndef HF_TG_EXACT
#define HF_TG_EXACT 1
#endif
// EXOK (both operands RM): the exact kernel where the shapes allow it
template <class LA, bool ARM, class LB, bool BRM, class Epi, bool COLSUM = false, bool EXOK = false>
hipError_t tgemm(const LA &ga, const LB &gb, const Epi &epi, int64_t I, int64_t J, int64_t R, int splits,
                 hipStream_t s, float *bias_part = nullptr) {
  if (I <= 0 || J <= 0) return hipSuccess;
  if (!ga.fits32() || !gb.fits32()) return hipErrorInvalidValue;  // 32-bit row offsets
  if ((!ARM || !BRM) && R % kKC != 0) return hipErrorInvalidValue;  // [i][r] operands: whole chunks
  int64_t rsplit = (R + splits - 1) / splits;
  rsplit = (rsplit + kKC - 1) / kKC * kKC;
  const int64_t S = R > 0 ? (R + rsplit - 1) / rsplit : 1;
  dim3 grid((unsigned)((I + kBM - 1) / kBM), (unsigned)((J + kBN - 1) / kBN), (unsigned)S);
  if constexpr (EXOK && ARM && BRM) {
    if (HF_TG_EXACT && R > 0 && I % kBM == 0 && J % kBN == 0 && R % kKC == 0 && ga.exact_ok(R) && gb.exact_ok(R)) {
      hipLaunchKernelGGL((tgemm_kernel<LA, ARM, LB, BRM, Epi, COLSUM, true>), grid, dim3(256), 0, s, ga, gb, epi, I, J,
                         R, rsplit, bias_part);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((tgemm_kernel<LA, ARM, LB, BRM, Epi, COLSUM>), grid, dim3(256), 0, s, ga, gb, epi, I, J, R,
                     rsplit > 0 ? rsplit : kKC, bias_part);
  return hipGetLastError();
}
// The NB = bt.n problems of bt in one launch (both operands along the
// reduction, EpiPart-style split partials): the exact kernel when every
// problem's shapes allow it, as tgemm.
template <class LA, class LB, class Epi, bool COLSUM>
hipError_t tgemm_batch(TgBatch<LA, LB, Epi> bt, int64_t I, int64_t J, int64_t R, int splits, hipStream_t s) {
  if (I <= 0 || J <= 0 || bt.n <= 0) return hipSuccess;
  if (bt.n > kTgMaxBatch) return hipErrorInvalidValue;
  bool exact = HF_TG_EXACT && R > 0 && I % kBM == 0 && J % kBN == 0 && R % kKC == 0;
  for (int p = 0; p < bt.n; ++p) {
    if (!bt.a[p].fits32() || !bt.b[p].fits32()) return hipErrorInvalidValue;
    exact = exact && bt.a[p].exact_ok(R) && bt.b[p].exact_ok(R);
  }
  int64_t rsplit = (R + splits - 1) / splits;
  rsplit = (rsplit + kKC - 1) / kKC * kKC;
  bt.S = R > 0 ? (R + rsplit - 1) / rsplit : 1;
  dim3 grid((unsigned)((I + kBM - 1) / kBM), (unsigned)((J + kBN - 1) / kBN), (unsigned)(bt.S * bt.n));
  if (exact)
    hipLaunchKernelGGL((tgemm_batch_kernel<LA, true, LB, true, Epi, COLSUM, true>), grid, dim3(256), 0, s, bt, I, J, R,
                       rsplit);
  else
    hipLaunchKernelGGL((tgemm_batch_kernel<LA, true, LB, true, Epi, COLSUM>), grid, dim3(256), 0, s, bt, I, J, R,
                       rsplit > 0 ? rsplit : kKC);
  return hipGetLastError();
}
// number of splits tgemm makes of R for a requested count
inline int64_t tgemm_splits(int64_t R, int splits) {
  int64_t rsplit = (R + splits - 1) / splits;
  rsplit = (rsplit + kKC - 1) / kKC * kKC;
  return R > 0 ? (R + rsplit - 1) / rsplit : 1;
}

}  // namespace tg
}  // namespace hf
