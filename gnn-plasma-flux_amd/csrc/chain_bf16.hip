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
// row e&3; capi.cpp packs the weights in that k order).
//
// Aggregation by linearity, on the output side:
//   W_b (h[i-1] + h[i+1]) / 2 = G(i-1) + G(i+1),   G = (W_b/2) bf16(h),
// so a layer's MFMAs read ONE activation fragment set, bf16(h): A = W_a h + b
// and G accumulate side by side (the packer already halves W_b, exactly:
// bf16(w/2) == bf16(w)/2), and the epilogue forms z = A + (G(i-1) + G(i+1))
// on the interleaved cell layout (one fp32 add of the two neighbours, a plain
// v_add or a DPP row rotation at the tile seam, then one add into A), ReLU,
// bf16 pairs.  Against a neighbour-sum B fragment this halves the activation
// registers; a wave fits in 256 VGPRs, so the windowed kernel runs NW = 8
// waves: two per SIMD, which hide each other's LDS, barrier and epilogue
// latency.  cfg4 (4096 ICs x 1024 cells) measured 35.3 % of the dense bf16
// peak with the neighbour-sum fragment at one wave per SIMD, 37.6 % with the
// sum as two shifted B operands (3 MFMAs per fragment, two waves per SIMD) and
// 43.2 % in this form (profiles/r02_cfg4_core_ab.json).  The arithmetic is
// oracle.hybrid_flux_edge_bf16 (float64-emulated f32 accumulation).
//
// Schedule: a layer is walked in OUTPUT-PAIR order (pair q = tiles 2q, 2q+1,
// 4 units = the 4 k-blocks of h, 2 x 2 x MT MFMAs each) and the epilogue of
// pair q-1 is spread over pair q's units, one fragment dword per unit.  The new
// fragments of pairs 0..2 are parked in LDS (the old ones still feed the
// layer) and read back when the layer ends; the epilogue of pair 3 runs under
// the first three k-blocks of the next layer's pair 0 (or the first readout
// tile), which produce nothing it needs.  The readout is pipelined tile by tile.
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
// ReLU of two f32 values packed to bf16.  HF_EXP_IRELU (experiment): convert
// first, then a signed 16-bit max with 0 on the bf16 bit patterns (one
// v_pk_max_i16 for two values); equal to bf16(relu(z)) except that a
// negative-signed NaN becomes +0.
__device__ __forceinline__ unsigned pk_relu_bf16(float a, float b) {
#ifdef HF_EXP_IRELU
  typedef short s2 __attribute__((ext_vector_type(2)));
  const s2 v = __builtin_bit_cast(s2, pk_bf16(a, b));
  return __builtin_bit_cast(unsigned, __builtin_elementwise_max(v, s2{0, 0}));
#else
  return pk_bf16(relu(a), relu(b));
#endif
}
__device__ __forceinline__ f4 mma(const u4 &a, const u4 &b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8, a), __builtin_bit_cast(b8, b), c, 0, 0, 0);
}

// Closes one unit's scheduling region: ND ds_reads first (the unit's 4
// fragments, or the seam reads after a ring barrier), then one MFMA and up to
// NV VALU (epilogue work of the previous pair) at a time.  The sched_barrier
// keeps the next unit's reads from being picked for this unit's DS group.
#ifndef HF_EXP_VFIRST
#define HF_EXP_VFIRST 0
#endif
template <int NM, int NV, int ND = 4>
__device__ __forceinline__ void interleave() {
  __builtin_amdgcn_sched_group_barrier(0x100, ND, 0);
  // experiment: VALU issued between the fragment reads and the first MFMA
  if constexpr (HF_EXP_VFIRST > 0 && NV > 0) __builtin_amdgcn_sched_group_barrier(0x002, HF_EXP_VFIRST, 0);
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
}

// NW = waves per workgroup sharing the weight ring: 8 (two per SIMD) for the
// flux kernels, 4 for the rollout kernel (one IC per wave beside its per-IC
// LDS scratch).  UPC = units (4 fragments, 4 KiB) per ring chunk: 4 (16 KiB
// chunks, 3 slots: one ring barrier per output pair) or 2 (8 KiB, 4 slots:
// the rollout, whose scratch leaves no room for the larger ring).  WMT =
// m-tiles per wave of the windowed flux kernel (64-cell windows).  PF = read
// the next unit's fragments one unit ahead (16 more registers: the rollout's
// one wave per SIMD has them; at two waves per SIMD the partner wave covers
// the latency and the registers are what let two waves fit).
//
// XCH (super-windows, chain_flux_sw_kernel): the NW waves of a workgroup hold
// consecutive 64-cell pieces of one long chain, overlapping by one cell, and
// trade the G values of their edge cells through LDS every layer, so only the
// workgroup's two outer edges see a wrong neighbour.  The trade needs a ring
// barrier between the pair whose G it is and that pair's epilogue: the ring's
// chunks start two units into a pair (the packed stream carries a copy of its
// first two units after the pass, kBF16StreamTail), so the barrier falls
// between unit 1's fragment reads and its MFMAs, after the seam publish in unit 0.
template <int NW, int UPC, int WMT = 4, bool PF = false, int SLOTS = (UPC == 4 ? 3 : 4), int WG = 1, int DMAU = 0,
          bool XCH = false, bool LDR = false>
struct CoreBF16 {
  static_assert(!XCH || (UPC == 4 && !PF && WMT == 4), "super-window core: 16 KiB chunks, 64-cell waves");
  static constexpr int kNW = NW;
  static constexpr int kWGPerCU = WG;
  static constexpr int kUPC = UPC;
  static constexpr int kSlots = SLOTS;
  static constexpr int kAhead = 2;
  static constexpr int kWinMT = WMT;
  static constexpr int kParkMT = WMT;
  static constexpr int kChunkFloats = 1024 * UPC;
  static constexpr int kKB = kH / 32;
  static constexpr int kStreamOffset = XCH ? kBF16StreamTail : 0;
  // parked h fragments of k-blocks 0..2: [kb 3][mt kParkMT][lane 64][4 dwords]
  static constexpr int kParkFloats = 3 * kParkMT * 64 * 4;
  // seam trade buffer (XCH): [parity 2][wave NW][side 2][g 4][tile 2] f4
  static constexpr int kSeamF4 = XCH ? 2 * NW * 2 * 4 * 2 : 0;
  // DMAU >= 0: the ring's DMA for chunk p+2 is issued in unit DMAU of chunk p
  // (after that unit's fragment reads) instead of right after the ring
  // barrier, where all waves' DMA and fragment reads would queue together:
  // cfg4 3-5 % less time at DMAU = 0 (unit 3: 2-3 %, units 1-2: 2 %; spreading
  // the DMA over the units by wave number: 10 % more), tools/gpu_diag_cfg4.sh.
  static constexpr int kDmaUnit = DMAU;
  using R_t = Ring<kChunkFloats, NW, kSlots, 2, (DMAU >= 0), LDR>;  // LDR: a loader wave issues the ring DMA
  // ring position of pair-unit U (of readout unit U: the same, counted from the readout's start)
  static constexpr int pos(int U) { return XCH ? (U + 2) & 3 : U % UPC; }

  template <int MT>
  struct Acts {
    u4 h[MT][kKB];  // B fragments of bf16(h)
  };
  // A (= b + W_a h) and G (= (W_b/2) h) accumulators of one output pair
  template <int MT>
  struct Pair {
    f4 a[MT][2], g[MT][2];
  };

  // XCH: this wave's view of the seam trade.  Side 0 = the wave's cell 1
  // (tile 1, lane column 0), read by the LEFT wave for its cell 63's right
  // neighbour; side 1 = cell 62 (tile 2, column 15), read by the RIGHT wave for
  // its cell 0's left neighbour (waves overlap by one cell: cell 63 of wave w
  // is cell 0 of wave w+1).
  struct Seam {
    f4 *pubw;  // this wave's side-0 slots at parity 0 (wave-uniform; side 1 is +8)
    f4 *rdl;   // the left wave's side-1 slots at parity 0 (wave-uniform)
    f4 *rdr;   // the right wave's side-0 slots at parity 0 (wave-uniform)
    // (waves 0 and NW-1 read each other: the super-window's ends are wrong after
    // any update layer and never output; with no update layer the traded G is
    // zero, so the ends stay exact)
    int par;
    // [parity 2][wave NW][side 2][g 4][tile 2] f4
    static __device__ __forceinline__ int slot(int w, int side) { return (w * 2 + side) * 8; }
    // This lane's id, from v_mbcnt in an opaque statement at each use: the
    // compiler then holds no per-lane seam address across the pass (held ones
    // were spilled, and each scratch reload waited for the ring's DMA).
    static __device__ __forceinline__ int lane_id() {
      int l;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
      return l;
    }
  };
  template <int MT>
  static __device__ __forceinline__ void publish(const Seam &sm, const Pair<MT> &P) {
#if defined(HF_DIAG_NOSEAM) || defined(HF_DIAG_NOPUB)  // timing diagnostic only: results are wrong (no seam trade)
    return;
#endif
    if constexpr (XCH) {
      const int l = Seam::lane_id(), j = l & 15;
      f4 *p = sm.pubw + sm.par * (NW * 16) + ((l >> 4) << 1);
      if (j == 0) {
        p[0] = P.g[1][0];
        p[1] = P.g[1][1];
      }
      if (j == 15) {
        p[8] = P.g[MT - 2][0];
        p[9] = P.g[MT - 2][1];
      }
    }
  }
  // After the ring barrier that follows publish(): the neighbours' seam G of
  // tile t (lanes j = 0 use L, lanes j = 15 use R).
  static __device__ __forceinline__ void seam_read(const Seam &sm, int t, f4 &L, f4 &R) {
#if defined(HF_DIAG_NOSEAM) || defined(HF_DIAG_NORD)
    L = R = f4{0.f, 0.f, 0.f, 0.f};
    return;
#endif
    const int l = Seam::lane_id(), o = sm.par * (NW * 16) + ((l >> 4) << 1) + t;
#ifdef HF_EXP_SEAM1
    // experiment: one read per tile: lanes j = 15 read the right wave's value,
    // every other lane the left wave's (only j = 0 uses L, only j = 15 uses R)
    L = R = ((l & 15) == 15 ? sm.rdr : sm.rdl)[o];
#else
    L = sm.rdl[o];
    R = sm.rdr[o];
#endif
  }

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
    // XCH starts at position 2 of the first chunk: no position kDmaUnit = 0
    // comes before the next barrier, so the DMA owed now is issued now
    if constexpr (XCH) R.issue_pending();
    if constexpr (PF) load_unit(F, 0, R.lane);
  }
  // The 4 fragments at ring position U (the last position of a chunk also
  // waits for, and releases, the next chunk).
  template <int U>
  static __device__ __forceinline__ void take(R_t &R, Feed &F, u4 (&w)[4]) {
    if constexpr (PF) {
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] = F.cur[i];
      if constexpr (U == kDmaUnit) R.issue_pending();
      if constexpr (U == UPC - 1) F.slot = R.next();
      load_unit(F, (U + 1) % UPC, R.lane);
    } else {
#ifdef HF_DIAG_NODS  // timing diagnostic only: results are wrong (no fragment ds_reads: lane-made fragments)
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] = u4{(unsigned)R.lane, (unsigned)(4 * U + i), 0x3f803f80u, (unsigned)R.lane};
#else
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] = __builtin_bit_cast(u4, ldf4(F.slot + ((4 * U + i) * 64 + R.lane) * 4));
#endif
      if constexpr (U == kDmaUnit) R.issue_pending();
      if constexpr (U == UPC - 1) F.slot = R.next();
    }
  }

  static __device__ __forceinline__ float *park_at(float *park, int kb, int mt, int lane) {
    return park + ((kb * kParkMT + mt) * 64 + lane) * 4;
  }

  // MFMAs of one update unit: k-block KB, fragments w[2t] = W_a, w[2t+1] = W_b/2 of tile t.
  template <int MT, int KB>
  static __device__ __forceinline__ void unit_mfma(const u4 (&w)[4], const Acts<MT> &X, Pair<MT> &P) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        P.a[mt][t] = mma(w[2 * t], X.h[mt][KB], P.a[mt][t]);
        P.g[mt][t] = mma(w[2 * t + 1], X.h[mt][KB], P.g[mt][t]);
      }
  }
  template <int MT, int KB>
  static __device__ __forceinline__ void unit(R_t &R, Feed &F, const Acts<MT> &X, Pair<MT> &P) {
    u4 w[4];
    take<pos(KB)>(R, F, w);
    unit_mfma<MT, KB>(w, X, P);
  }

  // b_l enters A as the C operand of its first MFMA
  template <int MT>
  static __device__ __forceinline__ void init(const float *bias, int q, int g4, Pair<MT> &P) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const f4 b = ldf4(bias + 16 * (2 * q + t) + g4);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        P.a[mt][t] = b;
        P.g[mt][t] = f4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }

  // Dword K of the k-block fragment made from one output pair (tile t = K>>1,
  // rows r0 = 2(K&1), r0+1): z = A + (G(i-1) + G(i+1)), ReLU, bf16 pairs.
  // PART 0: every m-tile (periodic 16*MT-cell window); 1: the inner m-tiles
  // 1..MT-2; 2 (XCH): the edge m-tiles 0 and MT-1, whose lane-column-0 left /
  // column-15 right neighbours are the seam values L / R of tile t.
  template <int MT, int K, int PART = 0>
  static __device__ __forceinline__ void piece(Pair<MT> &P, u4 (&nh)[MT], const f4 &L = f4{}, const f4 &R = f4{}) {
    constexpr int t = K >> 1, r0 = 2 * (K & 1);
#ifdef HF_DIAG_NOPIECE  // timing diagnostic only: results are wrong (one convert per dword, no epilogue VALU)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
      if (PART == 0 || (PART == 1) == (mt > 0 && mt < MT - 1)) nh[mt][K] = pk_bf16(P.a[mt][t][r0], P.g[mt][t][r0 + 1]);
    return;
#endif
    if constexpr (PART == 0) {
      float z[2][MT];
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
        float v[MT], sm[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) v[mt] = P.g[mt][t][r0 + rr];
        nb_sum<MT>(v, sm);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) z[rr][mt] = __fadd_rn(P.a[mt][t][r0 + rr], sm[mt]);
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) nh[mt][K] = pk_relu_bf16(z[0][mt], z[1][mt]);
    } else if constexpr (PART == 1) {
#pragma unroll
      for (int mt = 1; mt < MT - 1; ++mt) {
        float z[2];
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
          const int r = r0 + rr;
          z[rr] = __fadd_rn(P.a[mt][t][r], __fadd_rn(P.g[mt - 1][t][r], P.g[mt + 1][t][r]));
        }
        nh[mt][K] = pk_relu_bf16(z[0], z[1]);
      }
    } else {
      float z0[2], z1[2];
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) {
        const int r = r0 + rr;
        // cell 4j: left = cell 4j-1 (tile MT-1, column j-1), the seam value L at
        // j = 0.  Every lane first forms L + G(4j+1); one v_add_f32_dpp row_shr:1
        // without bound_ctrl then overwrites lanes j >= 1 with G(4j-1) + G(4j+1)
        // and leaves lane 0 (no source lane) as it is: the same single fp32 add
        // of the two neighbours in every lane.  (Inline asm: hipcc folds a DPP
        // mov into an add only when the mov's old value is zero.  The output is
        // tied to the compiler-written sum, and both sources are MFMA results of
        // the previous pair, so the asm adds no register hazard.)
        float sl = __fadd_rn(L[r], P.g[1][t][r]);
        asm("v_add_f32_dpp %0, %1, %2 row_shr:1 row_mask:0xf bank_mask:0xf"
            : "+v"(sl)
            : "v"(P.g[MT - 1][t][r]), "v"(P.g[1][t][r]));
        z0[rr] = __fadd_rn(P.a[0][t][r], sl);
        // cell 4j+MT-1: right = cell 4j+MT (tile 0, column j+1), the seam value R at j = 15
        float sr = __fadd_rn(R[r], P.g[MT - 2][t][r]);
        asm("v_add_f32_dpp %0, %1, %2 row_shl:1 row_mask:0xf bank_mask:0xf"
            : "+v"(sr)
            : "v"(P.g[0][t][r]), "v"(P.g[MT - 2][t][r]));
        z1[rr] = __fadd_rn(P.a[MT - 1][t][r], sr);
      }
      nh[0][K] = pk_relu_bf16(z0[0], z0[1]);
      nh[MT - 1][K] = pk_relu_bf16(z1[0], z1[1]);
    }
  }

  // Output pair q >= 1, with the epilogue of pair q-1 (prev) spread over its 4
  // units and parked as k-block q-1.
  template <int MT>
  static __device__ __forceinline__ void pair_with_prev(R_t &R, Feed &F, const Acts<MT> &X, const float *bias, int q,
                                                        int g4, Pair<MT> &acc, Pair<MT> &prev, float *park,
                                                        int lane, Seam &sm) {
    init<MT>(bias, q, g4, acc);
    u4 nh[MT];
    if constexpr (XCH) {
      unit<MT, 0>(R, F, X, acc);
      piece<MT, 0, 1>(prev, nh);
      piece<MT, 1, 1>(prev, nh);
      interleave<4 * MT, 2>();
      publish<MT>(sm, prev);
      unit<MT, 1>(R, F, X, acc);  // ring barrier: every wave's seam is published
      // each unit's seam VALU (waiting on the seam reads) come after
      // independent inner-tile work, so the reads' latency is covered
      f4 L0, R0;
      seam_read(sm, 0, L0, R0);
      piece<MT, 2, 1>(prev, nh);
      piece<MT, 0, 2>(prev, nh, L0, R0);
      interleave<4 * MT, 2, 2>();
      unit<MT, 2>(R, F, X, acc);
      f4 L1, R1;
      seam_read(sm, 1, L1, R1);
      piece<MT, 3, 1>(prev, nh);
      piece<MT, 1, 2>(prev, nh, L0, R0);
      interleave<4 * MT, 2, 6>();
      unit<MT, 3>(R, F, X, acc);
      piece<MT, 2, 2>(prev, nh, L1, R1);
      piece<MT, 3, 2>(prev, nh, L1, R1);
      sm.par ^= 1;
    } else {
      unit<MT, 0>(R, F, X, acc);
      piece<MT, 0>(prev, nh);
      interleave<4 * MT, 2>();
      unit<MT, 1>(R, F, X, acc);
      piece<MT, 1>(prev, nh);
      interleave<4 * MT, 2>();
      unit<MT, 2>(R, F, X, acc);
      piece<MT, 2>(prev, nh);
      interleave<4 * MT, 2>();
      unit<MT, 3>(R, F, X, acc);
      piece<MT, 3>(prev, nh);
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) *reinterpret_cast<u4 *>(park_at(park, q - 1, mt, lane)) = nh[mt];
    interleave<4 * MT, 2>();
  }

  // Pair 0 of a layer that follows another: k-blocks 0..2 come back from the
  // park, k-block 3 is the previous layer's pair 3 (pend), finished under the
  // first three units.
  template <int MT>
  static __device__ __forceinline__ void pair0_after(R_t &R, Feed &F, Acts<MT> &X, const float *bias, int g4,
                                                     Pair<MT> &acc, Pair<MT> &pend, float *park, int lane, Seam &sm) {
    wave_lds_sync();  // this wave's park writes of the previous layer have landed
#pragma unroll
    for (int kb = 0; kb < 3; ++kb)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) X.h[mt][kb] = __builtin_bit_cast(u4, ldf4(park_at(park, kb, mt, lane)));
    init<MT>(bias, 0, g4, acc);
    u4 nh[MT];
    if constexpr (XCH) {
      unit<MT, 0>(R, F, X, acc);
      piece<MT, 0, 1>(pend, nh);
      piece<MT, 1, 1>(pend, nh);
      piece<MT, 2, 1>(pend, nh);
      interleave<4 * MT, 3>();
      publish<MT>(sm, pend);
      unit<MT, 1>(R, F, X, acc);  // ring barrier
      f4 L0, R0, L1, R1;
      seam_read(sm, 0, L0, R0);
      seam_read(sm, 1, L1, R1);
      piece<MT, 3, 1>(pend, nh);
      piece<MT, 0, 2>(pend, nh, L0, R0);
      interleave<4 * MT, 2, 4>();
      unit<MT, 2>(R, F, X, acc);
      piece<MT, 1, 2>(pend, nh, L0, R0);
      piece<MT, 2, 2>(pend, nh, L1, R1);
      piece<MT, 3, 2>(pend, nh, L1, R1);
      interleave<4 * MT, 4>();
      sm.par ^= 1;
    } else {
      unit<MT, 0>(R, F, X, acc);
      piece<MT, 0>(pend, nh);
      piece<MT, 1>(pend, nh);
      interleave<4 * MT, 4>();
      unit<MT, 1>(R, F, X, acc);
      piece<MT, 2>(pend, nh);
      interleave<4 * MT, 2>();
      unit<MT, 2>(R, F, X, acc);
      piece<MT, 3>(pend, nh);
      interleave<4 * MT, 2>();
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) X.h[mt][3] = nh[mt];
    unit<MT, 3>(R, F, X, acc);
    interleave<4 * MT, 0>();
  }

  // Pair 0 of the first layer (X complete from the input layer).
  template <int MT>
  static __device__ __forceinline__ void pair0_first(R_t &R, Feed &F, const Acts<MT> &X, const float *bias, int g4,
                                                     Pair<MT> &acc) {
    init<MT>(bias, 0, g4, acc);
    unit<MT, 0>(R, F, X, acc);
    interleave<4 * MT, 0>();
    unit<MT, 1>(R, F, X, acc);
    interleave<4 * MT, 0>();
    unit<MT, 2>(R, F, X, acc);
    interleave<4 * MT, 0>();
    unit<MT, 3>(R, F, X, acc);
    interleave<4 * MT, 0>();
  }

  // Pairs 1..3 of a layer; leaves pair 3 in pend (its epilogue is pending).
  template <int MT>
  static __device__ __forceinline__ void pairs_rest(R_t &R, Feed &F, const Acts<MT> &X, const float *bias, int g4,
                                                    Pair<MT> &acc0, Pair<MT> &pend, float *park, int lane, Seam &sm) {
    Pair<MT> acc1, acc2;
    pair_with_prev<MT>(R, F, X, bias, 1, g4, acc1, acc0, park, lane, sm);
    pair_with_prev<MT>(R, F, X, bias, 2, g4, acc2, acc1, park, lane, sm);
    pair_with_prev<MT>(R, F, X, bias, 3, g4, pend, acc2, park, lane, sm);
  }

  // ------------------------------------------------------------- readout
  // MFMAs of readout unit U of one output tile: fragment i = 2*(kb - 2U) + (P|Q), kb = 2U, 2U+1.
  template <int MT, int U>
  static __device__ __forceinline__ void ro_mfma(const u4 (&w)[4], const Acts<MT> &X, f4 (&P)[MT], f4 (&Q)[MT]) {
#ifdef HF_DIAG_NOROMFMA  // timing diagnostic only: results are wrong (readout fragments read, no readout MFMA)
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(w[i]));
    return;
#endif
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
  // ... at ring position T.
  template <int MT, int U, int T>
  static __device__ __forceinline__ void ro_unit(R_t &R, Feed &F, const Acts<MT> &X, f4 (&P)[MT], f4 (&Q)[MT]) {
    u4 w[4];
    take<T>(R, F, w);
    ro_mfma<MT, U>(w, X, P, Q);
  }

  // Rows 2RP, 2RP+1 of one readout tile's epilogue: z_fwd(i) = P(i) + Q(i+1),
  // z_bwd(i) = P(i+1) + Q(i) (b_e already in P); partial += w2 . ReLU(z)
  // (src/flux_gnn.py:62-66), rows in order as readout_epilogue.
  template <int MT, int RP>
  static __device__ __forceinline__ void ro_piece(const f4 (&P)[MT], const f4 (&Q)[MT], const f4 &w2, float (&pf)[MT],
                                                  float (&pb)[MT]) {
#ifdef HF_DIAG_NOROPIECE  // timing diagnostic only: results are wrong (one add per accumulator pair)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) pf[mt] += P[mt][2 * RP] + Q[mt][2 * RP + 1];
    return;
#endif
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

  // Readout tile ot >= 1 (ring positions T0, T0+1), with the epilogue of tile
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
  // 0..2 comes from the park, k-block 3 is finished under the first readout unit
  // (XCH: its edge m-tiles after the second unit's ring barrier, before the
  // MFMAs that read k-block 3).
  template <int MT>
  static __device__ __forceinline__ void readout(const ChainW &W, const Small &S, R_t &R, Feed &F, Acts<MT> &X,
                                                 Pair<MT> &pend, float *park, int lane, int g4, float (&ffwd)[MT],
                                                 float (&fbwd)[MT], Seam &sm) {
#ifndef HF_DIAG_NOPARK
    wave_lds_sync();
#pragma unroll
    for (int kb = 0; kb < 3; ++kb)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) X.h[mt][kb] = __builtin_bit_cast(u4, ldf4(park_at(park, kb, mt, lane)));
#endif
    float pf[MT], pb[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) pf[mt] = pb[mt] = 0.f;
    f4 P[MT], Q[MT];
    init_ro<MT>(S, 0, g4, P, Q);
    {
      u4 nh[MT];
      if constexpr (XCH) {
        ro_unit<MT, 0, pos(0)>(R, F, X, P, Q);
        piece<MT, 0, 1>(pend, nh);
        piece<MT, 1, 1>(pend, nh);
        piece<MT, 2, 1>(pend, nh);
        piece<MT, 3, 1>(pend, nh);
        interleave<4 * MT, 4>();
        publish<MT>(sm, pend);
        u4 w[4];
        take<pos(1)>(R, F, w);  // ring barrier
        f4 L0, R0, L1, R1;
        seam_read(sm, 0, L0, R0);
        seam_read(sm, 1, L1, R1);
        // (with no update layer pend's G is zero, published and traded as such)
        piece<MT, 0, 2>(pend, nh, L0, R0);
        piece<MT, 1, 2>(pend, nh, L0, R0);
        piece<MT, 2, 2>(pend, nh, L1, R1);
        piece<MT, 3, 2>(pend, nh, L1, R1);
        sm.par ^= 1;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) X.h[mt][3] = nh[mt];
        ro_mfma<MT, 1>(w, X, P, Q);
        interleave<4 * MT, 5>();
      } else {
        ro_unit<MT, 0, 0>(R, F, X, P, Q);
        piece<MT, 0>(pend, nh);
        piece<MT, 1>(pend, nh);
        piece<MT, 2>(pend, nh);
        piece<MT, 3>(pend, nh);
        interleave<4 * MT, 4>();
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) X.h[mt][3] = nh[mt];
        ro_unit<MT, 1, 1>(R, F, X, P, Q);
        interleave<4 * MT, 0>();
      }
    }
    // tiles 1..7 at ring positions T0, T0+1: readout unit u (of 16) is at pos(u)
    constexpr int kOdd = XCH ? pos(2) : (UPC == 4 ? 2 : 0);
    constexpr int kEven = XCH ? pos(0) : 0;
    for (int ot = 1; ot < kNT - 1; ot += 2) {
      ro_tile<MT, kOdd>(R, F, X, S, ot, g4, P, Q, pf, pb);
      ro_tile<MT, kEven>(R, F, X, S, ot + 1, g4, P, Q, pf, pb);
    }
    ro_tile<MT, kOdd>(R, F, X, S, kNT - 1, g4, P, Q, pf, pb);
    {
      const f4 w2 = ldf4(S.w2 + 16 * (kNT - 1) + g4);
      ro_piece<MT, 0>(P, Q, w2, pf, pb);
      ro_piece<MT, 1>(P, Q, w2, pf, pb);
    }
    readout_finish<MT>(pf, pb, W.b2, ffwd, fbwd);
  }

  // Input MLP h0 = ReLU(W_in x + b_in) (src/flux_gnn.py:49), one bf16 MFMA per
  // 16-feature tile: lane group g's k-slots 8g, 8g+1 hold x_hi = bf16(x_g) and
  // x_lo = bf16(x_g - x_hi) against W_in[:, g] twice (W_in is bf16 in this
  // precision), so the product is W_in x to ~2^-17 relative, accumulated in f32,
  // at half the MFMA cycles of the f32 16x16x4 form.  ReLU, then bf16 pairs.
  template <int MT>
  static __device__ __forceinline__ void input(const Small &S, int lane, const float (&feat)[MT], Acts<MT> &X,
                                               f4 (&h67)[MT][2]) {
#ifdef HF_DIAG_NOINPUT  // timing diagnostic only: results are wrong (no input layer: the features' bits as h)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const unsigned v = __float_as_uint(feat[mt]);
#pragma unroll
      for (int kb = 0; kb < kKB; ++kb) X.h[mt][kb] = u4{v, v + kb, v, v};
      h67[mt][0] = h67[mt][1] = f4{feat[mt], feat[mt], feat[mt], feat[mt]};
    }
    return;
#endif
    const int g4 = 4 * (lane >> 4);
    u4 bx[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const float hi = __uint_as_float(pk_bf16(feat[mt], 0.f) << 16);
      bx[mt] = u4{pk_bf16(feat[mt], __fsub_rn(feat[mt], hi)), 0u, 0u, 0u};
    }
    const f4 a0 = ldf4(S.win + lane * 4), a1 = ldf4(S.win + 256 + lane * 4);
#pragma unroll
    for (int kb = 0; kb < kKB; ++kb) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int nt = 2 * kb + t;
        const float w = nt < 4 ? a0[nt & 3] : a1[nt & 3];
        const u4 aw = u4{pk_bf16(w, w), 0u, 0u, 0u};
        const f4 bias = ldf4(S.bin + 16 * nt + g4);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
#ifdef HF_DIAG_NOINMFMA  // timing diagnostic only: results are wrong (no input-layer MFMA)
          asm volatile("" ::"v"(aw), "v"(bx[mt]));
          const f4 h = relu4(bias);
#else
          const f4 h = relu4(mma(aw, bx[mt], bias));
#endif
          X.h[mt][kb][2 * t] = pk_bf16(h[0], h[1]);
          X.h[mt][kb][2 * t + 1] = pk_bf16(h[2], h[3]);
          if (kb == kKB - 1) h67[mt][t] = h;
        }
      }
    }
  }

  template <int MT>
  static __device__ __forceinline__ void gnn_seam(const ChainW &W, const Small &S, R_t &R, Feed &F, float *park,
                                                  Seam &sm, const float (&feat)[MT], float (&ffwd)[MT],
                                                  float (&fbwd)[MT]) {
    const int lane = R.lane;
    const int g4 = 4 * (lane >> 4);
    Acts<MT> X;
    Pair<MT> pend;
    {
      f4 h67[MT][2];  // tiles 6, 7 in f32 (the L = 0 hand-off below)
      input<MT>(S, lane, feat, X, h67);
      if (W.layers == 0) {
        // no update layer: hand the readout the input layer's output the way
        // a last layer would (k-blocks 0..2 parked, tiles 6, 7 pending with a
        // zero aggregation term; ReLU is idempotent)
#ifndef HF_DIAG_NOPARK  // timing diagnostic only (L = 0): results are wrong (no park round trip)
#pragma unroll
        for (int kb = 0; kb < 3; ++kb)
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) *reinterpret_cast<u4 *>(park_at(park, kb, mt, lane)) = X.h[mt][kb];
#endif
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          pend.a[mt][0] = h67[mt][0];
          pend.a[mt][1] = h67[mt][1];
          pend.g[mt][0] = pend.g[mt][1] = f4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
    // message passing (src/flux_gnn.py:53-60), pair-pipelined
    if (W.layers > 0) {
      Pair<MT> acc0;
      pair0_first<MT>(R, F, X, S.bl, g4, acc0);
      pairs_rest<MT>(R, F, X, S.bl, g4, acc0, pend, park, lane, sm);
    }
    // the layer count as a scalar: read from W as is, the compiler kept the
    // loop's trip counter in a VGPR, spilled it (256 VGPRs are in use) and
    // reloaded it with a scratch load whose s_waitcnt vmcnt(0) at the loop
    // latch also waited out the ring's in-flight DMA every layer
    const int nl = __builtin_amdgcn_readfirstlane(W.layers);
    for (int l = 1; l < nl; ++l) {
      const float *bias = S.bl + l * kH;
      Pair<MT> acc0;
      pair0_after<MT>(R, F, X, bias, g4, acc0, pend, park, lane, sm);
      pairs_rest<MT>(R, F, X, bias, g4, acc0, pend, park, lane, sm);
    }
    readout<MT>(W, S, R, F, X, pend, park, lane, g4, ffwd, fbwd, sm);
  }

  // The chain_common.h kernels' entry (periodic windows, no seam trade).
  template <int MT>
  static __device__ __forceinline__ void gnn(const ChainW &W, const Small &S, R_t &R, Feed &F, float *park,
                                             const float (&feat)[MT], float (&ffwd)[MT], float (&fbwd)[MT]) {
    static_assert(!XCH, "the super-window core runs in chain_flux_sw_kernel");
    Seam sm{};
    gnn_seam<MT>(W, S, R, F, park, sm, feat, ffwd, fbwd);
  }
};

// ---------------------------------------------------------------------------
// FluxGNN.forward on B periodic chains of any nx by super-windows
// (src/flux_gnn.py:40-67).  The B chains are laid end to end as one stream of
// padded segments: IC b owns stream cells [bP, bP + P), P = nx + 2L + 1, and
// segment cell p holds IC cell (p - L) mod nx, so face i (cells i, i+1) of
// IC b sits at segment cells L+i, L+i+1 and its L-layer receptive field
// [i - L, i + 1 + L] lies inside the segment.  A workgroup's NW waves take
// 63*NW + 1 consecutive stream cells (64 per wave, overlapping by one) and
// trade edge G values every layer (CoreBF16 XCH), so only the workgroup's own
// two ends are wrong after L layers: its faces [L, 63*NW - L) are exact, and
// consecutive super-windows start 63*NW - 2L cells apart.  Work per IC face:
// 64*NW / (63*NW - 2L) * P / nx, 1.04 at cfg4 (L = 4, NW = 8, nx = 1024),
// against 64/55 * 1216/1045 = 1.19 for independent 64-cell windows.
template <class Core>
__global__ __launch_bounds__(64 * Core::kNW, 1) void chain_flux_sw_kernel(ChainW W, const float *__restrict__ nf,
                                                                   const float *__restrict__ state,
                                                                   int64_t ld_state, const float *__restrict__ x,
                                                                   int B, int nx, int nsw,
                                                                   float *__restrict__ fe, float *__restrict__ ff) {
  constexpr int MT = 4, NW = Core::kNW;
  constexpr int kRingFloats = Core::kSlots * Core::kChunkFloats;
  constexpr int kBaseF4 = lds_floats<Core, false>() / 4;
  __shared__ f4 lds4[kBaseF4 + Core::kSeamF4];
  float *lds = reinterpret_cast<float *>(lds4);
  const Small S = stage_small(W, lds + kRingFloats);
  auto R = make_ring<Core>(W, lds);
  const int lane = R.lane, j = lane & 15, g = lane >> 4;
  using Seam = typename Core::Seam;
  Seam sm{lds4 + kBaseF4 + Seam::slot(R.wave, 0), lds4 + kBaseF4 + Seam::slot((R.wave + NW - 1) % NW, 1),
          lds4 + kBaseF4 + Seam::slot((R.wave + 1) % NW, 0), 0};
  __syncthreads();  // small weights staged (no DMA in flight yet)
#ifdef HF_EXP_PRIO_HI  // experiment: static issue priority 1 for the second-dispatched half (waves 4-7)
  if (R.wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
#endif
  R.prime(R.chunks - 1);  // the pass starts two units before chunk 0 (Core::pos)
  typename Core::Feed F;
  Core::begin(R, F);
  const int L = W.layers;
  const int P = nx + 2 * L + 1;
  const int faces = 63 * NW - 2 * L;  // exact faces per super-window
  const int total = B * P;            // < 2^31 (launch_flux_sw)
  // Stream cell s0 + c (c < 64) of this wave as (IC b, segment cell p): the
  // wave-uniform division once, then at most ceil(64 / P) subtractions per lane.
  auto locate = [&](int s0, int c, int &b, int &p) {
#ifdef HF_DIAG_NOLOC  // timing diagnostic only: results are wrong (IC = super-window, no index arithmetic)
    b = (s0 < 0 ? 0 : s0) / 1024 % B;
    p = c + L;
    return;
#endif
    const int base = s0 < 0 ? 0 : (s0 >= total ? total - 1 : s0);
    b = base / P;
    int s = s0 + c;
    s = s < 0 ? 0 : (s >= total ? total - 1 : s);  // outside the stream: any cell (its faces are discarded)
    p = s - b * P;
    while (p >= P) {
      p -= P;
      ++b;
    }
  };
  auto first = [&](int k) { return k * faces - L + 63 * R.wave; };  // this wave's first stream cell
  auto load_feat = [&](int k, float (&feat)[MT]) {
    const int s0 = __builtin_amdgcn_readfirstlane(first(k));
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      int b, p;
      locate(s0, cell_of<MT>(mt, j), b, p);
      int c = p - L;  // IC cell (p - L) mod nx; p - L is in [-L, nx + L]
      while (c < 0) c += nx;
      while (c >= nx) c -= nx;
#ifdef HF_DIAG_NOFEAT  // timing diagnostic only: results are wrong (no feature loads, no flux stores)
      feat[mt] = 0.01f * (float)(c + g);
#else
      feat[mt] = nf ? nf[((int64_t)b * nx + c) * kIn + g]
                    : (g < 3 ? state[b * ld_state + (int64_t)g * nx + c] : x[c]);
#endif
    }
  };
#ifdef HF_EXP_PREFETCH
  float pre[MT];
  if (blockIdx.x < nsw) load_feat(blockIdx.x, pre);
#endif
  for (int k = blockIdx.x; k < nsw; k += gridDim.x) {
    float feat[MT];
#ifdef HF_EXP_PREFETCH
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) feat[mt] = pre[mt];
    if (k + (int)gridDim.x < nsw) load_feat(k + gridDim.x, pre);  // in flight under this forward
#else
    load_feat(k, feat);
#endif
    float f_fwd[MT], f_bwd[MT];
    Core::template gnn_seam<MT>(W, S, R, F, park_of<Core, false>(lds, R.wave), sm, feat, f_fwd, f_bwd);
    const int s0 = __builtin_amdgcn_readfirstlane(first(k));
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int c = cell_of<MT>(mt, j), csw = 63 * R.wave + c;
      // the wave's last cell is the next wave's first: its face is the next wave's
      if (c == 63 || csw < L || csw >= L + faces || s0 + c >= total) continue;
      int b, p;
      locate(s0, c, b, p);
      const int i = p - L;  // face i of IC b: cells i, i+1 at segment cells p, p+1
      if (i < 0 || i >= nx) continue;
#ifdef HF_DIAG_NOFEAT
      if (f_fwd[mt] != 12345.f) continue;  // keeps the forward live; never false in practice
#endif
      if (fe && g == 0) fe[(int64_t)b * 2 * nx + i] = f_fwd[mt];
      if (fe && g == 1) fe[(int64_t)b * 2 * nx + nx + i] = f_bwd[mt];
      if (ff && g == 2) ff[(int64_t)b * nx + i] = face_flux(f_fwd[mt], f_bwd[mt]);
    }
  }
  R.drain();
}

// Super-windows of B chains of nx cells for a core of NW waves (63 exact
// faces per wave, less the L-layer halo): the one formula launch_flux_sw and
// chain_flux_work (hf_run's lane cuts) share.
inline int64_t sw_count(int NW, int layers, int64_t B, int nx) {
  const int64_t faces = 63 * NW - 2 * layers, total = B * (nx + 2 * layers + 1);
  return (total + faces - 1) / faces;
}

template <class Core>
hipError_t launch_flux_sw(const ChainW &w, const float *nf, const float *state, int64_t ld_state, const float *x,
                          int B, int nx, float *fe, float *ff, hipStream_t s) {
  const int64_t total = (int64_t)B * (nx + 2 * w.layers + 1);
  if (total >= (int64_t(1) << 31) - 64 * Core::kNW) return hipErrorInvalidValue;  // 32-bit stream index
  const int nsw = (int)sw_count(Core::kNW, w.layers, B, nx);
  const int64_t res = resident_groups();
  const int64_t blocks = nsw < res ? nsw : res;  // persistent: one per CU
  hipLaunchKernelGGL((chain_flux_sw_kernel<Core>), dim3((unsigned)blocks), dim3(64 * Core::kNW), 0, s, w, nf, state,
                     ld_state, x, B, nx, nsw, fe, ff);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Cell-split bf16 core for small batches (chain_common.h
// chain_rollout_cells_kernel / chain_flux_cells_kernel): 16 cells per wave
// (MT = 1), an IC of nx = 16*WPI cells over WPI waves.  The arithmetic is
// CoreBF16's MFMA chain for chain and add for add (A = b + W_a h and
// G = (W_b/2) h accumulated k-block by k-block, z = A + (G(i-1) + G(i+1)), the
// readout dot summed over tiles 0..7 in order), so a batch gets the
// IC-per-wave rollout's bits whichever kernel its size selects.  Not
// pipelined: a layer's four output pairs, then the G values of the wave's
// edge columns (j = 0, 15) of all 8 tiles traded through LDS around one
// barrier (CellHalo::exchange), then the epilogue; the readout trades column 0
// of P and Q the same way (CellHalo::xq).  It shares the weight ring of the
// bf16 rollout kernel (8 KiB chunks, 4 slots, fragments read a unit ahead).
template <bool LDR = false>
struct CellBF16T {
  using Base = CoreBF16<4, 2, 4, true, 4, 1, -1, false, LDR>;
  // barrier schedule of one pass (the loader wave's, chain_rollout_cells_kernel):
  // 8 ring chunks per update layer, then the G trade's barrier
  static constexpr int kLayerChunks = 8;
  static constexpr bool kLayerBarrier = true;
  static constexpr int kNW = Base::kNW;
  static constexpr int kSlots = Base::kSlots;
  static constexpr int kChunkFloats = Base::kChunkFloats;
  static constexpr int kStreamOffset = 0;
  using R_t = typename Base::R_t;
  using Feed = typename Base::Feed;
  using Acts = typename Base::template Acts<1>;
  using Pair = typename Base::template Pair<1>;
  static __device__ __forceinline__ void begin(R_t &R, Feed &F) { Base::begin(R, F); }

  static __device__ __forceinline__ void gnn_cells(const ChainW &W, const Small &S, R_t &R, Feed &F,
                                                   const float (&feat)[1], float (&ffwd)[1], float (&fbwd)[1],
                                                   CellHalo &X) {
    const int lane = R.lane, g4 = 4 * (lane >> 4);
    Acts A;
    {
      f4 h67[1][2];
      Base::template input<1>(S, lane, feat, A, h67);
    }
    // message passing (src/flux_gnn.py:53-60)
    for (int l = 0; l < W.layers; ++l) {
      const float *bias = S.bl + l * kH;
      Pair acc[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        Base::template init<1>(bias, q, g4, acc[q]);
        Base::template unit<1, 0>(R, F, A, acc[q]);
        interleave<4, 0>();
        Base::template unit<1, 1>(R, F, A, acc[q]);
        interleave<4, 0>();
        Base::template unit<1, 2>(R, F, A, acc[q]);
        interleave<4, 0>();
        Base::template unit<1, 3>(R, F, A, acc[q]);
        interleave<4, 0>();
      }
      {
        f4 G[1][kNT];
#pragma unroll
        for (int t = 0; t < kNT; ++t) G[0][t] = acc[t >> 1].g[0][t & 1];
        X.exchange(G);  // X.l / X.r: G of cell 16*pos - 1 / 16*pos + 16
      }
      // z = A + (G(i-1) + G(i+1)), ReLU, bf16 pairs: dword K of k-block q is
      // tile 2q + (K >> 1), rows 2(K & 1), 2(K & 1) + 1 (CoreBF16::piece)
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int K = 0; K < 4; ++K) {
          const int tt = K >> 1, t = 2 * q + tt, r0 = 2 * (K & 1);
          float z[2];
#pragma unroll
          for (int rr = 0; rr < 2; ++rr) {
            const int r = r0 + rr;
            const float v = acc[q].g[0][tt][r];
            const float gl = dpp_over<kRowShr1>(X.l[t][r], v), gr = dpp_over<kRowShl1>(X.r[t][r], v);
            z[rr] = __fadd_rn(acc[q].a[0][tt][r], __fadd_rn(gl, gr));
          }
          A.h[0][q][K] = pk_relu_bf16(z[0], z[1]);
        }
    }
    // edge readout, P/Q split (src/flux_gnn.py:62-66): all 8 tiles, then column
    // 0 of P and Q through LDS (P(i+1), Q(i+1) of lane j = 15 live on the right
    // wave), then the epilogue rows in CoreBF16::readout's order
    const int j = lane & 15, g = lane >> 4;
    f4 P[kNT][1], Q[kNT][1];
#pragma unroll
    for (int ot = 0; ot < kNT; ++ot) {
      Base::template init_ro<1>(S, ot, g4, P[ot], Q[ot]);
      Base::template ro_unit<1, 0, 0>(R, F, A, P[ot], Q[ot]);
      interleave<4, 0>();
      Base::template ro_unit<1, 1, 1>(R, F, A, P[ot], Q[ot]);
      interleave<4, 0>();
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
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float pv = P[ot][0][r], qv = Q[ot][0][r];
        const float pr = dpp_over<kRowShl1>(prh[r], pv), qr = dpp_over<kRowShl1>(qrh[r], qv);
        pf = fmaf(w2[r], relu(__fadd_rn(pv, qr)), pf);
        pb = fmaf(w2[r], relu(__fadd_rn(pr, qv)), pb);
      }
    }
    float pf1[1] = {pf}, pb1[1] = {pb};
    readout_finish<1>(pf1, pb1, W.b2, ffwd, fbwd);
  }
};
#ifndef HF_CELLS_LOADER
#define HF_CELLS_LOADER 1
#endif
using CellBF16Ld = CellBF16T<HF_CELLS_LOADER != 0>;  // with a loader wave (the cell-split kernels)

}  // namespace

// ring position of the deferred DMA: 0 (pair unit 2) measured best; 1, 2, 3: +3-10 % (profiles/r02_cfg4_diag.jsonl, run D)
#ifndef HF_SW_DMAU
#define HF_SW_DMAU 0
#endif
// the super-window core (any nx other than 16..64; cfg4's 1024): 8 waves, two per SIMD
using SwCoreBF16 = CoreBF16<8, 4, 4, false, 3, 1, HF_SW_DMAU, true>;

hipError_t launch_chain_flux_bf16(const ChainW &w, const float *nf, const float *state, int64_t ld_state,
                                  const float *x, int B, int nx, float *fe, float *ff, hipStream_t s) {
  // exact kernels (nx = 16..64, one wave per chain) and super-windows (any
  // other nx, e.g. cfg4's 1024): 8 waves, two per SIMD, 16 KiB chunks in 3 slots
  if (B <= 0) return hipSuccess;
  if (chain_rollout_prefers_cells(w, B, nx)) {  // small batches: each chain over nx/16 waves
    switch (nx) {
      case 32: return chain::flux_cells_launch<CellBF16Ld, 2>(w, nf, state, ld_state, x, B, fe, ff, s);
      case 48: return chain::flux_cells_launch<CellBF16Ld, 3>(w, nf, state, ld_state, x, B, fe, ff, s);
      case 64: return chain::flux_cells_launch<CellBF16Ld, 4>(w, nf, state, ld_state, x, B, fe, ff, s);
      default: break;
    }
  }
  if (nx == 16 || nx == 32 || nx == 48 || nx == 64)
    return chain::launch_flux_core<CoreBF16<8, 4>>(w, nf, state, ld_state, x, B, nx, fe, ff, s);
  return launch_flux_sw<SwCoreBF16>(w, nf, state, ld_state, x, B, nx, fe, ff, s);
}

FluxWork chain_flux_work(const ChainW &w, int64_t B, int nx) {
  FluxWork fw;
  if (w.prec != kPrecBF16 || B <= 0 || nx == 16 || nx == 32 || nx == 48 || nx == 64 ||
      chain_rollout_prefers_cells(w, (int)B, nx))
    return fw;  // not the super-window kernel
  fw.units = sw_count(SwCoreBF16::kNW, w.layers, B, nx);  // the core launch_chain_flux_bf16 runs

  fw.per_round = resident_groups();         // one per persistent workgroup per round
  return fw;
}

hipError_t launch_chain_rollout_bf16(const ChainW &w, const float *state0, float *state_final, const float *x,
                                     const double *pc, int B, int nx, int T, float c, float dt, float *traj,
                                     float *flux_traj, float *metrics, const RolloutExtras &ex, hipStream_t s) {
  // small batches: each IC over nx/16 waves (cell-split kernel, same bits)
  if (ex.mse == nullptr && ex.metrics_cl == nullptr && chain_rollout_prefers_cells(w, B, nx)) {
    switch (nx) {
      case 32: return chain::cells_launch<CellBF16Ld, 2>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, ex.poisson, s);
      case 48: return chain::cells_launch<CellBF16Ld, 3>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, ex.poisson, s);
      case 64: return chain::cells_launch<CellBF16Ld, 4>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, ex.poisson, s);
      default: break;
    }
  }
  return chain::launch_rollout_core<CoreBF16<4, 2, 4, true, 4, 1, -1>>(w, state0, state_final, x, pc, B, nx, T, c, dt, traj,
                                                             flux_traj, metrics, ex, s);
}

}  // namespace hf
