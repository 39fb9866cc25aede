// Shared machinery of the chain kernels (chain_f32.hip, chain_k32.hip):
// lane-shift neighbours, the LDS weight ring, and the two kernel bodies
// (FluxGNN.forward on B chains; the persistent hybrid rollout) written once
// over a precision "core" that supplies the GNN forward.
//
// Layout conventions shared by every core (one wave = 16*MT cells of one IC):
//   A 16x16 MFMA accumulator tile of a transposed GEMM Out^T = W X^T holds, in
//   lane l, features n = 16*nt + 4*(l>>4) + r (r = 0..3) of one cell per lane
//   column j = l&15.  The MT m-tiles are INTERLEAVED along the chain: tile mt,
//   column j holds cell MT*j + mt (cell_of).  The chain neighbours of a cell
//   are then the same lane of the adjacent tile, except across the tile-0 /
//   tile-(MT-1) seam, where they are one lane over: row_ror:1 / row_ror:15 of
//   that tile, which is also exactly the periodic wrap.  The neighbour mean
//   therefore costs one VALU per value (a plain add, or an add with a DPP
//   operand) instead of a shift, two seam patches and the add.
//
// Weight ring: a workgroup is 4 waves (4 ICs or windows, one per SIMD) that
// consume the same packed weight stream in lockstep.  The stream is a list of
// equal chunks staged through a 4-slot LDS ring by global_load_lds (LDS-DMA,
// no registers in flight): chunk p+2 is issued while chunk p feeds the MFMAs,
// each wave moving a quarter of every chunk.  Per chunk: counted vmcnt for the
// wave's own DMA, one s_barrier, issue p+2, ds_read_b128 the fragments.
#pragma once

#include "hf_device.h"
#include "hf_internal.h"


namespace hf {
namespace chain {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// GFX9 DPP controls.
constexpr int kRowShl1 = 0x101;
constexpr int kRowShl15 = 0x10F;
constexpr int kRowShr1 = 0x111;
constexpr int kRowShr15 = 0x11F;
constexpr int kRowRor1 = 0x121;
constexpr int kRowRor15 = 0x12F;

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
// Lanes whose DPP source falls outside their row keep `old`.
template <int CTRL>
__device__ __forceinline__ float dpp_over(float old, float v) {
  return __int_as_float(
      __builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Lanes read the DPP source without masking (row rotations have no
// out-of-row lanes), so the mov folds into a consuming VALU op as its DPP operand.
template <int CTRL>
__device__ __forceinline__ float dpp_zero(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}

// Cell held by column j of m-tile mt (interleaved layout, see above).
template <int MT>
__device__ __forceinline__ int cell_of(int mt, int j) { return MT * j + mt; }

// Value of cell m+1 for every lane (periodic over the 16*MT cells of the wave).
template <int MT>
__device__ __forceinline__ void right_nb(const float (&v)[MT], float (&r)[MT]) {
#pragma unroll
  for (int mt = 0; mt < MT - 1; ++mt) r[mt] = v[mt + 1];
  r[MT - 1] = dpp_zero<kRowRor15>(v[0]);  // cell MT*j + MT = MT*(j+1) + 0
}
// Value of cell m-1 for every lane.
template <int MT>
__device__ __forceinline__ void left_nb(const float (&v)[MT], float (&l)[MT]) {
  l[0] = dpp_zero<kRowRor1>(v[MT - 1]);  // cell MT*j - 1 = MT*(j-1) + MT-1
#pragma unroll
  for (int mt = 1; mt < MT; ++mt) l[mt] = v[mt - 1];
}

// v[i+1] + v[i-1] for every cell, one VALU per value: a single fp32 add of the
// two neighbours, bit-identical to the two-term sum the reference's
// index_add_ forms (src/flux_gnn.py:57; fp add is commutative).
template <int MT>
__device__ __forceinline__ void nb_sum(const float (&v)[MT], float (&s)[MT]) {
  float l[MT], r[MT];
  left_nb<MT>(v, l);
  right_nb<MT>(v, r);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    // the rotated (DPP) operand first: hipcc folds a row_ror mov into the add
    // only as src0.  (It still canonicalises the row_ror:15 add with the mov as
    // src1, where it does not fold: one extra VALU per seam value.  Writing the
    // DPP add as inline asm is NOT safe: hipcc then may reuse a VGPR an
    // in-flight MFMA still reads as the asm's destination.)
    if (mt == MT - 1 && MT > 1) s[mt] = __fadd_rn(r[mt], l[mt]);
    else s[mt] = __fadd_rn(l[mt], r[mt]);
  }
}

// Workgroup barrier that also orders this wave's LDS traffic.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ f4 relu4(f4 v) { return f4{relu(v.x), relu(v.y), relu(v.z), relu(v.w)}; }

__device__ __forceinline__ f4 ldf4(const float *p) { return *reinterpret_cast<const f4 *>(p); }

// Orders this wave's LDS traffic (the compiler may otherwise reorder a ds_read
// of another lane's word above the ds_write that produced it).
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// ------------------------------------------------------------------ LDS plan
constexpr int kWaves = 4;  // one IC (item) per wave
constexpr int kRingSlots = 4;

// --------------------------------------------------------- cell-split waves
// An IC of 16*W cells spread over W waves, 16 consecutive cells per wave
// (MT = 1, lane column j = cell 16*pos + j).  The chain neighbours that fall
// off a wave's 16 lanes come from the adjacent waves' boundary columns,
// exchanged through LDS once per layer (chain_rollout_cells_kernel, chain_f32.hip).
struct NoHalo {
  static constexpr bool kOn = false, kSecond = false;
};
// The readout's data gradient as a layer pass (chain_train_bwd_kernel): the
// B operand's second half (k-steps 32..63) is dQ itself, not a neighbour sum
// of the first half's array (which holds dP).
template <int MT>
struct SecondHalf {
  static constexpr bool kOn = false, kSecond = true;
  f4 q[MT][kNT];
};
struct CellHalo {
  static constexpr bool kOn = true, kSecond = false;
  f4 l[kNT], r[kNT];  // the lane's 32 features at cell 16*pos - 1 (lanes j=0) / 16*pos + 16 (lanes j=15)
  f4 *xh;             // [parity 2][wave 4][side 2][g 4][nt 8]: boundary columns of h
  f4 *xq;             // [wave 4][ot 8][P|Q 2][g 4]: column j=0 of the readout accumulators
  int wave, lw, rw, lane, par;
  // Publish this wave's boundary columns of h (j = 0: side 0, j = 15: side 1).
  __device__ __forceinline__ void publish(const f4 (&h)[1][kNT]) {
    f4 *b = xh + par * (kWaves * 2 * 4 * kNT);
    const int j = lane & 15, g = lane >> 4;
    if (j == 0 || j == 15) {
      const int side = j == 15;
#pragma unroll
      for (int nt = 0; nt < kNT; ++nt) b[((wave * 2 + side) * 4 + g) * kNT + nt] = h[0][nt];
    }
  }
  // After a workgroup barrier that follows every wave's publish(): the left
  // wave's side 1 and the right wave's side 0.  (The buffer alternates by
  // parity, so the next publish never overwrites columns still being read.)
  __device__ __forceinline__ void read() {
    const f4 *b = xh + par * (kWaves * 2 * 4 * kNT);
    const int g = lane >> 4;
#pragma unroll
    for (int nt = 0; nt < kNT; ++nt) {
      l[nt] = b[((lw * 2 + 1) * 4 + g) * kNT + nt];
      r[nt] = b[((rw * 2 + 0) * 4 + g) * kNT + nt];
    }
    par ^= 1;
  }
  __device__ __forceinline__ void exchange(const f4 (&h)[1][kNT]) {
    publish(h);
    lds_barrier();
    read();
  }
};

// Activation tape of the fused training forward (chain_train_fwd_kernel): the
// core stores h[l] and the readout's P (+ b_e) / Q in the row-major layout the
// backward GEMMs read (train_chain.hip ChainTape: h[l][row][feature],
// pq[row][P | Q]).  A lane holds features 16nt + 4g ..+3 of one cell per tile:
// one float4 store each.  h[l] is stored while it is the B operand of the
// next pass, one tile every other k-step (put_tile), not as a burst after the
// ReLU: every wave reaches the end of a layer at about the same time, and 32
// stores per lane at once stall the matrix pipe on the memory queue.
struct NoTape {
  static constexpr bool kOn = false;
};
// Row-major [N][kH] arrays, one per layer (h[l], or the backward's g[l]),
// written tile by tile from the lane layout.
struct TileStore {
  float *base;     // array 0; array l = base + l * stride
  int64_t stride;  // floats between the arrays
  int64_t row0;    // row of cell 0 of the wave's IC (b * nx)
  bool live;       // idle waves (mirroring a real IC) store nothing
  template <int MT>
  __device__ __forceinline__ void put(int l, const f4 &v, int mt, int nt, int lane) const {
    if (!live) return;
    // one lane base per array; tile (mt, nt) at a constant offset (cell_of(mt, j) = MT j + mt),
    // so the stores carry immediate offsets instead of 32 live addresses
    float *p = base + l * stride + (row0 + MT * (lane & 15)) * kH + 4 * (lane >> 4);
    *reinterpret_cast<f4 *>(p + mt * kH + 16 * nt) = v;
  }
  template <int MT, int IDX>
  __device__ __forceinline__ void put_tile(int l, const f4 (&h)[MT][kNT], int lane) const {
    put<MT>(l, h[IDX / kNT][IDX % kNT], IDX / kNT, IDX % kNT, lane);
  }
  template <int MT, int NT>
  __device__ __forceinline__ void put_col(int l, const f4 (&h)[MT][kNT], int lane) const {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) put<MT>(l, h[mt][NT], mt, NT, lane);
  }
  template <int MT>
  __device__ __forceinline__ void put_all(int l, const f4 (&h)[MT][kNT], int lane) const {
    put_col<MT, 0>(l, h, lane), put_col<MT, 1>(l, h, lane), put_col<MT, 2>(l, h, lane), put_col<MT, 3>(l, h, lane);
    put_col<MT, 4>(l, h, lane), put_col<MT, 5>(l, h, lane), put_col<MT, 6>(l, h, lane), put_col<MT, 7>(l, h, lane);
  }
};
struct TrainTape : TileStore {
  static constexpr bool kOn = true;
  float *pq;  // [N][2H]
  // ReLU'(h[l]) = h[l] > 0 of layers l <= L as bits in the lanes' own layout
  // (chain_train_bwd_kernel reads them back): word [l][b][mt][lane], bit 4nt + r
  unsigned *mbits;
  int64_t mstride;  // words per layer (B * MT * 64)
  int64_t mrow;     // b * MT * 64
  int layers;
  template <int MT>
  __device__ __forceinline__ void put_mask(int l, const f4 (&h)[MT][kNT], int lane) const {
    if (!live || l > layers) return;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      unsigned m = 0;
#pragma unroll
      for (int nt = 0; nt < kNT; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) m |= (h[mt][nt][r] > 0.f ? 1u : 0u) << (4 * nt + r);
      mbits[l * mstride + mrow + mt * 64 + lane] = m;
    }
  }
  template <int MT>
  __device__ __forceinline__ void put_pq(int ot, const f4 (&P)[MT], const f4 (&Q)[MT], int lane) const {
    if (!live) return;
    float *p = pq + row0 * 2 * kH + 16 * ot + 4 * (lane >> 4);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      float *r = p + (int64_t)cell_of<MT>(mt, lane & 15) * 2 * kH;
      *reinterpret_cast<f4 *>(r) = P[mt];
      *reinterpret_cast<f4 *>(r + kH) = Q[mt];
    }
  }
};
// The backward pass's tile stores of g[l+1] while it feeds layer l (g[L] is
// the pass's input, already in memory: not stored again).
struct GradTape : TileStore {
  static constexpr bool kOn = true;
};

// v[i-1] + v[i+1] for a cell-split wave: row shifts, with the lane that falls
// off the row taking the halo value.  The same single fp32 add as nb_sum.
__device__ __forceinline__ float nb_sum_halo(float v, float hl, float hr) {
  return __fadd_rn(dpp_over<kRowShr1>(hl, v), dpp_over<kRowShl1>(hr, v));
}

constexpr int kSmallFloats = 512 + kH * (3 + kMaxChainLayers);  // win, bin, be, w2, bl[L]
// per wave (floats): n,u,E,x | F | classical twin n,u,E | its F | rho, twin rho
// (64 doubles each) | the Poisson column twice (128 doubles, poisson_cell_nx)
constexpr int kWaveScratchFloats = 4 * 64 + 64 + 3 * 64 + 64 + 2 * 128 + 256;
constexpr int kScrF = 4 * 64, kScrCl = 5 * 64, kScrFc = 8 * 64, kScrRho = 9 * 64, kScrRhoC = 11 * 64, kScrC2 = 13 * 64;
static_assert(kScrC2 + 256 == kWaveScratchFloats, "per-wave scratch layout");

struct Small {  // LDS copies of the small weight arrays
  const float *win, *bin, *bl, *be, *w2;
};

// Stage the small arrays into LDS (all threads of the workgroup) and return views.
__device__ __forceinline__ Small stage_small(const ChainW &W, float *s) {
  for (int i = threadIdx.x; i < 512; i += blockDim.x) s[i] = W.win[i];
  for (int i = threadIdx.x; i < kH; i += blockDim.x) {
    s[512 + i] = W.bin[i];
    s[512 + kH + i] = W.be[i];
    s[512 + 2 * kH + i] = W.w2[i];
  }
  for (int i = threadIdx.x; i < W.layers * kH; i += blockDim.x) s[512 + 3 * kH + i] = W.bl[i];
  return Small{s, s + 512, s + 512 + 3 * kH, s + 512 + kH, s + 512 + 2 * kH};
}

// ----------------------------------------------------------------- the ring
// CF = chunk size in floats (2048 = 8 KiB or 4096 = 16 KiB); NW = waves sharing
// the ring; D = chunks in flight ahead of the one being consumed (the LDS-DMA
// fill latency, ~1.1 us from issue to landing, must fit in D chunk times);
// SLOTS = LDS slots, at least D + 1: at next() every wave has passed the
// barrier with its reads of chunk pos-1 retired, so pos+D may take that slot
// (D = 2 in 3 or 4 slots for the IC-per-wave kernels; 4 slots keep the slot
// arithmetic a mask).
// DEFER: next() only waits and barriers; the DMA it owes (chunk pos+D into the
// slot just released) is issued by issue_pending() at a point the core picks.
// LOADER: the NW waves only consume; one extra wave of the workgroup (wave NW)
// issues every piece of every chunk (loader_prime / loader_next), so the
// compute waves' instruction streams carry no DMA issue (~60 cycles per 1 KiB
// piece beside the MFMAs, MI355X_MICROARCH.md).  A consumer's next() is then
// only its LDS wait + the barrier; the loader waits for its own DMA of the
// chunk before the same barrier.
template <int CF, int NW = kWaves, int SLOTS = kRingSlots, int D = 2, bool DEFER = false, bool LOADER = false>
struct Ring {
  static_assert(SLOTS >= D + 1 && D >= 2 && D <= 6, "ring slots / prefetch distance");
  static_assert(!(LOADER && DEFER), "a loader ring issues at its own barrier");
  static constexpr bool kLoader = LOADER;
  static constexpr int kPerWave = CF / (NW * 256);  // 1 KiB DMA instructions per wave per chunk
  static constexpr int kPieces = CF / 256;          // 1 KiB DMA instructions per chunk (the loader's share)
  static_assert(kPerWave == 1 || kPerWave == 2 || kPerWave == 4, "ring chunk split over the waves");
  __amdgpu_buffer_rsrc_t rsrc;  // packed weight stream (global)
  int lane_off;                 // lane * 16 bytes (the only per-lane address term)
  float *lds;                   // SLOTS slots
  int chunks;        // chunks per forward pass
  int wave, lane;
  int pos;           // stream position being consumed
  int rd;            // its slot (pos % SLOTS)
  int ahead;         // chunk id of stream position pos + D
  int pend_chunk, pend_slot;  // DEFER: the DMA owed since the last next()

  // The DMA is issued from inline asm, hidden from hipcc's s_waitcnt
  // bookkeeping: with a visible LDS-DMA in the kernel hipcc gives every
  // ds_read an lgkmcnt(0) wait, which serialises the fragment prefetch.  The
  // ring's own counted vmcnt + barrier in next() order the DMA for readers.
  // buffer_load ... lds: the chunk offset is an SGPR (soffset), the lane
  // offset a fixed VGPR, so an issue costs no VALU address arithmetic.
  __device__ __forceinline__ void issue(int chunk, int slot, int j0 = 0, int j1 = kPerWave, bool all = false) const {
    const unsigned d = (unsigned)(uintptr_t)(lds_void *)(lds + slot * CF);
#pragma unroll
    for (int jj = j0; jj < j1; ++jj) {
      const int j = all ? jj : kPerWave * wave + jj;  // this wave's share of the chunk (the loader: all of it)
      const unsigned dst = __builtin_amdgcn_readfirstlane(d + j * 1024);
      const unsigned soff = __builtin_amdgcn_readfirstlane((unsigned)(chunk * CF + j * 256) * 4u);
      unsigned keep;
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
          "buffer_load_dwordx4 %1, %3, %4 offen lds\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(lane_off), "s"(dst), "s"(rsrc), "s"(soff)
          : "memory");
    }
  }
  // Start the stream at chunk `first` (chunks first .. first+D-1 in flight).
  __device__ __forceinline__ void prime(int first = 0) {
    pos = 0;
    rd = 0;
    if constexpr (!LOADER) {
#pragma unroll
      for (int i = 0; i < D; ++i) issue((first + i) % chunks, i);
    }
    ahead = (first + D) % chunks;
  }
  // LOADER: the loader wave's counterparts of prime() and next(), one call per
  // consumer call, in the same order (and one lds_barrier() per consumer
  // barrier outside the ring).
  __device__ __forceinline__ void loader_prime(int first = 0) {
    static_assert(LOADER, "loader ring only");
    pos = 0;
    rd = 0;
#pragma unroll
    for (int i = 0; i < D; ++i) issue((first + i) % chunks, i, 0, kPieces, true);
    ahead = (first + D) % chunks;
  }
  __device__ __forceinline__ void loader_next() {
    static_assert(LOADER, "loader ring only");
    constexpr int kVm = kPieces * (D - 1);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (kVm == 8) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
    else if constexpr (kVm == 16) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
    else if constexpr (kVm == 24) asm volatile("s_waitcnt vmcnt(24)\n\ts_barrier" ::: "memory");
    else if constexpr (kVm == 32) asm volatile("s_waitcnt vmcnt(32)\n\ts_barrier" ::: "memory");
    else if constexpr (kVm == 40) asm volatile("s_waitcnt vmcnt(40)\n\ts_barrier" ::: "memory");
    else static_assert(kVm == 8, "vmcnt of the loader ring");
    __builtin_amdgcn_sched_barrier(0);
    issue(ahead, rd + D >= SLOTS ? rd + D - SLOTS : rd + D, 0, kPieces, true);
    ahead = ahead + 1 == chunks ? 0 : ahead + 1;
    rd = rd + 1 == SLOTS ? 0 : rd + 1;
    ++pos;
  }
  // Wait for chunk `pos`, keep D chunks in flight, return its slot.
  __device__ __forceinline__ const float *next() {
    // own DMA for `pos` done (only the D-1 later chunks' instructions may
    // remain), every ds_read of this wave retired, then every wave has passed:
    // the slot pos+D is about to overwrite (pos-1's or an older one) is no
    // longer read by anyone.  sched_barrier(0) on both sides: the compiler may
    // otherwise move register-only MFMAs across the asm, which orders memory
    // operations only.
    __builtin_amdgcn_sched_barrier(0);
#if defined(HF_DIAG_NOSYNC)  // timing diagnostic only: results are wrong (no wait, no barrier, no DMA)
    if (false) {
#elif defined(HF_DIAG_NOBAR)  // timing diagnostic only: results are wrong
    asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
#else
    constexpr int kVm = kPerWave * (D - 1);
    if constexpr (LOADER) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (kVm == 1) asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (kVm == 2) asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (kVm == 3) asm volatile("s_waitcnt vmcnt(3) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (kVm == 4) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (kVm == 5) asm volatile("s_waitcnt vmcnt(5) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (kVm == 6) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (kVm == 8) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (kVm == 10) asm volatile("s_waitcnt vmcnt(10) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else if constexpr (kVm == 12) asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    else static_assert(kVm == 1, "vmcnt of the ring");
#endif
#if defined(HF_DIAG_NOSYNC)
    }
#endif
    __builtin_amdgcn_sched_barrier(0);
#if !defined(HF_DIAG_NODMA) && !defined(HF_DIAG_NOSYNC)  // timing diagnostics only
    if constexpr (LOADER) {
    } else if constexpr (DEFER) {
      pend_chunk = ahead;
      pend_slot = rd + D >= SLOTS ? rd + D - SLOTS : rd + D;
    } else {
      issue(ahead, rd + D >= SLOTS ? rd + D - SLOTS : rd + D);
    }
#endif
    ahead = ahead + 1 == chunks ? 0 : ahead + 1;
    const float *slot = lds + rd * CF;
    rd = rd + 1 == SLOTS ? 0 : rd + 1;
    ++pos;
    return slot;
  }
  // DEFER: issue the DMA the last next() owes (before the next next()).
  __device__ __forceinline__ void issue_pending(int j0 = 0, int j1 = kPerWave) const {
#if !defined(HF_DIAG_NODMA) && !defined(HF_DIAG_NOSYNC)
    if constexpr (DEFER) issue(pend_chunk, pend_slot, j0, j1);
#endif
  }
  __device__ __forceinline__ void drain() const { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
};

template <class Core>
__device__ __forceinline__ typename Core::R_t make_ring(const ChainW &W, float *ring_lds) {
  typename Core::R_t R;
  // the packed stream is chain_chunks() chunks of chain_chunk_bytes(); a core may move it in larger chunks
  R.chunks = chain_chunks(W.layers, W.prec) * chain_chunk_bytes(W.prec) / (Core::kChunkFloats * 4);
  R.rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char *>(static_cast<const char *>(W.stream)) + Core::kStreamOffset, 0,
      R.chunks * Core::kChunkFloats * 4, 0x00020000);
  R.lane_off = (threadIdx.x & 63) * 16;
  R.lds = ring_lds;
  R.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  R.lane = threadIdx.x & 63;
  R.pos = 0;
  R.rd = 0;
  R.ahead = 0;
  return R;
}

// LDS per workgroup: ring | small weights | per-wave scratch (rollouts only) |
// per-wave park (Core::kParkFloats: activations a core spills to LDS instead of VGPRs).
template <class Core, bool SCRATCH = true>
constexpr int lds_floats() {
  return Core::kSlots * Core::kChunkFloats + kSmallFloats +
         Core::kNW * ((SCRATCH ? kWaveScratchFloats : 0) + Core::kParkFloats);
}
template <class Core, bool SCRATCH = true>
__device__ __forceinline__ float *park_of(float *lds, int wave) {
  return lds + Core::kSlots * Core::kChunkFloats + kSmallFloats + (SCRATCH ? Core::kNW * kWaveScratchFloats : 0) +
         wave * Core::kParkFloats;
}

// Row R of the readout epilogue for one output tile ot: z_fwd(i) = P(i)+b + Q(i+1),
// z_bwd(i) = P(i+1)+b + Q(i); flux partial += w2 . ReLU(z)     (src/flux_gnn.py:62-66)
// BIASED: b_e is already in P (the C operand of P's first MFMA).
template <int MT, int R, bool BIASED = false>
__device__ __forceinline__ void readout_row(const f4 (&P)[MT], const f4 (&Q)[MT], const f4 be, const f4 w2,
                                            float (&pf)[MT], float (&pb)[MT]) {
  float pv[MT], qv[MT], pr[MT], qr[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    pv[mt] = BIASED ? P[mt][R] : __fadd_rn(P[mt][R], be[R]);
    qv[mt] = Q[mt][R];
  }
  right_nb<MT>(pv, pr);
  right_nb<MT>(qv, qr);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    pf[mt] = fmaf(w2[R], relu(__fadd_rn(pv[mt], qr[mt])), pf[mt]);
    pb[mt] = fmaf(w2[R], relu(__fadd_rn(pr[mt], qv[mt])), pb[mt]);
  }
}
// Row R of the readout epilogue on a cell-split wave (MT = 1, b_e in P):
// P(i+1) and Q(i+1) of lane j = 15 come from the right wave (prh, qrh).
template <int R>
__device__ __forceinline__ void readout_row_halo(const f4 &P, const f4 &Q, const f4 &prh, const f4 &qrh, const f4 w2,
                                                 float &pf, float &pb) {
  const float pv = P[R], qv = Q[R];
  const float pr = dpp_over<kRowShl1>(prh[R], pv), qr = dpp_over<kRowShl1>(qrh[R], qv);
  pf = fmaf(w2[R], relu(__fadd_rn(pv, qr)), pf);
  pb = fmaf(w2[R], relu(__fadd_rn(pr, qv)), pb);
}
// The whole epilogue of one tile: rows 0..3 in order.
template <int MT, bool BIASED = false>
__device__ __forceinline__ void readout_epilogue(const f4 (&P)[MT], const f4 (&Q)[MT], const f4 be, const f4 w2,
                                                 float (&pf)[MT], float (&pb)[MT]) {
#ifdef HF_DIAG_NOEPI  // timing diagnostic only: results are wrong (one add per value instead of the epilogue)
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) pf[mt] += P[mt][0] + P[mt][1] + P[mt][2] + P[mt][3], pb[mt] += Q[mt][0] + Q[mt][1] + Q[mt][2] + Q[mt][3];
  return;
#endif
  readout_row<MT, 0, BIASED>(P, Q, be, w2, pf, pb);
  readout_row<MT, 1, BIASED>(P, Q, be, w2, pf, pb);
  readout_row<MT, 2, BIASED>(P, Q, be, w2, pf, pb);
  readout_row<MT, 3, BIASED>(P, Q, be, w2, pf, pb);
}

// v[l] + v[l ^ 16] on every lane, by a VALU row swap (v_permlane16_swap:
// rows 1, 3 of the first operand trade places with rows 0, 2 of the second)
// instead of an LDS ds_bpermute; fp addition commutes, so the sum is the same
// bits as v + __shfl_xor(v, 16).
__device__ __forceinline__ float add_xor16(float v) {
  const unsigned u = __float_as_uint(v);
  const auto s = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}
// v[l] + v[l ^ 32] (v_permlane32_swap: upper half of the first operand
// against the lower half of the second).
__device__ __forceinline__ float add_xor32(float v) {
  const unsigned u = __float_as_uint(v);
  const auto s = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}

// The 128-feature dot product is split over the 4 lane groups of a column.
template <int MT>
__device__ __forceinline__ void readout_finish(float (&pf)[MT], float (&pb)[MT], float b2, float (&ffwd)[MT],
                                               float (&fbwd)[MT]) {
#ifdef HF_DIAG_NOFINISH  // timing diagnostic only: results are wrong (no cross-lane sums)
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) ffwd[mt] = pf[mt] + b2, fbwd[mt] = pb[mt] + b2;
  return;
#endif
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    pf[mt] = add_xor32(add_xor16(pf[mt]));
    pb[mt] = add_xor32(add_xor16(pb[mt]));
    ffwd[mt] = pf[mt] + b2;
    fbwd[mt] = pb[mt] + b2;
  }
}

// Input MLP: h0 = ReLU(W_in x + b_in), K = 4 = one f32 MFMA per tile  (src/flux_gnn.py:49)
template <int MT>
__device__ __forceinline__ void input_layer(const Small &S, int lane, const float (&feat)[MT], f4 (&h)[MT][kNT]) {
  const int g4 = 4 * (lane >> 4);
  const f4 a0 = ldf4(S.win + lane * 4), a1 = ldf4(S.win + 256 + lane * 4);
#pragma unroll
  for (int nt = 0; nt < kNT; ++nt) {
    const f4 bias = ldf4(S.bin + 16 * nt + g4);
    const float a = nt < 4 ? a0[nt & 3] : a1[nt & 3];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) h[mt][nt] = relu4(mfma4(a, feat[mt], bias));
  }
}

// ---------------------------------------------------------------------------
// FluxGNN.forward on B chains; items = (IC, window), one wave per item,
// Core::kNW items per workgroup.
//  EXACT: nx == 16*MT, the wave owns the whole periodic IC, every face exact.
//  else : window of 16*MT cells starting at w*(16MT-1-2L)-L (mod nx); faces
//         [L, 16MT-2-L] of the window (16MT - 1 - 2L per window, L = update
//         layers) are exact, the rest discarded.
template <class Core, int MT, bool EXACT>
__global__ __launch_bounds__(64 * Core::kNW, Core::kWGPerCU) void chain_flux_kernel(ChainW W, const float *__restrict__ nf,
                                                            const float *__restrict__ state,
                                                            int64_t ld_state,
                                                            const float *__restrict__ x, int nx,
                                                            int nwin, int64_t items,
                                                            float *__restrict__ fe,
                                                            float *__restrict__ ff) {
  constexpr int kRingFloats = Core::kSlots * Core::kChunkFloats;
  __shared__ f4 lds4[lds_floats<Core, false>() / 4];
  float *lds = reinterpret_cast<float *>(lds4);
  const Small S = stage_small(W, lds + kRingFloats);
  auto R = make_ring<Core>(W, lds);
  const int lane = R.lane, j = lane & 15, g = lane >> 4;
  __syncthreads();  // small weights staged (no DMA in flight yet)
  R.prime();
  typename Core::Feed F;
  Core::begin(R, F);
  // Persistent over groups of 4 items: the weight stream keeps flowing from one
  // group's forward pass into the next, so the ring fill is paid once per workgroup.
  // window halo: after L message-passing layers the L cells at each window
  // edge (and the readout of the faces between them) have seen the window's
  // artificial wrap; faces [L, 62 - L] of a 64-cell window are exact
  const int halo = W.layers, win_faces = win_faces_of(W.layers, 16 * MT);
  const int64_t groups = (items + Core::kNW - 1) / Core::kNW;
  // item (IC b, window w) of this wave in group grp; idle waves mirror a real item and write nothing
  auto locate = [&](int64_t grp, int64_t &b, int &w) {
    const int64_t item_raw = grp * Core::kNW + R.wave;
    const int64_t item = item_raw < items ? item_raw : items - 1;
    b = item / nwin;
    w = (int)(item - b * nwin);
    return item_raw < items;
  };
  auto cell_at = [&](int w, int mt) {
    int cidx = ((EXACT ? 0 : w * win_faces - halo) + cell_of<MT>(mt, j)) % nx;
    return cidx < 0 ? cidx + nx : cidx;
  };
  // node features of group grp: n, u, E, x of the wave's 16*MT cells (lane group g = feature g)
  auto load_feat = [&](int64_t grp, float (&feat)[MT]) {
    int64_t b;
    int w;
    locate(grp, b, w);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int cidx = cell_at(w, mt);
#ifdef HF_DIAG_NOFEAT  // timing diagnostic only: results are wrong (no feature loads, no flux stores)
      feat[mt] = 0.01f * (float)(cidx + g);
#else
      feat[mt] = nf ? nf[(b * nx + cidx) * kIn + g]
                    : (g < 3 ? state[b * ld_state + (int64_t)g * nx + cidx] : x[cidx]);
#endif
    }
  };
  // The next group's features are loaded while this group's forward runs.
  float pre[MT];
  if (blockIdx.x < groups) load_feat(blockIdx.x, pre);
  for (int64_t grp = blockIdx.x; grp < groups; grp += gridDim.x) {
    float feat[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) feat[mt] = pre[mt];
    if (grp + gridDim.x < groups) load_feat(grp + gridDim.x, pre);
    float f_fwd[MT], f_bwd[MT];
    Core::template gnn<MT>(W, S, R, F, park_of<Core, false>(lds, R.wave), feat, f_fwd, f_bwd);
    int64_t b;
    int w;
    const bool live = locate(grp, b, w);
#ifdef HF_DIAG_NOFEAT
    if (live && f_fwd[0] == 12345.f) {  // keeps the forward live; never true in practice
#else
    if (live) {
#endif
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int wc = cell_of<MT>(mt, j);
        int face = cell_at(w, mt);
        bool ok = true;
        if (!EXACT) {
          face = w * win_faces + (wc - halo);
          ok = wc >= halo && wc < halo + win_faces && face < nx;
        }
        if (!ok) continue;
        if (fe && g == 0) fe[b * 2 * nx + face] = f_fwd[mt];
        if (fe && g == 1) fe[b * 2 * nx + nx + face] = f_bwd[mt];
        if (ff && g == 2) ff[b * nx + face] = face_flux(f_fwd[mt], f_bwd[mt]);
      }
    }
  }
  R.drain();
}

// ---------------------------------------------------------------------------
// Fused training forward (FluxGNN.forward under autograd on tagged chains of
// nx = 16*MT cells, train_chain.hip launch_chain_forward_train): the flux
// kernel's IC-per-wave pass plus the activation tape (TrainTape) the backward
// GEMMs read.  W comes from pack_chain_f32_kernel (the parameters change every
// optimizer step); b2 is read from the device (*b2p).
template <class Core, int MT>
__global__ __launch_bounds__(64 * Core::kNW, Core::kWGPerCU) void chain_train_fwd_kernel(
    ChainW W, const float *__restrict__ b2p, const float *__restrict__ nf, int64_t items, float *__restrict__ fe,
    float *h0, int64_t hstride, float *pq, unsigned *mbits) {
  constexpr int nx = 16 * MT;
  constexpr int kRingFloats = Core::kSlots * Core::kChunkFloats;
  __shared__ f4 lds4[lds_floats<Core, false>() / 4];
  float *lds = reinterpret_cast<float *>(lds4);
  W.b2 = *b2p;
  const Small S = stage_small(W, lds + kRingFloats);
  auto R = make_ring<Core>(W, lds);
  const int lane = R.lane, j = lane & 15, g = lane >> 4;
  __syncthreads();
  R.prime();
  typename Core::Feed F;
  Core::begin(R, F);
  const int64_t groups = (items + Core::kNW - 1) / Core::kNW;
  auto load_feat = [&](int64_t grp, float (&feat)[MT]) {
    const int64_t item_raw = grp * Core::kNW + R.wave;
    const int64_t b = item_raw < items ? item_raw : items - 1;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) feat[mt] = nf[(b * nx + cell_of<MT>(mt, j)) * kIn + g];
  };
  float pre[MT];
  if (blockIdx.x < groups) load_feat(blockIdx.x, pre);
  for (int64_t grp = blockIdx.x; grp < groups; grp += gridDim.x) {
    float feat[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) feat[mt] = pre[mt];
    if (grp + gridDim.x < groups) load_feat(grp + gridDim.x, pre);
    const int64_t item_raw = grp * Core::kNW + R.wave;
    const bool live = item_raw < items;
    const int64_t b = live ? item_raw : items - 1;
    TrainTape T;
    T.base = h0, T.stride = hstride, T.row0 = b * nx, T.live = live;
    T.pq = pq, T.mbits = mbits, T.mstride = items * MT * 64, T.mrow = b * MT * 64, T.layers = W.layers;
    float f_fwd[MT], f_bwd[MT];
    Core::template gnn_tape<MT>(W, S, R, F, feat, f_fwd, f_bwd, T);
    if (live) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int face = cell_of<MT>(mt, j);
        if (g == 0) fe[b * 2 * nx + face] = f_fwd[mt];
        if (g == 1) fe[b * 2 * nx + nx + face] = f_bwd[mt];
      }
    }
  }
  R.drain();
}

// The readout's backward in the backward pass (train_chain.hip
// launch_chain_backward, fused path): from the forward's P/Q tape (P = W_a h +
// b_e, Q = W_b h, [N][P | Q]) and the flux gradient g ([B][2nx]: g_f, g_b),
// with z_f(i) = P_i + Q_{i+1}, z_b(i) = P_{i+1} + Q_i (src/flux_gnn.py:62-66),
//   dP_i = g_f(i) w2 [z_f(i) > 0] + g_b(i-1) w2 [z_b(i-1) > 0]
//   dQ_i = g_b(i) w2 [z_b(i) > 0] + g_f(i-1) w2 [z_f(i-1) > 0]
// in the lane layout (neighbours one m-tile over, or a row rotation at the
// seam), the sums and products of edge_backward_kernel bit for bit, stored to
// dpq ([N][dP | dQ], the readout weight gradient's operand and this pass's B
// operand), and this IC's dw2 = sum g_f ReLU(z_f) + g_b ReLU(z_b), db2 = sum
// g_f + g_b to part[b][0..H] (a fixed-order row reduction).  Replaces the
// separate edge_backward_h128_kernel pass over P/Q and dP/dQ.
#ifndef HF_TRAIN_EDGE_FOLD  // (train_chain.hip: measured and not kept; default off)
#define HF_TRAIN_EDGE_FOLD 0
#endif
struct EdgeFold {
  const float *pq;     // nullptr: no fold (the pass reads dpq as written by the edge kernel)
  const float *gflux;  // [B][2nx]
  const float *w2;     // [kH]
  float *dpq;          // [N][2 kH]
  float *part;         // [B][kH + 1]
};
template <int MT>
__device__ __forceinline__ void edge_fold_ic(const EdgeFold &E, int64_t b, bool live, int lane) {
  constexpr int nx = 16 * MT;
  const int j = lane & 15, g4 = 4 * (lane >> 4);
  const float *src = E.pq + b * nx * 2 * kH + g4;
  float *dst = E.dpq + b * nx * 2 * kH + g4;
  float gf[MT], gb[MT], gfl[MT], gbl[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    gf[mt] = E.gflux[b * 2 * nx + cell_of<MT>(mt, j)];
    gb[mt] = E.gflux[b * 2 * nx + nx + cell_of<MT>(mt, j)];
  }
  left_nb<MT>(gf, gfl);
  left_nb<MT>(gb, gbl);
  float dw[kNT][4];
#pragma unroll
  for (int nt = 0; nt < kNT; ++nt) {
    f4 P4[MT], Q4[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      P4[mt] = ldf4(src + (int64_t)cell_of<MT>(mt, j) * 2 * kH + 16 * nt);
      Q4[mt] = ldf4(src + (int64_t)cell_of<MT>(mt, j) * 2 * kH + kH + 16 * nt);
    }
    const f4 w = ldf4(E.w2 + 16 * nt + g4);
    f4 dP4[MT], dQ4[MT];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float P[MT], Q[MT], Pr[MT], Pl[MT], Qr[MT], Ql[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) P[mt] = P4[mt][r], Q[mt] = Q4[mt][r];
      right_nb<MT>(P, Pr);
      left_nb<MT>(P, Pl);
      right_nb<MT>(Q, Qr);
      left_nb<MT>(Q, Ql);
      float acc = 0.f;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const float zf = __fadd_rn(P[mt], Qr[mt]), zbp = __fadd_rn(P[mt], Ql[mt]);
        const float zb = __fadd_rn(Pr[mt], Q[mt]), zfp = __fadd_rn(Pl[mt], Q[mt]);
        dP4[mt][r] = __fadd_rn(zf > 0.f ? __fmul_rn(gf[mt], w[r]) : 0.f, zbp > 0.f ? __fmul_rn(gbl[mt], w[r]) : 0.f);
        dQ4[mt][r] = __fadd_rn(zb > 0.f ? __fmul_rn(gb[mt], w[r]) : 0.f, zfp > 0.f ? __fmul_rn(gfl[mt], w[r]) : 0.f);
        acc = fmaf(gf[mt], zf > 0.f ? zf : 0.f, acc);
        acc = fmaf(gb[mt], zb > 0.f ? zb : 0.f, acc);
      }
      dw[nt][r] = acc;
    }
    if (live) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        *reinterpret_cast<f4 *>(dst + (int64_t)cell_of<MT>(mt, j) * 2 * kH + 16 * nt) = dP4[mt];
        *reinterpret_cast<f4 *>(dst + (int64_t)cell_of<MT>(mt, j) * 2 * kH + kH + 16 * nt) = dQ4[mt];
      }
    }
  }
  float db = 0.f;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) db = __fadd_rn(db, __fadd_rn(gf[mt], gb[mt]));
  // sums over the row's 16 lanes (its 16 MT cells), in the same order in every lane
  auto row_sum = [](float v) {
    v = __fadd_rn(v, dpp_zero<0x128>(v));  // row_ror:8
    v = __fadd_rn(v, dpp_zero<0x124>(v));  // row_ror:4
    v = __fadd_rn(v, dpp_zero<0x122>(v));  // row_ror:2
    return __fadd_rn(v, dpp_zero<kRowRor1>(v));
  };
#pragma unroll
  for (int nt = 0; nt < kNT; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) dw[nt][r] = row_sum(dw[nt][r]);
  db = row_sum(db);
  if (live && j == 0) {
    float *o = E.part + b * (kH + 1);
#pragma unroll
    for (int nt = 0; nt < kNT; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[16 * nt + g4 + r] = dw[nt][r];
    if (g4 == 0) o[kH] = db;
  }
  __threadfence_block();  // this wave's dP / dQ stores complete before it reads them back
}

// Fused data gradient of the update layers (train_chain.hip
// launch_chain_backward): from g[L] = ReLU'(h[L]) * dh[L] (the readout's
// gradient, global) to g[l] = ReLU'(h[l]) * (W_a^T g[l+1] + W_b^T agg g[l+1])
// for l = L-1 .. 0 (the aggregation is self-adjoint on the periodic chain),
// one IC per wave through the flux kernel's layer pass: the same [x ; agg x]
// B operand from registers, the transposed weights streamed through the ring
// (pack_chain_bwd_f32_kernel), the ReLU' bits the forward stored
// (TrainTape::mbits).  g[l] = g0 + l * gstride, [N][H] each.
template <class Core, int MT>
__global__ __launch_bounds__(64 * Core::kNW, Core::kWGPerCU) void chain_train_bwd_kernel(
    ChainW W, int64_t items, float *g0, int64_t gstride, const unsigned *__restrict__ mbits,
    const float *__restrict__ dPQ, EdgeFold EF) {
  constexpr int nx = 16 * MT;
  __shared__ f4 lds4[Core::kSlots * Core::kChunkFloats / 4];
  float *lds = reinterpret_cast<float *>(lds4);
  const int L = W.layers;
  auto R = make_ring<Core>(W, lds);
  R.chunks = 16 * (L + (dPQ ? 1 : 0));  // (the readout's pass,) the update layers
  R.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(W.stream), 0, R.chunks * Core::kChunkFloats * 4,
                                             0x00020000);
  const int lane = R.lane, j = lane & 15, g4 = 4 * (lane >> 4);
  __syncthreads();
  R.prime();
  typename Core::Feed F;
  Core::begin(R, F);
  const int64_t groups = (items + Core::kNW - 1) / Core::kNW, mstride = items * MT * 64;
  for (int64_t grp = blockIdx.x; grp < groups; grp += gridDim.x) {
    const int64_t item_raw = grp * Core::kNW + R.wave;
    const bool live = item_raw < items;
    const int64_t b = live ? item_raw : items - 1;
    GradTape GT;
    GT.base = g0, GT.stride = gstride, GT.row0 = b * nx, GT.live = live;
    f4 g[MT][kNT];
    if (dPQ) {
      // g[L] = ReLU'(h[L]) * (W_a^T dP + W_b^T dQ): a layer pass with B = [dP ; dQ]
#if HF_TRAIN_EDGE_FOLD
      if (EF.pq) edge_fold_ic<MT>(EF, b, live, lane);  // dP / dQ of this IC into dPQ (= EF.dpq) first
#endif
      SecondHalf<MT> X;
      const float *src = dPQ + b * nx * 2 * kH + g4;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < kNT; ++nt) {
          g[mt][nt] = ldf4(src + (int64_t)cell_of<MT>(mt, j) * 2 * kH + 16 * nt);
          X.q[mt][nt] = ldf4(src + (int64_t)cell_of<MT>(mt, j) * 2 * kH + kH + 16 * nt);
        }
      unsigned mb[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) mb[mt] = mbits[L * mstride + b * MT * 64 + mt * 64 + lane];
      f4 acc[MT][kNT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < kNT; ++nt) acc[mt][nt] = f4{0.f, 0.f, 0.f, 0.f};
      float bop[MT];
      Core::template b_operand<MT, 0>(g, bop, X);
      Core::template layer_chunk<MT, 0>(R, F, g, bop, acc, X);
      Core::template layer_chunk<MT, 4>(R, F, g, bop, acc, X);
      Core::template layer_chunk<MT, 8>(R, F, g, bop, acc, X);
      Core::template layer_chunk<MT, 12>(R, F, g, bop, acc, X);
      Core::template layer_chunk<MT, 16>(R, F, g, bop, acc, X);
      Core::template layer_chunk<MT, 20>(R, F, g, bop, acc, X);
      Core::template layer_chunk<MT, 24>(R, F, g, bop, acc, X);
      Core::template layer_chunk<MT, 28>(R, F, g, bop, acc, X);
      Core::template layer_chunk<MT, 32>(R, F, g, bop, acc, X);
      Core::template layer_chunk<MT, 36>(R, F, g, bop, acc, X);
      Core::template layer_chunk<MT, 40>(R, F, g, bop, acc, X);
      Core::template layer_chunk<MT, 44>(R, F, g, bop, acc, X);
      Core::template layer_chunk<MT, 48>(R, F, g, bop, acc, X);
      Core::template layer_chunk<MT, 52>(R, F, g, bop, acc, X);
      Core::template layer_chunk<MT, 56>(R, F, g, bop, acc, X);
      Core::template layer_chunk<MT, 60>(R, F, g, bop, acc, X);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < kNT; ++nt)
#pragma unroll
          for (int r = 0; r < 4; ++r) g[mt][nt][r] = (mb[mt] >> (4 * nt + r)) & 1u ? acc[mt][nt][r] : 0.f;
    } else {
      const float *src = g0 + L * gstride + b * nx * kH + g4;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < kNT; ++nt) g[mt][nt] = ldf4(src + (int64_t)cell_of<MT>(mt, j) * kH + 16 * nt);
    }
    for (int l = L - 1; l >= 0; --l) {
      unsigned mb[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) mb[mt] = mbits[l * mstride + b * MT * 64 + mt * 64 + lane];
      f4 acc[MT][kNT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < kNT; ++nt) acc[mt][nt] = f4{0.f, 0.f, 0.f, 0.f};
      NoHalo X;
      // g[l+1] (the B operand) to memory, spread over the pass (g[L] only when made here)
      const int tl = l + 1 < L || dPQ ? l + 1 : -1;
      float bop[MT];
      Core::template b_operand<MT, 0>(g, bop, X);
      Core::template layer_chunk<MT, 0>(R, F, g, bop, acc, X, GT, tl);
      Core::template layer_chunk<MT, 4>(R, F, g, bop, acc, X, GT, tl);
      Core::template layer_chunk<MT, 8>(R, F, g, bop, acc, X, GT, tl);
      Core::template layer_chunk<MT, 12>(R, F, g, bop, acc, X, GT, tl);
      Core::template layer_chunk<MT, 16>(R, F, g, bop, acc, X, GT, tl);
      Core::template layer_chunk<MT, 20>(R, F, g, bop, acc, X, GT, tl);
      Core::template layer_chunk<MT, 24>(R, F, g, bop, acc, X, GT, tl);
      Core::template layer_chunk<MT, 28>(R, F, g, bop, acc, X, GT, tl);
      Core::template layer_chunk<MT, 32>(R, F, g, bop, acc, X, GT, tl);
      Core::template layer_chunk<MT, 36>(R, F, g, bop, acc, X, GT, tl);
      Core::template layer_chunk<MT, 40>(R, F, g, bop, acc, X, GT, tl);
      Core::template layer_chunk<MT, 44>(R, F, g, bop, acc, X, GT, tl);
      Core::template layer_chunk<MT, 48>(R, F, g, bop, acc, X, GT, tl);
      Core::template layer_chunk<MT, 52>(R, F, g, bop, acc, X, GT, tl);
      Core::template layer_chunk<MT, 56>(R, F, g, bop, acc, X, GT, tl);
      Core::template layer_chunk<MT, 60>(R, F, g, bop, acc, X, GT, tl);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < kNT; ++nt)
#pragma unroll
          for (int r = 0; r < 4; ++r) g[mt][nt][r] = (mb[mt] >> (4 * nt + r)) & 1u ? acc[mt][nt][r] : 0.f;
    }
    GT.template put_all<MT>(0, g, lane);  // g[0]: no pass follows
  }
  R.drain();
}

// ---------------------------------------------------------------------------
// Persistent hybrid rollout, one wave per IC (4 ICs per workgroup), nx = 16*MT:
// T steps of GNN -> symmetrise -> continuity -> Burgers -> spectral Poisson
// with the IC's state in LDS (src/hybrid_solver.py:34-73).  The weight stream
// runs continuously across steps.
template <class Core, int MT>
__global__ __launch_bounds__(256, 1) void chain_rollout_kernel(
    ChainW W, const float *state0, float *state_final,  // may alias (read whole before written)
    const float *__restrict__ x, const double *__restrict__ pc, int B, int T, float c, float dt,
    float *__restrict__ traj, float *__restrict__ flux_traj, float *__restrict__ metrics, RolloutExtras ex) {
  constexpr int NX = 16 * MT;
  constexpr int kRingFloats = Core::kSlots * Core::kChunkFloats;
  __shared__ f4 lds4[lds_floats<Core>() / 4];
  float *lds = reinterpret_cast<float *>(lds4);
  const Small S = stage_small(W, lds + kRingFloats);
  auto R = make_ring<Core>(W, lds);
  const int lane = R.lane, j = lane & 15, g = lane >> 4;
  float *scratch = lds + kRingFloats + kSmallFloats + R.wave * kWaveScratchFloats;
  float *s_st = scratch;  // n | u | E | x   (4 x 64)
  float *s_F = scratch + kScrF;
  double *s_rho = reinterpret_cast<double *>(scratch + kScrRho);
  double *s_c2 = reinterpret_cast<double *>(scratch + kScrC2);
  float *s_cl = scratch + kScrCl;  // classical twin n | u | E
  float *s_Fc = scratch + kScrFc;
  double *s_rhoc = reinterpret_cast<double *>(scratch + kScrRhoC);
  float *park = park_of<Core>(lds, R.wave);
  const bool twin = ex.mse != nullptr;
  static_assert(Core::kNW == kWaves, "rollout: 4 waves, one IC each");
  const int b_raw = blockIdx.x * kWaves + R.wave;
  const bool live = b_raw < B;
  const int64_t b = live ? b_raw : B - 1;
  const float *st0 = state0 + b * 3 * NX;
  for (int i = lane; i < 3 * NX; i += 64) {
    const float v = st0[i];
    s_st[(i / NX) * 64 + i % NX] = v;
    if (twin) s_cl[(i / NX) * 64 + i % NX] = v;
  }
  const bool tri = ex.poisson == HF_POISSON_TRIDIAG;  // plan = {h}: no circulant column
  const double h = tri ? pc[0] : 0.0;
  if (lane < NX) {
    s_st[3 * 64 + lane] = x[lane];
    if (!tri) s_c2[lane] = s_c2[NX + lane] = pc[lane];
  }
  __syncthreads();  // small weights + per-wave state visible (no DMA in flight yet)
  float *tj = (traj && live) ? traj + b * (int64_t)(T + 1) * 3 * NX : nullptr;
  float *mt_out = (metrics && live) ? metrics + b * (int64_t)(T + 1) * HF_NUM_METRICS : nullptr;
  float *mc_out = (ex.metrics_cl && live) ? ex.metrics_cl + b * (int64_t)(T + 1) * HF_NUM_METRICS : nullptr;
  float *mse_out = (twin && live) ? ex.mse + b * (int64_t)(T + 1) * 3 : nullptr;
  float *ftj = (flux_traj && live) ? flux_traj + b * (int64_t)T * NX : nullptr;
  auto emit = [&](int t) {
    if (tj)
      for (int i = lane; i < 3 * NX; i += 64) tj[(int64_t)t * 3 * NX + i] = s_st[(i / NX) * 64 + i % NX];
    if (mt_out) {
      MetricAcc m;
      m.init();
      if (lane < NX) m.add(s_st[lane], s_st[64 + lane], s_st[128 + lane]);
      m.wave_reduce();
      if (lane == 0) m.store(mt_out + t * HF_NUM_METRICS, NX);
    }
    if (mc_out) {
      MetricAcc m;
      m.init();
      if (lane < NX) m.add(s_cl[lane], s_cl[64 + lane], s_cl[128 + lane]);
      m.wave_reduce();
      if (lane == 0) m.store(mc_out + t * HF_NUM_METRICS, NX);
    }
    if (mse_out) {  // scripts/evaluation/evaluate_multi_ic.py:88-90
#pragma unroll
      for (int ch = 0; ch < 3; ++ch) {
        double d2 = 0.0;
        if (lane < NX) {
          const double d = (double)s_st[ch * 64 + lane] - (double)s_cl[ch * 64 + lane];
          d2 = d * d;
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) d2 += __shfl_xor(d2, o, 64);
        if (lane == 0) mse_out[t * 3 + ch] = (float)(d2 / NX);
      }
    }
  };
  emit(0);
  R.prime();
  typename Core::Feed F;
  Core::begin(R, F);
  for (int t = 0; t < T; ++t) {
    float feat[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) feat[mt] = s_st[g * 64 + cell_of<MT>(mt, j)];
    float f_fwd[MT], f_bwd[MT];
    Core::template gnn<MT>(W, S, R, F, park, feat, f_fwd, f_bwd);
    if (g == 0) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) s_F[cell_of<MT>(mt, j)] = face_flux(f_fwd[mt], f_bwd[mt]);
    }
    if (twin && lane < NX) s_Fc[lane] = __fmul_rn(s_cl[lane], s_cl[64 + lane]);  // F_n = n*u
    wave_lds_sync();
    float n_new = 0.f, u_new = 0.f, nc = 0.f, uc = 0.f;
    if (lane < NX) {
      const int im = lane == 0 ? NX - 1 : lane - 1;
      const float F = s_F[lane];
      n_new = continuity(s_st[lane], F, s_F[im], c);
      u_new = velocity_hybrid(s_st[64 + lane], s_st[64 + im], s_st[128 + lane], c, dt);
      s_rho[lane] = (double)__fsub_rn(n_new, 1.0f);
      if (ftj) ftj[(int64_t)t * NX + lane] = F;
      if (twin) {  // BaselineSolver.step (src/baseline_solver.py:80-101)
        const int ip = lane == NX - 1 ? 0 : lane + 1;
        nc = continuity(s_cl[lane], s_Fc[lane], s_Fc[im], c);
        uc = velocity_classical(s_cl[64 + lane], s_cl[64 + im], s_cl[64 + ip], s_cl[128 + lane], c, dt, ex.nu,
                                ex.dx2);
        s_rhoc[lane] = (double)__fsub_rn(nc, 1.0f);
      }
    }
    wave_lds_sync();
    float E_tri = 0.f, Ec_tri = 0.f;
    if (tri) {  // HF_POISSON_TRIDIAG: the wave's cyclic reduction over its rho row(s)
      tridiag_psi_wave<double>(s_rho, NX, lane);
      if (lane < NX) E_tri = (float)tri_E(s_rho, lane, NX, h);
      if (twin) {
        tridiag_psi_wave<double>(s_rhoc, NX, lane);
        if (lane < NX) Ec_tri = (float)tri_E(s_rhoc, lane, NX, h);
      }
    }
    if (lane < NX) {
      const float E_new = tri ? E_tri : poisson_cell_nx<NX>(s_rho, s_c2, lane);
      s_st[lane] = n_new;
      s_st[64 + lane] = u_new;
      s_st[128 + lane] = E_new;
      if (twin) {
        const float Ec = tri ? Ec_tri : poisson_cell_nx<NX>(s_rhoc, s_c2, lane);
        s_cl[lane] = nc;
        s_cl[64 + lane] = uc;
        s_cl[128 + lane] = Ec;
      }
    }
    wave_lds_sync();
    emit(t + 1);
  }
  R.drain();
  if (!live) return;
  float *out = state_final + b * 3 * NX;
  for (int i = lane; i < 3 * NX; i += 64) out[i] = s_st[(i / NX) * 64 + i % NX];
}

// ---------------------------------------------------------------------------
// Cell-split persistent rollout for small batches: an IC of NX = 16*WPI cells
// on WPI waves (16 consecutive cells each; cell core CC: CoreF32 at MT = 1 in
// chain_f32.hip, CellBF16 in chain_bf16.hip, CellF16x3 in chain_k32.hip), 4/WPI ICs per
// workgroup (WPI = 3: one IC and a shadow wave that keeps the weight ring's
// lockstep and writes nothing).  B ICs occupy B*WPI/4 CUs' worth of waves
// instead of B/4, for the same per-cell arithmetic as chain_rollout_kernel:
// every MFMA chain, neighbour sum, readout partial dot and FV/Poisson
// expression is evaluated in the same order, so the results are bit-identical
// to it.  The four waves share the LDS weight ring as in chain_rollout_kernel;
// per layer they swap boundary columns of h (f32) or G (bf16, f16x3) through
// CellHalo, per step column 0 of the readout accumulators.  The IC's first wave does FV + Poisson + outputs
// for all its cells, one per lane (src/hybrid_solver.py:45-63).
constexpr int kXhF4 = 2 * kWaves * 2 * 4 * kNT;  // CellHalo::xh
constexpr int kXqF4 = kWaves * kNT * 2 * 4;      // CellHalo::xq
template <class CC>
constexpr int cells_lds_floats() {
  return CC::kSlots * CC::kChunkFloats + kSmallFloats + kWaves * kWaveScratchFloats + 4 * (kXhF4 + kXqF4);
}

// threads of a cell-split rollout workgroup: 4 compute waves (+ the loader wave)
template <class CC>
constexpr int cells_threads() {
  return 64 * (kWaves + (CC::R_t::kLoader ? 1 : 0));
}

template <class CC, int WPI>
__global__ __launch_bounds__(cells_threads<CC>(), 1) void chain_rollout_cells_kernel(
    ChainW W, const float *state0, float *state_final,  // may alias (read whole before written)
    const float *__restrict__ x,
    const double *__restrict__ pc, int B, int T, float c, float dt, float *__restrict__ traj,
    float *__restrict__ flux_traj, float *__restrict__ metrics, int pm) {
  constexpr int NX = 16 * WPI;
  const bool tri = pm == HF_POISSON_TRIDIAG;  // plan = {h}: no circulant column
  const double h = tri ? pc[0] : 0.0;
  constexpr int IPW = kWaves / WPI;  // ICs per workgroup
  constexpr int kRingFloats = CC::kSlots * CC::kChunkFloats;
  __shared__ f4 lds4[cells_lds_floats<CC>() / 4];
  float *lds = reinterpret_cast<float *>(lds4);
  const Small S = stage_small(W, lds + kRingFloats);
  auto R = make_ring<CC>(W, lds);
  const int wave = R.wave, lane = R.lane, j = lane & 15, g = lane >> 4;
  constexpr bool kLd = CC::R_t::kLoader;
#ifndef HF_LDR_EMIT
#define HF_LDR_EMIT 0
#endif
  // HF_LDR_EMIT=1: the loader wave writes the per-step outputs instead of the
  // lead (measured equal on cfg2, profiles/r02_cfg2_loader_ab.json)
  constexpr bool kLdEmit = kLd && HF_LDR_EMIT;
  const bool shadow = wave >= IPW * WPI;     // (the loader wave, wave kWaves, too)
  const int slot = shadow ? 0 : wave / WPI;  // IC of this wave within the workgroup
  const int pos = shadow ? 0 : wave % WPI;   // cells 16*pos .. 16*pos + 15 of it
  // the lead (FV + Poisson + outputs) is the IC's wave 1 beside a loader
  // wave: the loader shares SIMD 0 with wave 0
  const bool lead = !shadow && pos == (kLd ? 1 : 0);
  CellHalo X;
  X.xh = reinterpret_cast<f4 *>(lds + kRingFloats + kSmallFloats + kWaves * kWaveScratchFloats);
  X.xq = X.xh + kXhF4;
  X.wave = wave;
  X.lane = lane;
  X.par = 0;
  X.lw = shadow ? wave : slot * WPI + (pos + WPI - 1) % WPI;  // periodic chain
  X.rw = shadow ? wave : slot * WPI + (pos + 1) % WPI;
  float *scratch = lds + kRingFloats + kSmallFloats + slot * kWaveScratchFloats;
  float *s_st = scratch;  // n | u | E | x   (4 x 64)
  float *s_F = scratch + kScrF;
  double *s_rho = reinterpret_cast<double *>(scratch + kScrRho);
  double *s_c2 = reinterpret_cast<double *>(scratch + kScrC2);
  const int b_raw = blockIdx.x * IPW + slot;
  const bool live = b_raw < B;
  const int64_t b = live ? b_raw : B - 1;  // a missing IC mirrors the last one and writes nothing
  if (lead) {
    const float *st0 = state0 + b * 3 * NX;
    for (int i = lane; i < 3 * NX; i += 64) s_st[(i / NX) * 64 + i % NX] = st0[i];
    if (lane < NX) {
      s_st[3 * 64 + lane] = x[lane];
      if (!tri) s_c2[lane] = s_c2[NX + lane] = pc[lane];
    }
  }
  __syncthreads();  // small weights + IC state visible (no DMA in flight yet)
  // outputs of state t of IC slot sl: trajectory row and metrics
  auto emit = [&](int sl, int t) {
    const int64_t bs = (int64_t)blockIdx.x * IPW + sl;
    if (bs >= B) return;
    const float *st = lds + kRingFloats + kSmallFloats + sl * kWaveScratchFloats;
    if (traj) {
      float *tj = traj + bs * (int64_t)(T + 1) * 3 * NX + (int64_t)t * 3 * NX;
      for (int i = lane; i < 3 * NX; i += 64) tj[i] = st[(i / NX) * 64 + i % NX];
    }
    if (metrics) {
      MetricAcc m;
      m.init();
      if (lane < NX) m.add(st[lane], st[64 + lane], st[128 + lane]);
      m.wave_reduce();
      if (lane == 0) m.store(metrics + bs * (int64_t)(T + 1) * HF_NUM_METRICS + t * HF_NUM_METRICS, NX);
    }
  };
  if constexpr (kLd) {
    if (wave == kWaves) {  // the loader: the compute waves' ring barriers and step barriers, in order
#ifdef HF_LDR_PRIO  // A/B: the loader's wave priority
      __builtin_amdgcn_s_setprio(HF_LDR_PRIO);
#endif
      R.loader_prime();
      R.loader_next();  // CC::begin
      const int ro_chunks = R.chunks - W.layers * CC::kLayerChunks;
      for (int t = 0; t < T; ++t) {  // one forward pass: update layers, then the readout
        for (int l = 0; l < W.layers; ++l) {
          for (int k = 0; k < CC::kLayerChunks; ++k) {
            R.loader_next();
            // state t is in LDS from the end of step t-1 to this step's FV
            // (after the second step barrier below): its outputs, off the lead's path
            if (kLdEmit && l == 0 && k == 0)
              for (int sl = 0; sl < IPW; ++sl) emit(sl, t);
          }
          if constexpr (CC::kLayerBarrier) lds_barrier();  // the layer's halo trade (CellHalo::exchange)
        }
        for (int k = 0; k < ro_chunks; ++k) R.loader_next();
        lds_barrier();  // the readout's column-0 trade
        lds_barrier();  // face fluxes
        lds_barrier();  // new state
      }
      if (kLdEmit)
        for (int sl = 0; sl < IPW; ++sl) emit(sl, T);
      R.drain();
      return;
    }
  }
  const bool out = lead && live;
  float *ftj = (flux_traj && out) ? flux_traj + b * (int64_t)T * NX : nullptr;
  if (!kLdEmit && lead) emit(slot, 0);
  R.prime();
  typename CC::Feed F;
  CC::begin(R, F);
  for (int t = 0; t < T; ++t) {
    const float feat[1] = {s_st[g * 64 + 16 * pos + j]};
    float ff[1], fb[1];
    CC::gnn_cells(W, S, R, F, feat, ff, fb, X);
    if (!shadow && g == 0) s_F[16 * pos + j] = face_flux(ff[0], fb[0]);
    lds_barrier();  // every wave's face fluxes in s_F
#ifdef HF_DIAG_NOFV  // timing diagnostic only: results are wrong (no FV, Poisson or outputs per step)
    if (false) {
#else
    if (lead) {     // src/hybrid_solver.py:45-63, one cell per lane
#endif
      float n_new = 0.f, u_new = 0.f;
      if (lane < NX) {
        const int im = lane == 0 ? NX - 1 : lane - 1;
        const float Fv = s_F[lane];
        n_new = continuity(s_st[lane], Fv, s_F[im], c);
        u_new = velocity_hybrid(s_st[64 + lane], s_st[64 + im], s_st[128 + lane], c, dt);
        s_rho[lane] = (double)__fsub_rn(n_new, 1.0f);
        if (ftj) ftj[(int64_t)t * NX + lane] = Fv;
      }
      wave_lds_sync();
      float E_tri = 0.f;
      if (tri) {  // HF_POISSON_TRIDIAG: the lead's cyclic reduction over the IC's rho row
        tridiag_psi_wave<double>(s_rho, NX, lane);
        if (lane < NX) E_tri = (float)tri_E(s_rho, lane, NX, h);
      }
      if (lane < NX) {
        const float E_new = tri ? E_tri : poisson_cell_nx<NX>(s_rho, s_c2, lane);
        s_st[lane] = n_new;
        s_st[64 + lane] = u_new;
        s_st[128 + lane] = E_new;
      }
    }
    lds_barrier();  // new state visible to every wave
    // the lead's outputs of the new state overlap the other waves' next
    // forward (nothing writes the state again before this step's FV); with a
    // loader wave, the loader writes them
    if (!kLdEmit && lead) emit(slot, t + 1);
  }
  R.drain();
  if (!out) return;
  float *dst = state_final + b * 3 * NX;
  for (int i = lane; i < 3 * NX; i += 64) dst[i] = s_st[(i / NX) * 64 + i % NX];
}

// FluxGNN.forward on B chains of 16*WPI cells, cell-split as above (the
// small-batch counterpart of chain_flux_kernel<CoreF32, MT, true>, bit-identical to it).
template <class CC, int WPI>
__global__ __launch_bounds__(cells_threads<CC>(), 1) void chain_flux_cells_kernel(ChainW W, const float *__restrict__ nf,
                                                                  const float *__restrict__ state, int64_t ld_state,
                                                                  const float *__restrict__ x, int B,
                                                                  float *__restrict__ fe, float *__restrict__ ff) {
  constexpr int NX = 16 * WPI;
  constexpr int IPW = kWaves / WPI;
  constexpr int kRingFloats = CC::kSlots * CC::kChunkFloats;
  __shared__ f4 lds4[cells_lds_floats<CC>() / 4];
  float *lds = reinterpret_cast<float *>(lds4);
  const Small S = stage_small(W, lds + kRingFloats);
  auto R = make_ring<CC>(W, lds);
  const int wave = R.wave, lane = R.lane, j = lane & 15, g = lane >> 4;
  const bool shadow = wave >= IPW * WPI;
  const int slot = shadow ? 0 : wave / WPI, pos = shadow ? 0 : wave % WPI;
  CellHalo X;
  X.xh = reinterpret_cast<f4 *>(lds + kRingFloats + kSmallFloats + kWaves * kWaveScratchFloats);
  X.xq = X.xh + kXhF4;
  X.wave = wave;
  X.lane = lane;
  X.par = 0;
  X.lw = shadow ? wave : slot * WPI + (pos + WPI - 1) % WPI;
  X.rw = shadow ? wave : slot * WPI + (pos + 1) % WPI;
  const int b_raw = blockIdx.x * IPW + slot;
  const bool out = !shadow && b_raw < B;
  const int64_t b = b_raw < B ? b_raw : B - 1;
  const int cell = 16 * pos + j;
  const float feat[1] = {nf ? nf[(b * NX + cell) * kIn + g]
                            : (g < 3 ? state[b * ld_state + (int64_t)g * NX + cell] : x[cell])};
  __syncthreads();  // small weights staged (no DMA in flight yet)
  if constexpr (CC::R_t::kLoader) {
    if (wave == kWaves) {  // the loader (chain_rollout_cells_kernel): one pass's barriers, in order
      R.loader_prime();
      R.loader_next();  // CC::begin
      for (int l = 0; l < W.layers; ++l) {
        for (int k = 0; k < CC::kLayerChunks; ++k) R.loader_next();
        if constexpr (CC::kLayerBarrier) lds_barrier();
      }
      for (int k = R.chunks - W.layers * CC::kLayerChunks; k > 0; --k) R.loader_next();
      lds_barrier();  // the readout's column-0 trade
      R.drain();
      return;
    }
  }
  R.prime();
  typename CC::Feed F;
  CC::begin(R, F);
  float f_fwd[1], f_bwd[1];
  CC::gnn_cells(W, S, R, F, feat, f_fwd, f_bwd, X);
  R.drain();
  if (!out) return;
  if (fe && g == 0) fe[b * 2 * NX + cell] = f_fwd[0];
  if (fe && g == 1) fe[b * 2 * NX + NX + cell] = f_bwd[0];
  if (ff && g == 2) ff[b * NX + cell] = face_flux(f_fwd[0], f_bwd[0]);
}

template <class CC, int WPI>
hipError_t flux_cells_launch(const ChainW &w, const float *nf, const float *state, int64_t ld_state, const float *x,
                             int B, float *fe, float *ff, hipStream_t s) {
  constexpr int IPW = kWaves / WPI;
  hipLaunchKernelGGL((chain_flux_cells_kernel<CC, WPI>), dim3((B + IPW - 1) / IPW), dim3(cells_threads<CC>()), 0, s, w, nf,
                     state, ld_state, x, B, fe, ff);
  return hipGetLastError();
}

template <class CC, int WPI>
hipError_t cells_launch(const ChainW &w, const float *state0, float *state_final, const float *x, const double *pc,
                        int B, int T, float c, float dt, float *traj, float *flux_traj, float *metrics,
                        int pm, hipStream_t s) {
  constexpr int IPW = kWaves / WPI;
  hipLaunchKernelGGL((chain_rollout_cells_kernel<CC, WPI>), dim3((B + IPW - 1) / IPW), dim3(cells_threads<CC>()), 0, s, w,
                     state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, pm);
  return hipGetLastError();
}


// ------------------------------------------------------------------ launchers
// Workgroups resident at once: one per CU (the chain kernels hold ~500
// registers per lane, so 4 waves = one per SIMD fill a CU).
inline int resident_groups() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  return cus;
}

template <class Core, int MT, bool EXACT>
hipError_t flux_launch(const ChainW &w, const float *nf, const float *state, int64_t ld_state, const float *x,
                       int nx, int nwin, int64_t items, float *fe, float *ff, hipStream_t s) {
  const int64_t groups = (items + Core::kNW - 1) / Core::kNW;
  const int64_t res = (int64_t)resident_groups() * Core::kWGPerCU;  // persistent: kWGPerCU per CU
  const int64_t blocks = groups < res ? groups : res;
  hipLaunchKernelGGL((chain_flux_kernel<Core, MT, EXACT>), dim3((unsigned)blocks), dim3(64 * Core::kNW), 0, s,
                     w, nf, state, ld_state, x, nx, nwin, items, fe, ff);
  return hipGetLastError();
}

// Windowed flux for any nx: windows of 16*Core::kWinMT cells.
template <class Core>
hipError_t launch_flux_windowed(const ChainW &w, const float *nf, const float *state, int64_t ld_state,
                                const float *x, int B, int nx, float *fe, float *ff, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  constexpr int WMT = Core::kWinMT;
  const int faces = win_faces_of(w.layers, 16 * WMT);
  const int nwin = (nx + faces - 1) / faces;
  return flux_launch<Core, WMT, false>(w, nf, state, ld_state, x, nx, nwin, (int64_t)B * nwin, fe, ff, s);
}

template <class Core>
hipError_t launch_flux_core(const ChainW &w, const float *nf, const float *state, int64_t ld_state,
                            const float *x, int B, int nx, float *fe, float *ff, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  switch (nx) {
    case 16: return flux_launch<Core, 1, true>(w, nf, state, ld_state, x, nx, 1, B, fe, ff, s);
    case 32: return flux_launch<Core, 2, true>(w, nf, state, ld_state, x, nx, 1, B, fe, ff, s);
    case 48: return flux_launch<Core, 3, true>(w, nf, state, ld_state, x, nx, 1, B, fe, ff, s);
    case 64: return flux_launch<Core, 4, true>(w, nf, state, ld_state, x, nx, 1, B, fe, ff, s);
    default: return launch_flux_windowed<Core>(w, nf, state, ld_state, x, B, nx, fe, ff, s);
  }
}

template <class Core, int MT>
hipError_t rollout_launch(const ChainW &w, const float *state0, float *state_final, const float *x,
                          const double *pc, int B, int T, float c, float dt, float *traj, float *flux_traj,
                          float *metrics, const RolloutExtras &ex, hipStream_t s) {
  const int blocks = (B + kWaves - 1) / kWaves;
  hipLaunchKernelGGL((chain_rollout_kernel<Core, MT>), dim3(blocks), dim3(64 * kWaves), 0, s, w, state0,
                     state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, ex);
  return hipGetLastError();
}

template <class Core>
hipError_t launch_rollout_core(const ChainW &w, const float *state0, float *state_final, const float *x,
                               const double *pc, int B, int nx, int T, float c, float dt, float *traj,
                               float *flux_traj, float *metrics, const RolloutExtras &ex, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  switch (nx) {
    case 16: return rollout_launch<Core, 1>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, ex, s);
    case 32: return rollout_launch<Core, 2>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, ex, s);
    case 48: return rollout_launch<Core, 3>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, ex, s);
    case 64: return rollout_launch<Core, 4>(w, state0, state_final, x, pc, B, T, c, dt, traj, flux_traj, metrics, ex, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace chain
}  // namespace hf
