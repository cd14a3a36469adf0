// Lab: persistent 256 x 128 bf16 GEMM, ONE wave per SIMD, with the epilogue of tile i run
// inside tile i+1's main loop (VERDICT r3 "Next" #1).
//
// y[M][N] = act(A[M][K] . B[N][K]^T + bias)      (the Linear forward, "NT")
//
// * 4 waves x 512 registers.  Wave w owns rows 128 (w >> 1) .. +127 and columns 64 (w & 1) ..
//   +63 of the tile: 8 x 4 blocks of 16 x 16 accumulators (128 AGPRs).  Tiles alternate
//   between two 128-AGPR accumulator sets: while tile i+1 accumulates into one set, the
//   epilogue reads tile i's results from the other (MFMAs in inline asm with the accumulator
//   tied in place, so each set keeps one fixed AGPR assignment).
// * MFMAs are issued transposed (B . A^T), so a lane holds one output ROW and 4 consecutive
//   columns per block - the row-segment layout of the epilogue's stores.
// * LDS (160 KiB): a 3-deep ring of K-tiles (A rows 0-127 | A rows 128-255 | B rows 0-127,
//   16 KiB each, filled by buffer_load ... lds, source-swizzled), a 2 KiB staging area per
//   wave for the epilogue's row-major re-layout and two 256-B bias slots per wave (the
//   computed tile's bias lands in one while the drained tile's is read from the other).
// * The K-tile stream is continuous across tiles: K-tile k + 2 (possibly the next tile's)
//   is prefetched while k computes, so the pipeline never drains at a tile boundary.
// * One K-tile = 64 slots (2 k32 steps x 32 MFMAs).  Per slot: one MFMA plus, by slot:
//   fragment reads (step 1 of this K-tile in [0, 32), step 0 of the next in [32, 64)), DMA
//   pieces of K-tile k + 2 (6 in [0, 32), 6 in [32, 64)), one `s_waitcnt vmcnt` + barrier
//   at slot 32, and the previous tile's epilogue:
//     unit u = 16 rows of the wave tile (4 accumulator blocks):
//       A (K-tile u + 1, spread over all slots): other set -> (+bias) -> act -> packed bf16
//       B (K-tile u + 2, slots 0-31): ds_write to staging, ds_read back row-major
//       C (K-tile u + 2, slots 56-63): full-line global stores (8 rows x 128 B each)
//   The stores are counted in the next K-tile's vmcnt (they drain for a whole K-tile
//   instead of stalling the main loop the way a burst at the tile end does).
#include <hip/hip_runtime.h>

#include <utility>

#include "act.h"
#include "common.h"
#include "mfma.h"

// ---- lab knobs ----
#ifndef G4P_MASK
#define G4P_MASK 15
#endif
// lab: 1 = every store to the tile's first rows (L2-resident lines), 2 = 8 extra ops allowed
// outstanding at the slot-32 wait (timing only: the reads may then see stale LDS)
// lab: 1 = write-through (sc1) stores: the output lines are not allocated in the XCD's L2
#ifndef G4P_SC1
#define G4P_SC1 0
#endif
#ifndef G4P_STORE_MODE
#define G4P_STORE_MODE 0
#endif

namespace dpa {
namespace g4p {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_v;

constexpr int KT_BYTES = 49152;          // one K-tile: A0 | A1 | B, 16 KiB each
constexpr int STG_OFF = 3 * KT_BYTES;    // 147456
constexpr int STG_BYTES = 2048;          // per wave (the outputs of a unit are staged in turn)
constexpr int BIAS_OFF = STG_OFF + 4 * STG_BYTES;   // 155648: 2 x 256 B per wave (tile parity)
constexpr int LDS_BYTES = BIAS_OFF + 4 * 512;       // 157696
constexpr int U = 8;                     // epilogue units (16 rows each) per tile

enum { EPI_NONE = -1, EPI_BIAS = 0, EPI_ACT_D = 6 };

// MFMAs in inline asm with the accumulator TIED in place ("+a"): the accumulators then keep
// one AGPR assignment for the whole kernel (with the builtin, the many distinct K-tile code
// instances and the zero-start of each tile let the allocator rename them between regions and
// shuffle them through VGPRs and scratch).  mfma_acc: c += a . b;  mfma_zero: c = a . b.
__device__ __forceinline__ void mfma_acc(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_zero(f32x4& c, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "+a"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) char*)p);
}
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }
template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory"); }
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

typedef __attribute__((ext_vector_type(4))) unsigned u32x4_v;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2_v;

struct Kern {
  // ---- operands ----
  const bf16_t* A;
  const bf16_t* B;
  int64_t lda, ldb;
  int NT, nk, ntiles, G;
  bf16_t* C;
  bf16_t* Z;
  int64_t ldc;
  const bf16_t* bias;
  // ---- per wave ----
  char* smem;
  int w, wm, wn;
  uint32_t offA[4], offB[4];   // DMA per-lane byte offsets within an image
  uint32_t rdA[2], rdB[2];     // fragment read bases (k32 step 0 / 1), buffer 0
  uint32_t stg;                // this wave's staging area (LDS byte address)
  uint32_t bslot;              // this wave's bias slots (LDS byte address of slot 0)
  bool has_bias;
  int bpar;                    // bias slot of the computed tile (the drained one is bpar ^ 1)
  // ---- prefetch cursor (wave-uniform) ----
  int pf_tile, pf_k, pf_buf;
  const bf16_t* pfA;           // A rows of pf_tile (row 0 of the 256-row panel)
  const bf16_t* pfB;
  int cur_buf;
  // ---- tile being drained ----
  int64_t drow0;               // first output row of this wave's 128 rows in the drained tile
  int dcol0;                   // first output column of this wave's 64 columns
  int cur_tile;                // the tile being computed (its bias is DMA'd in K-tile nk - 2)

  __device__ __forceinline__ void set_pf(int tile) {
    const int t = tile < ntiles ? tile : 0;  // past the end: a harmless valid reload
    const int mt = t / NT, nt = t - (t / NT) * NT;
    pfA = A + (int64_t)mt * 256 * lda;
    pfB = B + (int64_t)nt * 128 * ldb;
  }
  // DMA piece q (0..11) of the prefetch K-tile
  __device__ __forceinline__ void piece(int q) const {
    char* img = smem + pf_buf * KT_BYTES;
    if (q < 8) {
      const int h = q >> 2, j = q & 3;
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(pfA + (int64_t)h * 128 * lda), (short)0,
                                                        0x7fffffff, 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(img + h * 16384 + (w * 4 + j) * 1024), 16, offA[j],
                                               pf_k * 128, 0, 0);
    } else {
      const int j = q - 8;
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(pfB), (short)0, 0x7fffffff, 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(img + 32768 + (w * 4 + j) * 1024), 16, offB[j],
                                               pf_k * 128, 0, 0);
    }
  }
  // the computed tile's 128 bias columns -> this wave's bias slot (every wave its own copy:
  // the VMEM op counts stay uniform); A's first row when there is no bias (values unused)
  __device__ __forceinline__ void bias_dma(int lane) const {
    const int nt = cur_tile - (cur_tile / NT) * NT;
    const char* src = has_bias ? reinterpret_cast<const char*>(bias + nt * 128) : reinterpret_cast<const char*>(A);
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + lane * 4),
                                     (lds_void*)(smem + BIAS_OFF + w * 512 + bpar * 256), 4, 0, 0);
  }
  __device__ __forceinline__ void advance_pf() {
    if (++pf_k == nk) {
      pf_k = 0;
      pf_tile += G;
      set_pf(pf_tile);
    }
    pf_buf = pf_buf == 2 ? 0 : pf_buf + 1;
  }
};

template <int I, int KK>
__device__ __forceinline__ void fragA(bf16x8& f, const Kern& k, uint32_t buf_off) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f) : "v"(k.rdA[KK] + buf_off), "i"(I * 2048));
}
template <int J, int KK>
__device__ __forceinline__ void fragB(bf16x8& f, const Kern& k, uint32_t buf_off) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f) : "v"(k.rdB[KK] + buf_off), "i"(J * 2048));
}

// Epilogue registers of the units in flight: P = packed results of phase A, Q = staged rows
struct Epi {
  uint32_t P[2][2][8];  // [unit parity][output][block j * 2 + half]: row li, columns 16j + 4g + (0..3)
                        // (unit u + 1's phase A runs while unit u's phase B stages u's values)
  u32x4_v Q[2][2];   // [output][q]: row (lane >> 3) + 8q, columns 8 (lane & 7) .. +7
  u32x2_v bias[4];   // the drained tile's bias, block j: columns 16j + 4g + (0..3)
};

// the drained tile's bias of block j (columns 16j + 4g .. +3 of this wave's 64) from its slot
template <int J>
__device__ __forceinline__ void bias_read(Epi& e, const Kern& k, int lane) {
  const uint32_t a = k.bslot + (k.bpar ^ 1) * 256 + (uint32_t)((64 * k.wn + 16 * J + 4 * (lane >> 4)) * 2);
  asm volatile("ds_read_b64 %0, %1" : "=v"(e.bias[J]) : "v"(a));
}

template <int EPI>
struct Outs { static constexpr int n = EPI == EPI_ACT_D ? 2 : EPI == EPI_NONE ? 0 : 1; };

// phase A of unit u, part p (0..7: pairs of columns of block j = p >> 1, registers 2(p&1)..+1):
// accumulators of the drained tile -> (+bias) -> act -> bf16 pairs
template <int EPI, int ACT, int UNIT, int P>
__device__ __forceinline__ void phaseA(Epi& e, f32x4 (&acc2)[8][4], const Kern& k) {
  // (acc2: the drained tile's accumulator set)
  constexpr int j = P >> 1, r = (P & 1) * 2;
  // an opaque "write" of the block right here: without it hipcc hoists every v_accvgpr_read
  // of the drained set to the start of the tile (128 VGPRs live at once -> spills)
  if constexpr ((P & 1) == 0) asm volatile("" : "+a"(acc2[UNIT][j]));
  const float x0 = acc2[UNIT][j][r], x1 = acc2[UNIT][j][r + 1];
  const uint32_t bw = k.has_bias ? e.bias[j][P & 1] : 0u;
  f32x2 z = f32x2{x0 + __uint_as_float(bw << 16), x1 + __uint_as_float(bw & 0xffff0000u)};
  if constexpr (EPI == EPI_BIAS) {
    e.P[UNIT & 1][0][P] = pack_bf2(z.x, z.y);
  } else if constexpr (EPI == EPI_ACT_D) {
    // GELU / SiLU computed from the bf16-rounded pre-activation (as the 8-wave kernel)
    const uint32_t zb = pack_bf2(z.x, z.y);
    z = f32x2{__uint_as_float(zb << 16), __uint_as_float(zb & 0xffff0000u)};
    f32x2 d;
    const f32x2 y = act_dact2<ACT>(z, d);
    e.P[UNIT & 1][0][P] = pack_bf2(y.x, y.y);
    e.P[UNIT & 1][1][P] = pack_bf2(d.x, d.y);
  }
}

// phase B of a unit: this wave's 16 x 64 block of output o -> staging (row-major, 128-B rows,
// 16-B chunks XOR-swizzled by row) -> back as full rows
template <int UNIT, int O, int PART>
__device__ __forceinline__ void phaseB_write(const Epi& e, const Kern& k, int lane) {
  // PART j: block j's 4 columns (two bf16x2) of row li
  const int g = lane >> 4, li = lane & 15;
  const int c = 2 * PART + (g >> 1);
  const uint32_t a = k.stg + li * 128 + ((c ^ (li & 7)) << 4) + (g & 1) * 8;
  const u32x2_v v = {e.P[UNIT & 1][O][2 * PART], e.P[UNIT & 1][O][2 * PART + 1]};
  asm volatile("ds_write_b64 %0, %1" ::"v"(a), "v"(v) : "memory");
}
template <int O, int Q>
__device__ __forceinline__ void phaseB_read(Epi& e, const Kern& k, int lane) {
  const int row = (lane >> 3) + 8 * Q, c = lane & 7;
  const uint32_t a = k.stg + row * 128 + ((c ^ (row & 7)) << 4);
  asm volatile("ds_read_b128 %0, %1" : "=v"(e.Q[O][Q]) : "v"(a));
}
__device__ __forceinline__ int opaque(int x) {
  int y;
  asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
  return y;
}

template <int O, int Q>
__device__ __forceinline__ void phaseC(const Epi& e, const Kern& k, int lane_, int unit) {
  const int lane = opaque(lane_);  // (per-unit addresses computed here, not hoisted and kept live)
  const int64_t row = G4P_STORE_MODE == 1 ? (int64_t)(lane >> 3) : k.drow0 + 16 * unit + (lane >> 3) + 8 * Q;
  const int col = k.dcol0 + 8 * (lane & 7);
  bf16_t* dst = (O == 0 ? k.C : k.Z) + row * k.ldc + col;
  // (s_nop 1: the next instruction must not overwrite the data registers before the store
  // has read them - hipcc pads nothing inside an asm statement)
#if G4P_SC1
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(dst), "v"(e.Q[O][Q]) : "memory");
#else
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(dst), "v"(e.Q[O][Q]) : "memory");
#endif
}

// ---------------------------------------------------------------------------------------
// One K-tile.  KIDX: 0..U+1 = K-tile index inside a tile whose previous tile is being
// drained (units A at KIDX-1, B/C at KIDX-2), -1 = plain.  FIRST: K-tile 0 of a tile (step 0
// starts from zero).  SET: the accumulator set of the computed tile.  PST: stores issued by the
// previous K-tile (counted in this K-tile's vmcnt).
template <int EPI, int ACT, int KIDX, bool FIRST, int SET, int PST_>
struct KTile {
  static constexpr int PST = (G4P_MASK & 4) ? PST_ : 0;
  // bias of the drained tile into registers one K-tile before its first phase A use
  static constexpr int NO = Outs<EPI>::n;
  static constexpr int UA = (G4P_MASK & 1) && KIDX >= 1 && KIDX <= U ? KIDX - 1 : -1;       // phase A unit
  static constexpr int UB = (G4P_MASK & 2) && KIDX >= 2 && KIDX <= U + 1 ? KIDX - 2 : -1;   // phase B unit
  static constexpr int UBC = (G4P_MASK & 4) && KIDX >= 2 && KIDX <= U + 1 ? KIDX - 2 : -1;  // phase C unit
  static constexpr int NST = UBC >= 0 ? 2 * NO : 0;                       // stores issued here

  template <int S>
  static __device__ __forceinline__ void slot(Kern& k, f32x4 (&acc)[2][8][4], bf16x8 (&fa0)[8],
                                              bf16x8 (&fb0)[4], bf16x8 (&fa1)[8], bf16x8 (&fb1)[4], Epi& e,
                                              uint32_t cur, uint32_t nxt, int lane, int kt) {
    constexpr int step = S >> 5, blk = S & 31, i = blk >> 2, j = blk & 3;
    // the computed tile's bias -> its LDS slot, two K-tiles before the tile ends (retired by
    // this K-tile's slot-32 wait: it is older than the pieces issued after it)
    if constexpr (S == 0 && NO > 0) {
      if (kt == k.nk - 2) k.bias_dma(lane);
    }
    if constexpr (step == 0) {
      if constexpr (FIRST) mfma_zero(acc[SET][i][j], fb0[j], fa0[i]);
      else mfma_acc(acc[SET][i][j], fb0[j], fa0[i]);
    } else {
      mfma_acc(acc[SET][i][j], fb1[j], fa1[i]);
    }
    // step-1 fragments of this K-tile: A block r at slot 4r, B block r at slot 4r + 2
    if constexpr (S < 32 && (S & 3) == 0) fragA<(S >> 2), 1>(fa1[S >> 2], k, cur);
    if constexpr (S < 16 && (S & 3) == 2) fragB<(S >> 2), 1>(fb1[S >> 2], k, cur);
    // phase B of unit UBC: 4 x NO staging writes (slots 17..), 2 x NO reads (slots 25..)
    // (one staging area: output 0 written and read back, then output 1; a wave's LDS ops
    // execute in order, so output 1's writes cannot overtake output 0's reads)
    if constexpr (UB >= 0 && NO >= 1 && S >= 17 && S <= 20) phaseB_write<UB, 0, S - 17>(e, k, lane);
    if constexpr (UB >= 0 && NO >= 1 && S == 21) phaseB_read<0, 0>(e, k, lane);
    if constexpr (UB >= 0 && NO >= 1 && S == 22) phaseB_read<0, 1>(e, k, lane);
    if constexpr (UB >= 0 && NO >= 2 && S >= 23 && S <= 26) phaseB_write<UB, 1, S - 23>(e, k, lane);
    if constexpr (UB >= 0 && NO >= 2 && S == 27) phaseB_read<1, 0>(e, k, lane);
    if constexpr (UB >= 0 && NO >= 2 && S == 28) phaseB_read<1, 1>(e, k, lane);
    if constexpr (S == 31) wait_lgkm0();
    // DMA of K-tile k + 2: 6 pieces in [0, 32), 6 in [32, 64)
    if constexpr (S < 32 && S % 5 == 1 && S / 5 < 6) k.piece(S / 5);
    if constexpr (S == 32) {
      wait_vm<6 + PST + (G4P_STORE_MODE == 2 ? 8 : 0)>();
      barrier();
    }
    if constexpr (S >= 33 && (S - 33) % 4 == 0 && (S - 33) / 4 < 6) k.piece(6 + (S - 33) / 4);
    // step-0 fragments of the next K-tile: A block r at 32 + 3r (r < 8), B block r at 33 + 3r (r < 4)
    if constexpr (S >= 32 && S < 56 && (S - 32) % 3 == 0) fragA<(S - 32) / 3, 0>(fa0[(S - 32) / 3], k, nxt);
    if constexpr (S >= 33 && S < 45 && (S - 33) % 3 == 0) fragB<(S - 33) / 3, 0>(fb0[(S - 33) / 3], k, nxt);
    // the drained tile's bias for the NEXT K-tile's phase A (retired by the slot-63 wait)
    if constexpr (NO > 0 && KIDX >= 0 && KIDX < U && S >= 34 && S <= 37) bias_read<S - 34>(e, k, lane);
    // phase A of unit UA: part p at slot 8p + 4
    if constexpr (UA >= 0 && NO >= 1 && (S & 7) == 4) phaseA<EPI, ACT, UA, (S >> 3)>(e, acc[SET ^ 1], k);
    // phase C of unit UBC: stores at 56, 58 (y) and 60, 62 (d)
    if constexpr (UBC >= 0 && NO >= 1 && S == 56) phaseC<0, 0>(e, k, lane, UBC);
    if constexpr (UBC >= 0 && NO >= 1 && S == 58) phaseC<0, 1>(e, k, lane, UBC);
    if constexpr (UBC >= 0 && NO >= 2 && S == 60) phaseC<1, 0>(e, k, lane, UBC);
    if constexpr (UBC >= 0 && NO >= 2 && S == 62) phaseC<1, 1>(e, k, lane, UBC);
    if constexpr (S == 63) wait_lgkm0();
    __builtin_amdgcn_sched_barrier(0);
  }

  template <int... S>
  static __device__ __forceinline__ void all(Kern& k, f32x4 (&acc)[2][8][4], bf16x8 (&fa0)[8],
                                             bf16x8 (&fb0)[4], bf16x8 (&fa1)[8], bf16x8 (&fb1)[4], Epi& e,
                                             uint32_t cur, uint32_t nxt, int lane, int kt,
                                             std::integer_sequence<int, S...>) {
    (slot<S>(k, acc, fa0, fb0, fa1, fb1, e, cur, nxt, lane, kt), ...);
  }

  static __device__ __forceinline__ void run(Kern& k, f32x4 (&acc)[2][8][4], bf16x8 (&fa0)[8],
                                             bf16x8 (&fb0)[4], bf16x8 (&fa1)[8], bf16x8 (&fb1)[4], Epi& e,
                                             int lane, int kt) {
    const uint32_t cur = (uint32_t)(k.cur_buf * KT_BYTES);
    const int nb = k.cur_buf == 2 ? 0 : k.cur_buf + 1;
    const uint32_t nxt = (uint32_t)(nb * KT_BYTES);
    __builtin_amdgcn_s_setprio(1);
    all(k, acc, fa0, fb0, fa1, fb1, e, cur, nxt, lane, kt, std::make_integer_sequence<int, 64>{});
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    k.cur_buf = nb;
    k.advance_pf();
  }
};

template <int EPI, int ACT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
gemm4p_kernel(const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ B, int64_t ldb, int M, int N,
              int nk, bf16_t* __restrict__ C, bf16_t* __restrict__ Z, int64_t ldc, const bf16_t* __restrict__ bias) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  Kern k;
  k.A = A; k.B = B; k.lda = lda; k.ldb = ldb;
  k.NT = N / 128;
  k.nk = nk;
  k.ntiles = (M / 256) * k.NT;
  k.G = gridDim.x;
  k.C = C; k.Z = Z; k.ldc = ldc; k.bias = bias;
  k.smem = smem;
  k.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  k.wm = k.w >> 1;
  k.wn = k.w & 1;
  const int lane = threadIdx.x & 63;
  const uint32_t sbase = lds_u32(smem);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = (k.w * 4 + j) * 8 + (lane >> 3), phys = lane & 7;
    k.offA[j] = (uint32_t)(r * (int)lda + ((phys ^ ((r >> 1) & 7)) << 3)) * 2u;
    k.offB[j] = (uint32_t)(r * (int)ldb + ((phys ^ ((r >> 1) & 7)) << 3)) * 2u;
  }
  {
    const int g = lane >> 4, li = lane & 15, s = (li >> 1) & 7;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      k.rdA[kk] = sbase + k.wm * 16384 + (uint32_t)(li * 128 + (((kk * 4 + g) ^ s) << 4));
      k.rdB[kk] = sbase + 32768 + (uint32_t)((64 * k.wn + li) * 128 + (((kk * 4 + g) ^ s) << 4));
    }
  }
  k.stg = sbase + STG_OFF + k.w * STG_BYTES;

  int tile = xcd_remap(blockIdx.x, k.G);
  if (tile >= k.ntiles) return;

  f32x4 acc[2][8][4];  // [set]: the computed tile's and the drained tile's accumulators
  bf16x8 fa0[8], fb0[4], fa1[8], fb1[4];
  Epi e;

  // prologue: K-tiles 0 and 1 of the first tile into buffers 0, 1; K-tile 0's step-0 fragments
  k.pf_tile = tile;
  k.set_pf(tile);
  k.pf_k = 0;
  k.pf_buf = 0;
#pragma unroll
  for (int q = 0; q < 12; ++q) k.piece(q);
  k.advance_pf();
#pragma unroll
  for (int q = 0; q < 12; ++q) k.piece(q);
  k.advance_pf();
  k.cur_buf = 0;
  wait_vm<12>();
  barrier();
  fragA<0, 0>(fa0[0], k, 0); fragA<1, 0>(fa0[1], k, 0); fragA<2, 0>(fa0[2], k, 0); fragA<3, 0>(fa0[3], k, 0);
  fragA<4, 0>(fa0[4], k, 0); fragA<5, 0>(fa0[5], k, 0); fragA<6, 0>(fa0[6], k, 0); fragA<7, 0>(fa0[7], k, 0);
  fragB<0, 0>(fb0[0], k, 0); fragB<1, 0>(fb0[1], k, 0); fragB<2, 0>(fb0[2], k, 0); fragB<3, 0>(fb0[3], k, 0);
  wait_lgkm0();

  constexpr int NO = Outs<EPI>::n;
  k.has_bias = bias != nullptr;
  k.bslot = sbase + BIAS_OFF + k.w * 512;
  k.bpar = 0;
  k.cur_tile = tile;
  using KT0 = KTile<EPI, ACT, -1, true, 0, 0>;
  using KTP0 = KTile<EPI, ACT, -1, false, 0, 0>;
  // first tile (accumulator set 0): nothing to drain
  KT0::run(k, acc, fa0, fb0, fa1, fb1, e, lane, 0);
  for (int kt = 1; kt < k.nk; ++kt) KTP0::run(k, acc, fa0, fb0, fa1, fb1, e, lane, kt);

  // A tile computed into set SET while the previous tile (set SET ^ 1) is drained in the
  // first U + 2 K-tiles.  Past the last tile the stream continues on clamped (valid) prefetch
  // data for those K-tiles only, so the last tile's epilogue runs on the same code path.
  // Returns false when that was the drain-only pass.
  auto tile_pass = [&](auto SET_) -> bool {
    constexpr int SET = decltype(SET_)::value;
    {
      const int mt = tile / k.NT, nt = tile - (tile / k.NT) * k.NT;
      k.drow0 = (int64_t)mt * 256 + k.wm * 128;
      k.dcol0 = nt * 128 + k.wn * 64;
      k.bpar ^= 1;
    }
    tile += k.G;
    const bool last = tile >= k.ntiles;
    k.cur_tile = last ? 0 : tile;
    KTile<EPI, ACT, 0, true, SET, 0>::run(k, acc, fa0, fb0, fa1, fb1, e, lane, 0);
    KTile<EPI, ACT, 1, false, SET, 0>::run(k, acc, fa0, fb0, fa1, fb1, e, lane, 1);
    KTile<EPI, ACT, 2, false, SET, 0>::run(k, acc, fa0, fb0, fa1, fb1, e, lane, 2);
    KTile<EPI, ACT, 3, false, SET, 2 * NO>::run(k, acc, fa0, fb0, fa1, fb1, e, lane, 3);
    KTile<EPI, ACT, 4, false, SET, 2 * NO>::run(k, acc, fa0, fb0, fa1, fb1, e, lane, 4);
    KTile<EPI, ACT, 5, false, SET, 2 * NO>::run(k, acc, fa0, fb0, fa1, fb1, e, lane, 5);
    KTile<EPI, ACT, 6, false, SET, 2 * NO>::run(k, acc, fa0, fb0, fa1, fb1, e, lane, 6);
    KTile<EPI, ACT, 7, false, SET, 2 * NO>::run(k, acc, fa0, fb0, fa1, fb1, e, lane, 7);
    KTile<EPI, ACT, 8, false, SET, 2 * NO>::run(k, acc, fa0, fb0, fa1, fb1, e, lane, 8);
    KTile<EPI, ACT, 9, false, SET, 2 * NO>::run(k, acc, fa0, fb0, fa1, fb1, e, lane, 9);
    if (last) return false;
    KTile<EPI, ACT, -1, false, SET, 2 * NO>::run(k, acc, fa0, fb0, fa1, fb1, e, lane, 10);
    for (int kt = U + 3; kt < k.nk; ++kt)
      KTile<EPI, ACT, -1, false, SET, 0>::run(k, acc, fa0, fb0, fa1, fb1, e, lane, kt);
    return true;
  };
  while (tile_pass(std::integral_constant<int, 1>{}) && tile_pass(std::integral_constant<int, 0>{})) {
  }
  // the last units' stores and the clamped prefetch pieces are still in flight
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace g4p

// y[M][N] = act(A[M][K] . B[N][K]^T + bias) (act' into Z for EPI 6); M % 256, N % 128, K % 64,
// K >= 704 (nk >= U + 3: the drained tile's units fit the next tile's K-tiles)
template <int EPI, int ACT>
inline void launch_gemm4p(const uint16_t* A, const uint16_t* B, const uint16_t* bias, uint16_t* C, uint16_t* Z,
                          int M, int N, int K, int ncu, hipStream_t s) {
  const int tiles = (M / 256) * (N / 128);
  const int grid = tiles < ncu ? tiles : ncu;
  hipLaunchKernelGGL((g4p::gemm4p_kernel<EPI, ACT>), dim3(grid), dim3(256), 0, s, (const bf16_t*)A, (int64_t)K,
                     (const bf16_t*)B, (int64_t)K, M, N, K / 64, (bf16_t*)C, (bf16_t*)Z, (int64_t)N,
                     (const bf16_t*)bias);
}

}  // namespace dpa
