// 256 x 256 bf16 MFMA GEMM, 8-phase software pipeline (CDNA4 / gfx950).
//
// Same three Linear-layer products as gemm.hip (fwd "MK.NK", dgrad "MK.KN",
// wgrad "KM.KN"), restructured for one workgroup per CU at high MFMA density:
//
// * 512 threads = 8 waves, 256 x 256 output tile, BK = 64, v_mfma_f32_16x16x32_bf16.
// * LDS (one 128 KiB array): 2 K-tile buffers (even / odd K-tile) x 4 half-tile
//   images {A rows 0-127, A rows 128-255, B rows 0-127, B rows 128-255} of
//   16 KiB.  Images are written by global_load_lds_dwordx4 (lane-linear, so the
//   XOR swizzle is applied to the per-lane global *source* address and undone on
//   the read).  Row-form images ([128][64], 128-B rows) are read with
//   ds_read_b128; transposed images ([64 k][128], 256-B rows: operands whose
//   reduction dimension is outermost in memory) with ds_read_b64_tr_b16.
// * A K-tile is computed in 4 phases, one 128 x 128 C quadrant per phase
//   (A0.B0, A0.B1, A1.B1, A1.B0), each wave owning a 64 x 32 block of it (16
//   MFMAs per phase).  Fragments are reused across phases (phase 4 reads
//   nothing), so a K-tile costs 24 row-form LDS reads per wave instead of 48.
// * One half-tile image is prefetched per phase and a counted `s_waitcnt
//   vmcnt(8)` in every phase retires the half staged four phases earlier, so four
//   half-tiles (64 KiB) stay in flight across the barriers (no vmcnt(0) in the
//   main loop, raw s_barrier).  The staging slots satisfy, for every half:
//   restaged >= 2 phases after its last read (WAR) and first read >= 1 phase
//   after the wait that retires it (RAW), both needed because the two wave
//   groups run staggered by one barrier.
// * Wave group 1 (waves 4-7) runs one barrier behind group 0, so on every SIMD
//   one wave issues MFMAs while the other issues LDS reads and DMA.
// * Workgroups are remapped so consecutive tiles (sharing an A panel) run on one XCD.
//
// Epilogues: bf16 (+bias, +activation, pre-activation copy) staged through LDS
// as 16-B row stores, or fp32 atomic accumulation into the fp32 gradient buffer
// (split-K wgrad) with the bias gradient reduced from the staged dy images.
#include <cstdlib>

#include "act.h"
#include "common.h"
#include "launchers.h"
#include "mfma.h"

namespace dpa {
namespace g256 {

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void glob_void;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_v;

// LDS map (bytes): A images in [0, 64K), B images in [64K, 128K), so every
// fragment read is one per-lane base VGPR + an immediate offset (< 64 KiB):
//   A(buf, h) = buf * 32K + h * 16K,   B(buf, h) = 64K + buf * 32K + h * 16K
constexpr int HALF = 16384;
constexpr int B_REGION = 65536;
__host__ __device__ constexpr int img_off(int buf, int h) { return buf * 2 * HALF + h * HALF; }

// EPI_DACT: dgrad with the previous layer's activation backward fused in:
// C = (A.B) * act'(aux), aux = pre-activation z (gelu, silu) or output y (tanh).
// EPI_NONE: no store (accumulators kept live) - timing probe of the main loop only.
enum { EPI_BF16 = 0, EPI_BIAS_ACT = 1, EPI_ATOMIC_F32 = 2, EPI_DACT = 3, EPI_NONE = 4 };

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_v, a),
                                                 __builtin_bit_cast(bf16x8_v, b), c, 0, 0, 0);
}

__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) char*)p);
}

// Chunk XOR of a transposed image row: conflict-free ds_read_b64_tr_b16 for the
// 16x16x32 operand (a 32-lane half reads rows {q, 8+q} (+16n) of two 16-B chunks).
__device__ __forceinline__ int tr_x(int row) { return ((row & 3) << 1) | (((row >> 3) & 1) << 3); }

__device__ __forceinline__ float act_f(float z, int act) { return act_apply(z, act); }
__device__ __forceinline__ float dact_f(float a, int act) { return act_deriv(a, act); }

__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }

// ---- one operand (A or B) --------------------------------------------------
template <bool TR>
struct Operand {
  const bf16_t* base;  // element (row 0 of this tile, k = 0) - wave-uniform
  int64_t ld;
  uint32_t off[2];     // byte offsets of this thread's two DMA pieces within a half image
                       // (unsigned 32-bit: the DMA uses SGPR base + VGPR offset addressing)
  uint32_t rd[4];      // LDS read byte offsets (relative to a half image)
  int wv;              // wave id (wave-uniform)
  int hstep;           // rows (row form) / columns (TR form) between the two half images

  // row0: first row (row form) / column (TR form) of the 256-wide tile; this
  // wave's sub-block starts at row/col wsub * wrows of a half; region: LDS byte
  // address of this operand's images.
  // remap (B operand of the persistent kernel): half image h holds the 4 x 32 rows /
  // columns {64 c + 32 h + (0..31) : c = 0..3} of the 256-wide tile instead of rows
  // 128 h .. 128 h + 127, so the wave owning image block c of both halves owns 64
  // CONTIGUOUS output columns (full 128-B lines in its epilogue stores).
  __device__ __forceinline__ void init(const bf16_t* p, int64_t ld_, int row0, int w, int lane,
                                       int wsub, int wrows, uint32_t region, bool remap = false) {
    ld = ld_;
    wv = w;
    hstep = remap ? 32 : 128;
    base = TR ? p + row0 : p + (int64_t)row0 * ld_;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int piece = w * 2 + j;
      if constexpr (TR) {
        const int k = piece * 4 + (lane >> 4), phys = lane & 15;
        const int lc = phys ^ tr_x(k);                              // 16-B chunk of the image row
        const int gc = remap ? lc * 8 + ((lc >> 2) << 5) : lc * 8;  // its first tile column
        off[j] = (uint32_t)(k * (int)ld_ + gc) * 2u;
      } else {
        const int r = piece * 8 + (lane >> 3), phys = lane & 7;
        const int rg = remap ? r + ((r >> 5) << 5) : r;             // tile row of image row r
        off[j] = (uint32_t)(rg * (int)ld_ + ((phys ^ ((r >> 1) & 7)) << 3)) * 2u;
      }
    }
    const int g = lane >> 4, li = lane & 15;
    if constexpr (TR) {
      const int q = li >> 2, p = li & 3;
      const int x = (q << 1) | ((g & 1) << 3);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int cb = wsub * wrows + c * 16;
        const int ch = ((cb >> 3) + (p >> 1)) ^ x;
        rd[c] = region + (uint32_t)((8 * g + q) * 256 + ch * 16 + (p & 1) * 8);
      }
    } else {
      const int row = wsub * wrows + li;
      const int s = (row >> 1) & 7;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) rd[kk] = region + (uint32_t)(row * 128 + (((kk * 4 + g) ^ s) << 4));
      rd[2] = rd[3] = 0;
    }
  }

  // DMA one half image (h = 0/1) of K-tile t into LDS at `img`: buffer_load ... lds
  // with a wave-uniform descriptor at the half image's origin and the 32-bit per-lane
  // offsets (no 64-bit per-lane addresses to keep live across the main loop).
  __device__ __forceinline__ void stage(char* img, int h, int t) const {
    const bf16_t* src = TR ? base + (int64_t)t * 64 * ld + h * hstep : base + (int64_t)h * hstep * ld + t * 64;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(src), (short)0, 0x7fffffff,
                                                      0x00020000);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(img + (wv * 2 + j) * 1024), 16, off[j], 0, 0,
                                               0);
  }

  // Fragment of 16-row (row form) / 16-column (TR form) block I, k-step KK, of
  // the half image at byte offset IMG within the operand's region.  Issued from
  // asm (no compiler vmcnt drain against the in-flight DMA); the caller retires
  // it with lgkmcnt.
  template <int IMG, int I, int KK>
  __device__ __forceinline__ void frag(bf16x8& f) const {
    if constexpr (TR) {
      bf16x4 a, b;
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(a) : "v"(rd[I]), "i"(IMG + KK * 32 * 256));
      asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(b) : "v"(rd[I]), "i"(IMG + KK * 32 * 256 + 1024));
      f = cat44(a, b);
    } else {
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f) : "v"(rd[KK]), "i"(IMG + I * 2048));
    }
  }
};

template <int IMG, bool TR>
__device__ __forceinline__ void read4(bf16x8 (&f)[4][2], const Operand<TR>& op) {
  op.template frag<IMG, 0, 0>(f[0][0]); op.template frag<IMG, 0, 1>(f[0][1]);
  op.template frag<IMG, 1, 0>(f[1][0]); op.template frag<IMG, 1, 1>(f[1][1]);
  op.template frag<IMG, 2, 0>(f[2][0]); op.template frag<IMG, 2, 1>(f[2][1]);
  op.template frag<IMG, 3, 0>(f[3][0]); op.template frag<IMG, 3, 1>(f[3][1]);
}
template <int IMG, bool TR>
__device__ __forceinline__ void read2(bf16x8 (&f)[2][2], const Operand<TR>& op) {
  op.template frag<IMG, 0, 0>(f[0][0]); op.template frag<IMG, 0, 1>(f[0][1]);
  op.template frag<IMG, 1, 0>(f[1][0]); op.template frag<IMG, 1, 1>(f[1][1]);
}

// Bias-gradient partial sums from a transposed [64 k][128] dy image (at byte
// offset IMG of the A region), read by the wave group that owns it: thread t
// (0..255) sums column (t & 127) over rows 32*(t>>7) .. +31 with eight
// ds_read_b64_tr_b16 (4 rows of its column each) into ONE register.
// csa[0/1]: per-thread read bases for rows with bit 3 clear / set.
template <int IMG>
__device__ __forceinline__ void colsum_read(float& cs, const uint32_t (&csa)[2]) {
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    bf16x4 v;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(v) : "v"(csa[(r >> 1) & 1]), "i"(IMG + 4 * r * 256));
#pragma unroll
    for (int e = 0; e < 4; ++e) cs += __uint_as_float(((uint32_t)(uint16_t)v[e]) << 16);
  }
}

// SWAP: B.A^T instead of A.B^T - the accumulator then holds C transposed (lane =
// row of C, registers = 4 consecutive columns), the layout of the persistent
// kernel's register-direct epilogue.
// Z: the quadrant's first MFMAs of a tile take the inline constant 0 as their C operand (no
// accumulator zeroing pass: 128 v_mov per wave per tile between the epilogue and the next main loop)
template <int QA, int QB, bool SWAP = false, bool Z = false>
__device__ __forceinline__ void mfma_quadrant(f32x4 (&acc)[2][2][4][2], const bf16x8 (&fa)[4][2],
                                              const bf16x8 (&fb)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const f32x4 c = (Z && kk == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[QA][QB][i][j];
        if constexpr (SWAP) acc[QA][QB][i][j] = mfma16(fb[j][kk], fa[i][kk], c);
        else acc[QA][QB][i][j] = mfma16(fa[i][kk], fb[j][kk], c);
      }
  __builtin_amdgcn_s_setprio(0);
}

template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory"); }

// Sum over the 16 lanes of a DPP row (every lane gets the row total): four DPP adds
// (quad xor 1, quad xor 2, half-row mirror, row rotate by 8) - no LDS, no address VGPRs.
__device__ __forceinline__ float row16_sum(float x) {
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, true));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xF, 0xF, true));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x141, 0xF, 0xF, true));
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xF, 0xF, true));
  return x;
}

// Lane id recomputed from the EXEC mask (no VGPR has to stay live for it).
__device__ __forceinline__ int lane_id() {
  return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// A copy of x the compiler cannot see through (keeps loop-invariant lane
// arithmetic from being hoisted across a long-lived register-heavy loop).
__device__ __forceinline__ int opaque(int x) {
  int y;
  asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
  return y;
}

// One phase P (0..7) of a 2-K-tile iteration; te = even K-tile of the iteration.
// XS / extra (persistent kernel): `extra` = XS stores of the previous tile were
// issued between this tile's prologue DMA and its first iteration, so the waits
// of phases 0-3 of that iteration leave them in flight.
template <int P, bool A_TR, bool B_TR, bool CS, bool SWAP = false, int XS = 0, int DRAIN = 0, bool HM = false,
          bool Z = false>
__device__ __forceinline__ void phase(f32x4 (&acc)[2][2][4][2], bf16x8 (&fa)[4][2],
                                      bf16x8 (&fb0)[2][2], bf16x8 (&fb1)[2][2], float& cs,
                                      const Operand<A_TR>& opA, const Operand<B_TR>& opB,
                                      char* smem, const uint32_t (&csa)[2], int te, bool more, bool do_cs,
                                      int grp, bool extra = false) {
  constexpr int q = P & 3;
  constexpr int bf = P < 4 ? 0 : 1;
  char* const smB = smem + B_REGION;
  // 1. LDS fragment reads (B first, then A)
  if constexpr (q == 0) {
    read2<img_off(bf, 0)>(fb0, opB);
    __builtin_amdgcn_sched_barrier(0);
    read4<img_off(bf, 0)>(fa, opA);
  } else if constexpr (q == 1) {
    read2<img_off(bf, 1)>(fb1, opB);
  } else if constexpr (q == 2 && !HM) {
    read4<img_off(bf, 1)>(fa, opA);
  }
  // group 0 sums the A0 image, group 1 the A1 image (wave-uniform branch)
  if constexpr (CS && q == 0) { if (do_cs && grp == 0) colsum_read<img_off(bf, 0)>(cs, csa); }
  if constexpr (CS && q == 2) { if (do_cs && grp == 1) colsum_read<img_off(bf, 1)>(cs, csa); }
  // 2. prefetch one half image (schedule in the header comment), then retire the
  //    half staged 4 phases ago (4 half-tiles = 8 DMA ops stay in flight); in the
  //    last iteration fewer halves are issued, so drain instead.
  if constexpr (P == 0) opB.stage(smB + img_off(1, 1), 1, te + 1);
  if constexpr (P == 1) opA.stage(smem + img_off(1, 1), 1, te + 1);
  if constexpr (P == 2) { if (more) opA.stage(smem + img_off(0, 0), 0, te + 2); }
  if constexpr (P == 3) { if (more) opB.stage(smB + img_off(0, 0), 0, te + 2); }
  if constexpr (P == 4) { if (more) opB.stage(smB + img_off(0, 1), 1, te + 2); }
  if constexpr (P == 5) { if (more) opA.stage(smem + img_off(0, 1), 1, te + 2); }
  if constexpr (P == 6) { if (more) opA.stage(smem + img_off(1, 0), 0, te + 3); }
  if constexpr (P == 7) { if (more) opB.stage(smB + img_off(1, 0), 0, te + 3); }
  if (more) {
    if constexpr (XS > 0 && P < 4) {
      if (extra) wait_vm<8 + XS>();
      else wait_vm<8>();
    } else {
      wait_vm<8>();
    }
  } else {
    wait_vm<DRAIN>();  // DRAIN: ops issued after the last DMA that may stay in flight
  }
  // 3. barrier, retire reads, 16 MFMAs on one quadrant, barrier
  barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (q == 0) mfma_quadrant<0, 0, SWAP, Z>(acc, fa, fb0);
  if constexpr (q == 1) mfma_quadrant<0, 1, SWAP, Z>(acc, fa, fb1);
  // HM (128-row tiles): the A1 image is a copy of A0 (DMA kept: the counted waits stay
  // exact) and its two quadrants are skipped
  if constexpr (q == 2 && !HM) mfma_quadrant<1, 1, SWAP, Z>(acc, fa, fb1);
  if constexpr (q == 3 && !HM) mfma_quadrant<1, 0, SWAP, Z>(acc, fa, fb0);
  __builtin_amdgcn_sched_barrier(0);
  barrier();
}

// Token segments of a multi-segment weight gradient: dW += sum_s dy_s^T x_s, every segment
// ktiles_total K-tiles long (the reference schedule's deferred micro-batch pairs).
constexpr int WG_MAXSEG = 8;
struct WgSegs {
  const bf16_t* a[WG_MAXSEG];
  const bf16_t* b[WG_MAXSEG];
  int n;  // 0: the kernel's A / B are the only segment
};

template <bool A_TR, bool B_TR, int EPI>
__global__ void __launch_bounds__(512) gemm256_kernel(
    const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ B, int64_t ldb, int M,
    int N, int ktiles_total, int ktiles_per_split, int splits, bf16_t* __restrict__ C, int64_t ldc,
    float* __restrict__ Cf, const bf16_t* __restrict__ bias, int act, bf16_t* __restrict__ Zout,
    float* __restrict__ colsum, float* __restrict__ wsp = nullptr, WgSegs segs = WgSegs{}) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * B_REGION];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = (w >> 2) & 1, wn = w & 3;  // 2 x 4 waves over a 128 x 128 quadrant
  const int grp = __builtin_amdgcn_readfirstlane(w >> 2);
  const int MT = M / 256, NT = N / 256;
  const int nseg = segs.n > 0 ? segs.n : 1;
  const int tile = xcd_remap(blockIdx.x, MT * NT * splits * nseg);
  const int nt = tile % NT, mt = (tile / NT) % MT, z = tile / (NT * MT);  // z: workspace slab
  const int m0 = mt * 256, n0 = nt * 256;
  const int zs = z % splits;  // split within the segment
  if (segs.n > 0) {
    const int sg = z / splits;
#pragma unroll
    for (int i = 0; i < WG_MAXSEG; ++i)  // uniform selects: no dynamic index into the kernarg struct
      if (sg == i) {
        A = segs.a[i];
        B = segs.b[i];
      }
  }
  const int t0 = zs * ktiles_per_split;
  const int nk = min(ktiles_total - t0, ktiles_per_split);  // even, >= 2 (host guarantees)

  Operand<A_TR> opA;
  Operand<B_TR> opB;
  const uint32_t sbase = lds_u32(smem);
  opA.init(A + (A_TR ? (int64_t)t0 * 64 * lda : (int64_t)t0 * 64), lda, m0, w, lane, wm, 64, sbase);
  opB.init(B + (B_TR ? (int64_t)t0 * 64 * ldb : (int64_t)t0 * 64), ldb, n0, w, lane, wn, 32,
           sbase + B_REGION);

  constexpr bool CS = (EPI == EPI_ATOMIC_F32) && A_TR;
  const bool do_cs = CS && colsum != nullptr && nt == 0;
  float cs = 0.f;

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa[4][2], fb0[2][2], fb1[2][2];
  // colsum transposed-read bases: lane 4q+p of its 16-lane group addresses row
  // 32*(t>>7) + 4r + q, columns 16*((t>>4)&7) + 4p .. +3
  uint32_t csa[2];
  {
    const int t = tid & 255, q = (lane & 15) >> 2, p = lane & 3;
#pragma unroll
    for (int b3 = 0; b3 < 2; ++b3) {
      const int row = q + 8 * b3;  // tr_x depends on row & 3 and row bit 3 only
      const int ch = (2 * ((t >> 4) & 7) + (p >> 1)) ^ tr_x(row);
      csa[b3] = sbase + (uint32_t)((32 * (t >> 7) + q) * 256 + ch * 16 + (p & 1) * 8);
    }
  }

  // prologue: K-tile 0 complete; K-tile 1 halves A0, B0 in flight
  char* const smB = smem + B_REGION;
  opA.stage(smem + img_off(0, 0), 0, 0);
  opB.stage(smB + img_off(0, 0), 0, 0);
  opB.stage(smB + img_off(0, 1), 1, 0);
  opA.stage(smem + img_off(0, 1), 1, 0);
  opA.stage(smem + img_off(1, 0), 0, 1);
  opB.stage(smB + img_off(1, 0), 0, 1);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // K-tile 0 halves A0, B0 landed
  barrier();
  if (grp == 1) barrier();

  const int niter = nk >> 1;
  for (int it = 0; it < niter; ++it) {
    const int te = 2 * it;
    const bool more = it + 1 < niter;
    phase<0, A_TR, B_TR, CS>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, do_cs, grp);
    phase<1, A_TR, B_TR, CS>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, do_cs, grp);
    phase<2, A_TR, B_TR, CS>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, do_cs, grp);
    phase<3, A_TR, B_TR, CS>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, do_cs, grp);
    phase<4, A_TR, B_TR, CS>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, do_cs, grp);
    phase<5, A_TR, B_TR, CS>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, do_cs, grp);
    phase<6, A_TR, B_TR, CS>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, do_cs, grp);
    phase<7, A_TR, B_TR, CS>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, do_cs, grp);
  }
  if (grp == 0) barrier();  // re-align the groups; all LDS reads are retired past here

  // ---- epilogue: acc[qa][qb][i][j] reg r -> row qa*128 + wm*64 + i*16 + 4*(lane>>4) + r,
  //                                           col qb*128 + wn*32 + j*16 + (lane&15)
  const int g4 = (lane >> 4) * 4, li = lane & 15;
  if constexpr (EPI == EPI_NONE) {
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) asm volatile("" ::"v"(acc[qa][qb][i][j]));
  } else if constexpr (EPI == EPI_ATOMIC_F32) {
    if (do_cs) {
      float* red = reinterpret_cast<float*>(smem);  // [2 row halves][256 cols]
      const int t = tid & 255;
      red[(t >> 7) * 256 + grp * 128 + (t & 127)] = cs;
      __syncthreads();
      // split-K: this slab's bias partial into the workspace's [slabs][M] tail (summed in slab
      // order by the launcher's reduce, no atomics); one slab: the only adder of these rows
      if (tid < 256) {
        if (wsp) wsp[(int64_t)splits * nseg * M * N + (int64_t)z * M + m0 + tid] = red[tid] + red[256 + tid];
        else colsum[m0 + tid] += red[tid] + red[256 + tid];
      }
    }
    // Stage each 128-row half of the fp32 tile in LDS ([128][256], 16-float blocks
    // XOR-swizzled by row & 3), then add it with fully coalesced atomics (a wave
    // covers 256 contiguous bytes of one gradient row).
    float* ct = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int qa = 0; qa < 2; ++qa) {
      __syncthreads();
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = wm * 64 + i * 16 + g4 + r;
              const int col = (qb * 128 + wn * 32 + j * 16 + li) ^ ((row & 3) << 4);
              ct[row * 256 + col] = acc[qa][qb][i][j][r];
            }
      __syncthreads();
      if (wsp) {
        // split-K partial of split z into the workspace [splits][M][N] with plain 16-B
        // stores (HBM rate); wgrad_reduce_kernel adds the splits into Cf afterwards
        float* dst = wsp + ((int64_t)z * M + m0 + qa * 128) * N + n0;
#pragma unroll 4
        for (int c = 0; c < 16; ++c) {
          const int idx = tid + c * 512;
          const int row = idx >> 6, col = (idx & 63) * 4;
          const f32x4 v = *reinterpret_cast<const f32x4*>(ct + row * 256 + (col ^ ((row & 3) << 4)));
          *reinterpret_cast<f32x4*>(dst + (int64_t)row * N + col) = v;
        }
      } else {
        float* dst = Cf + (int64_t)(m0 + qa * 128) * ldc + n0;
#pragma unroll 4
        for (int c = 0; c < 64; ++c) {
          const int idx = tid + c * 512;
          const int row = idx >> 8, col = idx & 255;
          atomicAdd(dst + (int64_t)row * ldc + col, ct[row * 256 + (col ^ ((row & 3) << 4))]);
        }
      }
    }
  } else {
    constexpr int LDC = 264;  // padded staging row (elements)
    bf16_t* ct = reinterpret_cast<bf16_t*>(smem);
    float bv[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
    if (EPI == EPI_BIAS_ACT && bias) {
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int j = 0; j < 2; ++j) bv[qb][j] = bf2f(bias[n0 + qb * 128 + wn * 32 + j * 16 + li]);
    }
#pragma unroll
    for (int qa = 0; qa < 2; ++qa) {
      if (qa) __syncthreads();  // previous half's rows have been stored
      // EPI_DACT: fetch this half's activation-backward operand before staging, so
      // its latency overlaps the LDS round trip
      uint4 av[8];
      if constexpr (EPI == EPI_DACT) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const int idx = tid + c * 512;
          const int64_t o = (int64_t)(m0 + qa * 128 + (idx >> 5)) * ldc + n0 + (idx & 31) * 8;
          av[c] = *reinterpret_cast<const uint4*>(Zout + o);
        }
      }
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = wm * 64 + i * 16 + g4 + r;
              const int col = qb * 128 + wn * 32 + j * 16 + li;
              ct[row * LDC + col] = f2bf(acc[qa][qb][i][j][r] + bv[qb][j]);
            }
      __syncthreads();
      // 128 rows x 32 chunks of 8 elements
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int idx = tid + c * 512;
        const int row = idx >> 5, ch = idx & 31;
        uint4 v = *reinterpret_cast<const uint4*>(ct + row * LDC + ch * 8);
        const int64_t o = (int64_t)(m0 + qa * 128 + row) * ldc + n0 + ch * 8;
        if constexpr (EPI == EPI_DACT) {
          uint32_t wv[4] = {v.x, v.y, v.z, v.w};
          const uint32_t aw[4] = {av[c].x, av[c].y, av[c].z, av[c].w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float lo = __uint_as_float(wv[q] << 16) * dact_f(__uint_as_float(aw[q] << 16), act);
            const float hi = __uint_as_float(wv[q] & 0xffff0000u) *
                             dact_f(__uint_as_float(aw[q] & 0xffff0000u), act);
            wv[q] = pack_bf2(lo, hi);
          }
          v = make_uint4(wv[0], wv[1], wv[2], wv[3]);
        }
        if (EPI == EPI_BIAS_ACT && act != 0) {
          if (Zout) *reinterpret_cast<uint4*>(Zout + o) = v;
          uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float lo = act_f(__uint_as_float(wv[q] << 16), act);
            const float hi = act_f(__uint_as_float(wv[q] & 0xffff0000u), act);
            wv[q] = pack_bf2(lo, hi);
          }
          v = make_uint4(wv[0], wv[1], wv[2], wv[3]);
        }
        *reinterpret_cast<uint4*>(C + o) = v;
      }
    }
  }
}

// ---- grouped weight gradient (one launch per deferral flush) -----------------
// The reference schedule's deferred weight gradients (ops/nn.py _WgradDeferral) of EVERY Linear
// of a flush in one launch: the sites together have ~1300 256 x 256 tiles, ~5 rounds of the 256
// CUs, so no tile is split over the tokens.  Workgroup = one tile of one site; it walks all of
// the site's token segments (a prologue + 8-phase main loop each) with its accumulators live and
// adds the tile into dW with a plain read-add-write: one writer per element, no split-K slabs,
// no reduce pass, deterministic.  The site table lives in device memory (uniform scalar loads).
__global__ void __launch_bounds__(512) wgrad_group_kernel(const WgGroupSite* __restrict__ sites, int nsites,
                                                          int ntiles) {
  static_assert(WG_MAXSEG == 8, "WgGroupSite holds 8 segments");
  __shared__ __attribute__((aligned(1024))) char smem[2 * B_REGION];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = (w >> 2) & 1, wn = w & 3;
  const int grp = __builtin_amdgcn_readfirstlane(w >> 2);
  const int tile = xcd_remap(blockIdx.x, ntiles);
  int si = 0;
  for (int i = 1; i < nsites; ++i)
    if (sites[i].tile0 <= tile) si = i;
  const WgGroupSite* st = sites + si;
  const int M = st->M, N = st->N, nseg = st->nseg, ktiles = st->ktiles;
  float* const dW = st->dW;
  float* const colsum = st->colsum;
  const int local = tile - st->tile0, NT = N / 256;
  const int mt = local / NT, nt = local - mt * NT;
  const int m0 = mt * 256, n0 = nt * 256;
  const bool do_cs = colsum != nullptr && nt == 0;
  float cs = 0.f;

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa[4][2], fb0[2][2], fb1[2][2];
  const uint32_t sbase = lds_u32(smem);
  uint32_t csa[2];
  {
    const int t = tid & 255, q = (lane & 15) >> 2, p = lane & 3;
#pragma unroll
    for (int b3 = 0; b3 < 2; ++b3) {
      const int row = q + 8 * b3;
      const int ch = (2 * ((t >> 4) & 7) + (p >> 1)) ^ tr_x(row);
      csa[b3] = sbase + (uint32_t)((32 * (t >> 7) + q) * 256 + ch * 16 + (p & 1) * 8);
    }
  }
  char* const smB = smem + B_REGION;
  const int niter = ktiles >> 1;
  for (int sg = 0; sg < nseg; ++sg) {
    Operand<true> opA;
    Operand<true> opB;
    opA.init((const bf16_t*)st->a[sg], M, m0, w, lane, wm, 64, sbase);
    opB.init((const bf16_t*)st->b[sg], N, n0, w, lane, wn, 32, sbase + B_REGION);
    opA.stage(smem + img_off(0, 0), 0, 0);
    opB.stage(smB + img_off(0, 0), 0, 0);
    opB.stage(smB + img_off(0, 1), 1, 0);
    opA.stage(smem + img_off(0, 1), 1, 0);
    opA.stage(smem + img_off(1, 0), 0, 1);
    opB.stage(smB + img_off(1, 0), 0, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    barrier();
    if (grp == 1) barrier();
    for (int it = 0; it < niter; ++it) {
      const int te = 2 * it;
      const bool more = it + 1 < niter;
      phase<0, true, true, true>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, do_cs, grp);
      phase<1, true, true, true>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, do_cs, grp);
      phase<2, true, true, true>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, do_cs, grp);
      phase<3, true, true, true>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, do_cs, grp);
      phase<4, true, true, true>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, do_cs, grp);
      phase<5, true, true, true>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, do_cs, grp);
      phase<6, true, true, true>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, do_cs, grp);
      phase<7, true, true, true>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, do_cs, grp);
    }
    if (grp == 0) barrier();  // re-align the groups; every LDS read of this segment is retired
  }

  // epilogue: bias column sums (one workgroup per tile row: a single adder per element), then each
  // 128-row half of the fp32 tile staged in LDS and added into dW with 16-B read-add-writes
  const int g4 = (lane >> 4) * 4, li = lane & 15;
  if (do_cs) {
    float* red = reinterpret_cast<float*>(smem);
    const int t = tid & 255;
    red[(t >> 7) * 256 + grp * 128 + (t & 127)] = cs;
    __syncthreads();
    if (tid < 256) colsum[m0 + tid] += red[tid] + red[256 + tid];
  }
  float* ct = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int qa = 0; qa < 2; ++qa) {
    __syncthreads();
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = wm * 64 + i * 16 + g4 + r;
            const int col = (qb * 128 + wn * 32 + j * 16 + li) ^ ((row & 3) << 4);
            ct[row * 256 + col] = acc[qa][qb][i][j][r];
          }
    __syncthreads();
    float* dst = dW + (int64_t)(m0 + qa * 128) * N + n0;
#pragma unroll 4
    for (int c = 0; c < 16; ++c) {
      const int idx = tid + c * 512;
      const int row = idx >> 6, col = (idx & 63) * 4;
      const f32x4 v = *reinterpret_cast<const f32x4*>(ct + row * 256 + (col ^ ((row & 3) << 4)));
      f32x4* d = reinterpret_cast<f32x4*>(dst + (int64_t)row * N + col);
      *d = *d + v;
    }
  }
}

// ---- persistent variant (forward / data-gradient GEMMs) ----------------------
//
// One workgroup per CU walks tiles tile = first, first + G, ... (G = grid).  What it
// fixes (measured in tools/gemm_lab, profiles/gemm_lab_r2.txt): the non-persistent
// kernel's 128 KiB output tile per CU costs ~25% of a K = 768 GEMM, because
//  (a) a store instruction that covers 16 rows x 64 B (the MFMA accumulator layout,
//      half cache lines) drains at ~33 GB/s per CU, while 8 rows x 128 B (full lines)
//      drains at ~111 GB/s per CU - the epilogue is store-issue bound, and
//  (b) the next tile's first loads queue behind those stores.
// So:
//  * the MFMAs run transposed (SWAP): a lane holds 4 consecutive columns of one row,
//    and v_permlane16_swap pairs two such 16-column blocks into 16 contiguous bytes;
//  * the B operand is remapped (Operand::init remap) so each wave owns 64 CONTIGUOUS
//    output columns; each wave transposes its 16-row x 64-column blocks through a
//    private 2 KiB LDS slot (no workgroup barrier) and stores full 128-B lines;
//  * the NEXT tile's prologue DMA is issued before the epilogue, and the waits of the
//    first half of its first K-iteration leave the XS epilogue ops in flight;
//  * the bias of each tile comes into a double-buffered 512-B LDS slot by one DMA per
//    wave in the prologue (uniform op counts per wave).
// EPI: 0 plain (+bias), 1 act(x+bias) (y only), 2 y = act(z), z = x+bias (both stored),
// 3 x * act'(aux) (data gradient fused with the previous layer's activation backward;
// aux = pre-activation z for gelu/silu, the output y for tanh), 5 x + aux (a residual-
// branch gradient accumulated by the GEMM; aux may alias C), 4 = 3 plus the column
// sums of the result (that layer's bias gradient) as per-(tile, 128-row half) partials
// colpart[(M/256)*2][N] (reduced by the caller).  ACT: act.h code.  Activations are
// applied to the bf16-rounded value, exactly as a separate elementwise pass would.
constexpr int P_BIAS_OFF = 2 * B_REGION;         // 2 x 512 B bias slots after the operand images
constexpr int P_STAGE_OFF = 2 * B_REGION + 1024;  // 8 waves x 2 KiB epilogue transpose slots
constexpr int P_NEXT_OFF = P_STAGE_OFF + 8 * 2048;  // dynamic schedule: next tile index
constexpr int P_LDS = P_NEXT_OFF + 16;

template <int EPI>
struct PEpi {
  // VMEM ops each lane issues after the next tile's prologue DMA: 16 stores (8 rounds x 2),
  // EPI 2 a second 16 (z and y), EPI 3/4 the 12 aux loads of rounds 2..7, EPI 4 two partial stores
  static constexpr int XS = (EPI == 2 || EPI == 6 || EPI == 8) ? 32 : (EPI == 3 || EPI == 5 || EPI == 7) ? 28
                            : EPI == 4 ? 30 : 16;
  // 128-row tiles: 4 rounds (8 stores, EPI 2/6/8 16; aux loads of rounds 2..3)
  static constexpr int XS_H = (EPI == 2 || EPI == 6 || EPI == 8) ? 16 : (EPI == 3 || EPI == 5 || EPI == 7) ? 12 : 8;
};

template <int ACT>
__device__ __forceinline__ float act_t(float z) { return act_apply(z, ACT); }
template <int ACT>
__device__ __forceinline__ float dact_t(float a) { return act_deriv(a, ACT); }

typedef __attribute__((ext_vector_type(4))) unsigned u32x4_v;
__device__ __forceinline__ void lds_write_b128(uint32_t addr, const uint4& v) {
  const u32x4_v x = {v.x, v.y, v.z, v.w};
  asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(x) : "memory");
}
__device__ __forceinline__ uint4 lds_read_b128_sync(uint32_t addr) {
  u32x4_v v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  return make_uint4(v[0], v[1], v[2], v[3]);
}

// 8 bf16 (one uint4) -> act(z) (returned) and act'(z) (d), on packed float pairs
template <int ACT>
__device__ __forceinline__ uint4 act_dact8(const uint4& u, uint4& dv) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
  uint32_t o[4], g[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f32x2 d;
    const f32x2 y = act_dact2<ACT>(f32x2{__uint_as_float(w[q] << 16), __uint_as_float(w[q] & 0xffff0000u)}, d);
    o[q] = pack_bf2(y.x, y.y);
    g[q] = pack_bf2(d.x, d.y);
  }
  dv = make_uint4(g[0], g[1], g[2], g[3]);
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// 8 bf16 (one uint4) -> act on packed float pairs -> 8 bf16
template <int ACT>
__device__ __forceinline__ uint4 act8(const uint4& u) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
  uint32_t o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x2 y = act2<ACT>(f32x2{__uint_as_float(w[q] << 16), __uint_as_float(w[q] & 0xffff0000u)});
    o[q] = pack_bf2(y.x, y.y);
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// act'(z) as an 8-bit code (EPI 8 stores it, ACT 5 epilogues read it), two linear segments
// meeting at code 93 = act' 0.5:
//   c in [0, 93]:    act' = (c - 19) * 0.5 / 74        -> [-0.1284, 0.5], step 0.0068
//   c in [93, 255]:  act' = (c + 35) / 256             -> [0.5, 1.1328],  step 2^-8
// The upper segment's grid IS bf16's grid on [0.5, 1) (and finer on [1, 1.13]), so every act'
// >= 0.5 is stored exactly as a bf16 act' would be; 0 (code 19) and 1 (code 221) - the
// saturated regions, most elements of a trained layer - are exact; below 0.5 within 0.0034.
// Covers gelu' [-0.129, 1.129] (its minimum clamped by 0.0006), silu' [-0.0998, 1.0998] and
// tanh' [0, 1].  Half the bytes of the bf16 act' the forward writes and the backward reads.
// The segments are convex / concave at the joint, so the code is the max of the two lines'
// codes and the value the min of the two lines' values (no compare / select).
constexpr float Q8_LO_STEP = 0.5f / 74.f;
// The codes of an act' pair: both lines of both elements on packed fp32 (two v_pk_fma_f32) and
// one max per element; v_cvt_pk_u8_f32 then rounds to nearest (no explicit rint).  No clamp is
// needed: every act' this encodes (gelu', silu', tanh') lies in [-0.1285, 1.13], i.e. codes in
// [-0.02, 254.6].  DPA_Q8_CVT: 1 (default) = the conversion rounds to nearest; 0 = explicit rint.
#ifndef DPA_Q8_CVT
#define DPA_Q8_CVT 1
#endif
__device__ __forceinline__ f32x2 q8_codes2(f32x2 d) {
  const f32x2 l1 = d * 148.f + 19.f;
  const f32x2 l2 = d * 256.f - 35.f;
  f32x2 c = {fmaxf(l1.x, l2.x), fmaxf(l1.y, l2.y)};
  if constexpr (DPA_Q8_CVT == 0) c = f32x2{__builtin_rintf(c.x), __builtin_rintf(c.y)};
  return c;
}

// 8 bf16 -> act(z) (returned, bf16) and act'(z) as 8 u8 codes (c)
template <int ACT>
__device__ __forceinline__ uint4 act_dact8q(const uint4& u, uint2& c) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
  uint32_t o[4], cw[2] = {0u, 0u};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f32x2 d;
    const f32x2 y = act_dact2<ACT>(f32x2{__uint_as_float(w[q] << 16), __uint_as_float(w[q] & 0xffff0000u)}, d);
    o[q] = pack_bf2(y.x, y.y);
    const f32x2 cc = q8_codes2(d);
    cw[q >> 1] = __builtin_amdgcn_cvt_pk_u8_f32(cc.x, (q & 1) * 2, cw[q >> 1]);
    cw[q >> 1] = __builtin_amdgcn_cvt_pk_u8_f32(cc.y, (q & 1) * 2 + 1, cw[q >> 1]);
  }
  c = make_uint2(cw[0], cw[1]);
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// decoded act' of elements 2q, 2q + 1 of an 8-code group: min((c - 19) * 0.5 / 74, (c + 35) / 256)
// on packed fp32 (the same roundings as the element-wise form, so 0 and 1 stay exact)
__device__ __forceinline__ f32x2 q8_pair(const uint4& a, int q) {
  const uint32_t c = (q >> 1) ? a.y : a.x;
  const int sh = (q & 1) * 16;
  const f32x2 cv = {(float)((c >> sh) & 0xffu), (float)((c >> (sh + 8)) & 0xffu)};
  const f32x2 lo = (cv - 19.f) * Q8_LO_STEP;
  const f32x2 hi = cv * (1.f / 256.f) + 35.f / 256.f;
  return f32x2{fminf(lo.x, hi.x), fminf(lo.y, hi.y)};
}

__device__ __forceinline__ void lds_write_b32(uint32_t addr, int v) {
  asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(addr), "v"(v) : "memory");
}
__device__ __forceinline__ int lds_read_b32_sync(uint32_t addr) {
  int v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  return v;
}

__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// Early issue of the DACT epilogue's first aux rounds inside the last K-iteration
// (DPA_GEMM_EARLY_AUX at compile time; 1 = on)
#ifndef DPA_GEMM_EARLY_AUX
#define DPA_GEMM_EARLY_AUX 1
#endif
constexpr int PEARLY_AUX = DPA_GEMM_EARLY_AUX;

// Lab knobs (tools/gemm_lab; the library uses the defaults): POL bit 0 = non-temporal
// epilogue stores, bit 1 = non-temporal aux loads; GM > 1 walks tiles in groups of GM tile
// rows, column-major inside a group (GM x NT tiles share GM A panels and NT B panels).
template <int POL>
__device__ __forceinline__ void st_out(bf16_t* p, const uint4& v) {
  if constexpr (POL & 4) {
    // write-through: the line is not allocated in the XCD's L2, which keeps the operand
    // panels the next tiles read resident (s_nop 1: the data registers must not be
    // overwritten before the store has read them - hipcc pads nothing inside an asm)
    const u32x4_v x = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(x) : "memory");
  } else if constexpr (POL & 1) {
    const u32x4_v x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<u32x4_v*>(p));
  } else {
    *reinterpret_cast<uint4*>(p) = v;
  }
}
template <int POL>
__device__ __forceinline__ uint4 ld_aux(const bf16_t* p) {
  if constexpr (POL & 2) {
    const u32x4_v x = __builtin_nontemporal_load(reinterpret_cast<const u32x4_v*>(p));
    return make_uint4(x[0], x[1], x[2], x[3]);
  } else {
    return *reinterpret_cast<const uint4*>(p);
  }
}
typedef __attribute__((ext_vector_type(2))) unsigned u32x2_v;
template <int POL>
__device__ __forceinline__ void st_out8(uint8_t* p, const uint2& v) {
  if constexpr (POL & 1) {
    __builtin_nontemporal_store(u32x2_v{v.x, v.y}, reinterpret_cast<u32x2_v*>(p));
  } else {
    *reinterpret_cast<uint2*>(p) = v;
  }
}
template <int POL>
__device__ __forceinline__ uint2 ld_aux8(const uint8_t* p) {
  if constexpr (POL & 2) {
    const u32x2_v x = __builtin_nontemporal_load(reinterpret_cast<const u32x2_v*>(p));
    return make_uint2(x[0], x[1]);
  } else {
    return *reinterpret_cast<const uint2*>(p);
  }
}

// Epilogue parameters beyond the operands: the residual-dropout epilogue (EPI 7) draws its
// dropout bits from pair_hash (common.h) with the seed mix of (seed, offset + device base).
struct EpiArgs {
  uint32_t seed = 0, offset = 0, thr16 = 0;
  float scale = 1.f;
};

template <int GM>
__device__ __forceinline__ void tile_mn(int t, int NT, int& mt, int& nt) {
  if constexpr (GM <= 1) {
    mt = t / NT;
    nt = t - mt * NT;
  } else {
    const int gs = GM * NT, g = t / gs, r = t - g * gs;
    mt = g * GM + r % GM;
    nt = r / GM;
  }
}

template <bool B_TR, int EPI, int ACT, int POL = 0, int GM = 1, int STG = 0, int DU = 0, bool HMT = false>
__global__ void __launch_bounds__(512) gemmp_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                    const bf16_t* __restrict__ B, int64_t ldb, int M, int N,
                                                    int nk, bf16_t* __restrict__ C, int64_t ldc,
                                                    const bf16_t* __restrict__ bias,
                                                    bf16_t* __restrict__ Zout, float* __restrict__ colpart,
                                                    int* __restrict__ tile_ctr, int hm, EpiArgs ea) {
  __shared__ __attribute__((aligned(1024))) char smem[P_LDS];
  // HMT: 128 x 256 tiles (twice the tiles of a small-T launch: the reference schedule's
  // 8192-token micro-batches give a 768-wide layer 96 256-row tiles for 256 CUs)
  static_assert(!(HMT && EPI == 4), "column-sum partials are laid out per 256-row tile");
  constexpr int TM = HMT ? 128 : 256, NRO = HMT ? 4 : 8;
  constexpr int XS = HMT ? PEpi<EPI>::XS_H : PEpi<EPI>::XS;
  constexpr bool DACT = EPI == 3 || EPI == 4 || EPI == 5;  // data-gradient epilogues reading aux
  constexpr bool AUXR = DACT || EPI == 7;                  // epilogues that read aux
  constexpr bool Q8 = DACT && ACT == 5;                    // aux = act' as tile-native u8 codes
  static_assert(!(EPI == 8 && ACT == 0), "EPI 8 stores an activation derivative");
  // wave id in an SGPR, lane id re-derived from EXEC wherever needed: nothing
  // lane-dependent has to stay live across the register-full main loop
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = (w >> 2) & 1, wn = w & 3;
  const int grp = w >> 2;
  const int NT = N / 256, ntiles = (M / TM) * NT;
  const int G = gridDim.x;
  const uint32_t sbase = lds_u32(smem);
  char* const smB = smem + B_REGION;
  const int niter = nk >> 1;
  const bool has_bias = bias != nullptr;

  Operand<false> opA;
  Operand<B_TR> opB;
  f32x4 acc[2][2][4][2];
  bf16x8 fa[4][2], fb0[2][2], fb1[2][2];
  float cs = 0.f;
  const uint32_t csa[2] = {0u, 0u};

  auto prologue = [&](int t, int slot) {
    int mt, nt;
    tile_mn<GM>(t, NT, mt, nt);
    const int lane = lane_id();
    opA.init(A, lda, mt * TM, w, lane, wm, 64, sbase);
    if constexpr (HMT) opA.hstep = 0;  // the A1 half image re-reads rows 0..127 (L2 hits)
    opB.init(B, ldb, nt * 256, w, lane, wn, 32, sbase + B_REGION, /*remap=*/true);
    // bias slot: the tile's 256 bf16 = 2 x (64 lanes x 4 B); every wave issues one such
    // DMA (waves of equal parity write identical bytes) so the vmcnt counts stay uniform
    const int bh = (w & 1) * 256;
    const char* bsrc = (has_bias ? reinterpret_cast<const char*>(bias + nt * 256)
                                 : reinterpret_cast<const char*>(A)) + bh + lane * 4;
    __builtin_amdgcn_global_load_lds((glob_void*)bsrc, (lds_void*)(smem + P_BIAS_OFF + slot * 512 + bh),
                                     4, 0, 0);
    opA.stage(smem + img_off(0, 0), 0, 0);
    opB.stage(smB + img_off(0, 0), 0, 0);
    opB.stage(smB + img_off(0, 1), 1, 0);
    opA.stage(smem + img_off(0, 1), 1, 0);
    opA.stage(smem + img_off(1, 0), 0, 1);
    opB.stage(smB + img_off(1, 0), 0, 1);
  };

  // Epilogue rounds ro = qa*4 + i (0..7): this wave's rows qa*128 + wm*64 + i*16 + (0..15) of
  // the tile, its 64 columns wn*64 + (0..63).  In the row-major domain (after the LDS
  // transpose) lane l handles rows 8k + (l >> 3) (k = 0, 1) of the round, columns 8 (l & 7) .. +7.
  auto row_off = [&](int t, int ro, int k, int ln) -> int64_t {
    int mt, nt;
    tile_mn<GM>(t, NT, mt, nt);
    const int qa = ro >> 2, i = ro & 3;
    const int lrow = qa * 128 + wm * 64 + i * 16 + k * 8 + (ln >> 3);  // row within the tile, < 256
    const int col = nt * 256 + wn * 64 + (ln & 7) * 8;
    if (EPI == 0 && hm) {
      // head-major store [R >> hm][ldc / 64][1 << hm][64]: row = (b, l), col = (head j, d); a
      // wave's 64 columns are one head, so a store instruction's 8 rows are 1 KiB contiguous
      const int64_t row = (int64_t)mt * TM + lrow;
      const int64_t b = row >> hm, l = row & ((1 << hm) - 1);
      return ((b * (ldc >> 6) + (col >> 6)) << hm) * 64 + l * 64 + (col & 63);
    }
    // the tile origin's 64-bit offset is wave-uniform (scalar); the in-tile row takes one
    // full-rate 24-bit multiply (lrow < 256, ldc < 2^24) instead of a 64-bit one per address
    return (int64_t)(mt * TM) * ldc + (int64_t)__umul24((unsigned)lrow, (unsigned)ldc) + col;
  };
  // Tile-native byte offset of a u8 act' code group (EPI 8 writes, ACT 5 reads): the 8 codes
  // of (tile, wave, round, k, lane) are consecutive, so one wave instruction moves 512
  // contiguous bytes (the row-major u8 layout would give half-line 64-B row segments).  Both
  // kernels tile the same [T][N] matrix with the same 256 x 256 tiles and wave / lane roles.
  auto q8_off = [&](int t, int ro, int k, int ln) -> int64_t {
    int mt, nt;
    tile_mn<GM>(t, NT, mt, nt);
    if constexpr (HMT) {  // the 256-row tile's layout: 128-row tile mt is its rounds (mt & 1) * 4 + ro
      ro += (mt & 1) * 4;
      mt >>= 1;
    }
    return (((((int64_t)mt * NT + nt) * 8 + w) * 8 + ro) * 2 + k) * 512 + ln * 8;
  };
  auto load_aux = [&](int t, int ro, int k, int ln) -> uint4 {
    if constexpr (Q8) {
      const uint2 v = ld_aux8<POL>(reinterpret_cast<const uint8_t*>(Zout) + q8_off(t, ro, k, ln));
      return make_uint4(v.x, v.y, 0u, 0u);
    } else {
      return ld_aux<POL>(Zout + row_off(t, ro, k, ln));
    }
  };
  const uint32_t dsm = EPI == 7 ? pair_seedmix(ea.seed, ea.offset + rng_base()) : 0u;

  auto epilogue = [&](int t, int slot, uint4 (&aux)[2][2], bool has_next) {
    // lane-derived addressing recomputed here from an opaque lane id: hoisted out of
    // the tile loop it would be live across the main loop and spill
    const int ln = opaque(lane_id());
    const int R = ln >> 4, li = ln & 15;
    const int cofs = ((R & 1) << 4) | ((R >> 1) << 3);  // after the permlane16 swap
    const uint32_t bslot = sbase + P_BIAS_OFF + slot * 512;
    const uint32_t stg = sbase + P_STAGE_OFF + w * 2048;
    const int rr = ln >> 3, ch = ln & 7;
    float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float bv[2][2][4];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (!DACT && has_bias) {
          // asm read: a compiler-visible LDS read here would be ordered behind the
          // next tile's in-flight DMA (vmcnt(0)); the bias slot was retired long ago
          uint2 b2;
          asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                       : "=v"(b2) : "v"(bslot + (uint32_t)(wn * 64 + qb * 32 + j * 16 + 4 * R) * 2));
          bv[qb][j][0] = bf_lo(b2.x); bv[qb][j][1] = bf_hi(b2.x);
          bv[qb][j][2] = bf_lo(b2.y); bv[qb][j][3] = bf_hi(b2.y);
        } else {
          bv[qb][j][0] = bv[qb][j][1] = bv[qb][j][2] = bv[qb][j][3] = 0.f;
        }
      }
#pragma unroll
    for (int ro = 0; ro < NRO; ++ro) {
      const int qa = ro >> 2, i = ro & 3;
      // stage: pack (+bias), permlane16 swap, one 16-B row segment per qb
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        float v[2][4];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) v[j][r] = acc[qa][qb][i][j][r] + bv[qb][j][r];
        uint32_t x0 = pack_bf2(v[0][0], v[0][1]), x1 = pack_bf2(v[0][2], v[0][3]);
        uint32_t y0 = pack_bf2(v[1][0], v[1][1]), y1 = pack_bf2(v[1][2], v[1][3]);
        auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
        auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
        const int lchunk = qb * 4 + (cofs >> 3);
        lds_write_b128(stg + li * 128 + ((lchunk ^ (li & 7)) << 4), make_uint4(s0[0], s1[0], s0[1], s1[1]));
      }
      // read back row-major (the wave's own LDS ops complete in order) and store full lines
      uint4 val[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int row = k * 8 + rr;
        val[k] = lds_read_b128_sync(stg + row * 128 + ((ch ^ (row & 7)) << 4));
      }
      if constexpr (AUXR) {
        // wait for this round's aux.  Issue order: aux(0) aux(1) [DMA: 13] | r0: wait aux(2)
        // st(0) | r1: wait aux(3) st(1) | ... | r5: wait aux(7) st(5) | r6: wait st(6) | r7: wait
        // st(7); the ops younger than aux(ro) at its wait (2 each; the DMA only when there is
        // a next tile):  ro 0: aux1 DMA;  ro 1: DMA aux2 st0;  ro 2..6: st(ro-2) aux(ro+1)
        // st(ro-1);  ro 7: st5 st6
        if (ro == 0) {
          if (has_next) wait_vm<15>(); else wait_vm<2>();
        } else if (ro == 1) {
          if (has_next) wait_vm<17>(); else wait_vm<4>();
        } else if (ro < NRO - 1) {
          wait_vm<6>();
        } else {
          wait_vm<4>();  // the last round: no aux(ro + 1) was issued after it
        }
        // pair_hash(dsm, row, col) = mix32(dsm ^ row A ^ (col / 2) B) with row = drow + 8 k and
        // col / 2 = dcol / 2 + q: the two products strength-reduced to one per round (rA) and one
        // per tile (cB) plus constant offsets (v_mul_lo_u32 is quarter rate)
        uint32_t rA = 0, cB = 0;
        if constexpr (EPI == 7) {
          int mt, nt;
          tile_mn<GM>(t, NT, mt, nt);
          rA = (uint32_t)(mt * TM + qa * 128 + wm * 64 + i * 16 + (ln >> 3)) * 0x9E3779B1u;
          cB = (uint32_t)((nt * 256 + wn * 64 + (ln & 7) * 8) >> 1) * 0x85EBCA77u;
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const uint4 a = aux[ro & 1][k];
          const uint32_t aw[4] = {a.x, a.y, a.z, a.w};
          const uint32_t vw[4] = {val[k].x, val[k].y, val[k].z, val[k].w};
          uint32_t o[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const f32x2 x = f32x2{bf_lo(vw[q]), bf_hi(vw[q])};
            f32x2 d;
            if constexpr (Q8) {
              d = x * q8_pair(a, q);
            } else if constexpr (EPI == 7) {
              // h = residual + dropout(y): y = the bf16 GEMM output (+bias), as a separate
              // dropout-add pass would see it; the bits are norm.hip's pair-hash mode's
              const f32x2 r = f32x2{bf_lo(aw[q]), bf_hi(aw[q])};
              const uint32_t hsh = mix32(dsm ^ (rA + (uint32_t)k * (8u * 0x9E3779B1u)) ^
                                         (cB + (uint32_t)q * 0x85EBCA77u));
              const f32x2 m = {(hsh & 0xffffu) >= ea.thr16 ? ea.scale : 0.f, (hsh >> 16) >= ea.thr16 ? ea.scale : 0.f};
              d = x * m + r;
            } else {
              const f32x2 av = f32x2{bf_lo(aw[q]), bf_hi(aw[q])};
              d = EPI == 5 ? x + av : x * dact2<ACT>(av);
            }
            o[q] = pack_bf2(d.x, d.y);
            if constexpr (EPI == 4) {
              csum[2 * q] += bf_lo(o[q]);
              csum[2 * q + 1] += bf_hi(o[q]);
            }
          }
          val[k] = make_uint4(o[0], o[1], o[2], o[3]);
        }
        // this round's aux slot is consumed: prefetch round ro + 2 into it
        if (ro + 2 < NRO) {
#pragma unroll
          for (int k = 0; k < 2; ++k) aux[ro & 1][k] = load_aux(t, ro + 2, k, ln);
        }
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int64_t o = row_off(t, ro, k, ln);
        if constexpr (EPI == 2) st_out<POL>(Zout + o, val[k]);
        if constexpr (EPI == 1 || EPI == 2) val[k] = act8<ACT>(val[k]);
        if constexpr (EPI == 6) {
          uint4 dv;
          val[k] = act_dact8<ACT>(val[k], dv);
          st_out<POL>(Zout + o, dv);
        }
        if constexpr (EPI == 8) {
          uint2 code;
          val[k] = act_dact8q<ACT>(val[k], code);
          st_out8<POL>(reinterpret_cast<uint8_t*>(Zout) + q8_off(t, ro, k, ln), code);
        }
        st_out<POL>(C + o, val[k]);
      }
    }
    if constexpr (EPI == 4) {
      // column sums over this wave's 128 rows: reduce over the 8 lanes sharing a column
      // chunk (lane bits 3, 4, 5), then lanes 0-7 store their 8 columns
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float x = csum[e];
        x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xF, 0xF, true));
        // (a permlane swap of a register with itself is ambiguous under register
        // allocation: cross-row steps go through ds_bpermute)
        x += __shfl_xor(x, 16, 64);
        x += __shfl_xor(x, 32, 64);
        csum[e] = x;
      }
      int mt, nt;
    tile_mn<GM>(t, NT, mt, nt);
      float* dst = colpart + ((int64_t)mt * 2 + wm) * (int64_t)(NT * 256) + nt * 256 + wn * 64 + ch * 8;
      if (ln < 8) {
        *reinterpret_cast<float4*>(dst) = make_float4(csum[0], csum[1], csum[2], csum[3]);
        *reinterpret_cast<float4*>(dst + 4) = make_float4(csum[4], csum[5], csum[6], csum[7]);
      }
    }
  };

  int tile = xcd_remap(blockIdx.x, G);
  if (tile >= ntiles) return;
  // Dynamic schedule (tile_ctr != nullptr, G >= 8): the first tile is static; later ones
  // are claimed from a per-XCD queue (blockIdx % 8, the round-robin dispatch xcd_remap
  // assumes for locality only), item i of queue x = tile (1 + i / |J_x|) G + J_x[i % |J_x|]
  // with J_x the XCD's static column range - the static schedule's tile set, but a
  // workgroup that starts late (its CU held by a concurrent RCCL kernel) just takes fewer
  // tiles instead of finishing last.  Claimed items form a prefix, so the first claim past
  // ntiles ends the workgroup.
  // Self-resetting queues: every workgroup of queue x ends with exactly one claim past the
  // end, then bumps the queue's done counter; the queue's last workgroup (done == qsize - 1:
  // no claim on the queue can follow) zeroes both counters.  A launch leaves its counters as
  // it found them, so a HIP graph that bakes the counter address replays correctly whatever
  // state the host-side slot ring was in at capture.
  const bool dyn = tile_ctr != nullptr && G >= 8;
  int qbase = 0, qsize = 1;
  int* qctr = nullptr;
  if (dyn) {
    const int qg = G >> 3, rg = G & 7, x = blockIdx.x & 7;
    qbase = x < rg ? x * (qg + 1) : rg * (qg + 1) + (x - rg) * qg;
    qsize = x < rg ? qg + 1 : qg;
    qctr = tile_ctr + x * 16;  // one 64-byte line per queue: [0] claims, [1] finished workgroups
  }
  int slot = 0;
  bool extra = false;
  if constexpr (STG > 1) {
    // start-phase stagger: workgroup j of an XCD starts (j % STG) * DU x ~1 us late, so the
    // epilogue store bursts of the workgroups no longer coincide
    const int ph = (blockIdx.x >> 3) % STG;
    for (int i = 0; i < ph * DU; ++i) __builtin_amdgcn_s_sleep(32);
  }
  prologue(tile, slot);
  wait_vm<8>();  // K-tile 0 halves A0, B0 (and the bias slot) landed
  barrier();
  if (grp == 1) barrier();

  while (true) {
    // claim the next tile now (wave 0, lane 0); the result is consumed after the main
    // loop, whose counted waits at most over-wait by this one extra VMEM op
    int claimed = 0;
    if (dyn && w == 0 && lane_id() == 0) claimed = atomicAdd(qctr, 1);
    // first iteration: the previous tile's XS epilogue ops may still be in flight
    {
      const bool more = 1 < niter;
      phase<0, false, B_TR, false, true, XS, 0, HMT, true>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, 0, more, false, grp, extra);
      phase<1, false, B_TR, false, true, XS, 0, HMT, true>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, 0, more, false, grp, extra);
      phase<2, false, B_TR, false, true, XS, 0, HMT, true>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, 0, more, false, grp, extra);
      phase<3, false, B_TR, false, true, XS, 0, HMT, true>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, 0, more, false, grp, extra);
      phase<4, false, B_TR, false, true, 0, 0, HMT>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, 0, more, false, grp);
      phase<5, false, B_TR, false, true, 0, 0, HMT>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, 0, more, false, grp);
      phase<6, false, B_TR, false, true, 0, 0, HMT>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, 0, more, false, grp);
      phase<7, false, B_TR, false, true, 0, 0, HMT>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, 0, more, false, grp);
    }
    // the epilogue's activation-backward operand (EPI 3/4/5) of rounds 0 and 1: issued in the
    // last K-iteration once its DMA is out (phases 2-7 then leave these 4 loads in flight),
    // so their HBM latency hides under that iteration's MFMAs instead of the epilogue's first
    // rounds (niter == 1: issued after the main loop as before)
    uint4 aux[2][2];
    constexpr bool EARLY_AUX = AUXR && (PEARLY_AUX != 0);
    for (int it = 1; it < niter - (EARLY_AUX ? 1 : 0); ++it) {
      const int te = 2 * it;
      const bool more = it + 1 < niter;
      phase<0, false, B_TR, false, true, 0, 0, HMT>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, false, grp);
      phase<1, false, B_TR, false, true, 0, 0, HMT>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, false, grp);
      phase<2, false, B_TR, false, true, 0, 0, HMT>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, false, grp);
      phase<3, false, B_TR, false, true, 0, 0, HMT>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, false, grp);
      phase<4, false, B_TR, false, true, 0, 0, HMT>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, false, grp);
      phase<5, false, B_TR, false, true, 0, 0, HMT>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, false, grp);
      phase<6, false, B_TR, false, true, 0, 0, HMT>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, false, grp);
      phase<7, false, B_TR, false, true, 0, 0, HMT>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, more, false, grp);
    }
    bool aux_issued = false;
    if constexpr (EARLY_AUX) {
      if (niter > 1) {  // the peeled last iteration
        const int te = 2 * (niter - 1);
        phase<0, false, B_TR, false, true, 0, 0, HMT>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, false, false, grp);
        phase<1, false, B_TR, false, true, 0, 0, HMT>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, false, false, grp);
        {
          const int ln = opaque(lane_id());
#pragma unroll
          for (int ro = 0; ro < 2; ++ro)
#pragma unroll
            for (int k = 0; k < 2; ++k) aux[ro][k] = load_aux(tile, ro, k, ln);
        }
        aux_issued = true;
        phase<2, false, B_TR, false, true, 0, 4, HMT>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, false, false, grp);
        phase<3, false, B_TR, false, true, 0, 4, HMT>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, false, false, grp);
        phase<4, false, B_TR, false, true, 0, 4, HMT>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, false, false, grp);
        phase<5, false, B_TR, false, true, 0, 4, HMT>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, false, false, grp);
        phase<6, false, B_TR, false, true, 0, 4, HMT>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, false, false, grp);
        phase<7, false, B_TR, false, true, 0, 4, HMT>(acc, fa, fb0, fb1, cs, opA, opB, smem, csa, te, false, false, grp);
      }
    }
    if (dyn && w == 0) {
      // every wave's main loop ended in vmcnt(0): the claim has landed
      const int i = __builtin_amdgcn_readfirstlane(claimed);
      if (lane_id() == 0) lds_write_b32(sbase + P_NEXT_OFF, (1 + i / qsize) * G + qbase + i % qsize);
    }
    if (grp == 0) barrier();  // re-align the groups: every wave's LDS reads are retired
    const int next = dyn ? __builtin_amdgcn_readfirstlane(lds_read_b32_sync(sbase + P_NEXT_OFF)) : tile + G;
    const bool has_next = next < ntiles;
    if (AUXR && !aux_issued) {
      // activation-backward operand of rounds 0 and 1 (row-major, full lines), issued
      // before the next tile's prologue DMA so that waiting for it leaves the DMA in flight
      const int ln = opaque(lane_id());
#pragma unroll
      for (int ro = 0; ro < 2; ++ro)
#pragma unroll
        for (int k = 0; k < 2; ++k) aux[ro][k] = load_aux(tile, ro, k, ln);
    }
    if (has_next) prologue(next, slot ^ 1);
    epilogue(tile, slot, aux, has_next);
    if (!has_next) {
      if (dyn && w == 0 && lane_id() == 0) {
        // (vector atomics: the counters are reset through the vector memory path)
        if (atomicAdd(qctr + 1, 1) == qsize - 1) {
          atomicExch(qctr, 0);
          atomicExch(qctr + 1, 0);
        }
      }
      break;
    }
    wait_vm<8 + XS>();  // next tile's K-tile 0 halves landed; this tile's epilogue ops may fly
    barrier();
    if (grp == 1) barrier();
    tile = next;
    slot ^= 1;
    extra = true;
  }
}

}  // namespace g256

// Default on; DPA_GEMM256=0 or set_gemm256(false) routes every shape to gemm.hip.
static int g_gemm256 = -1;
void set_gemm256(bool on) { g_gemm256 = on ? 1 : 0; }
static bool g256_enabled() {
  if (g_gemm256 < 0) {
    const char* e = std::getenv("DPA_GEMM256");
    g_gemm256 = (e && e[0] == '0') ? 0 : 1;
  }
  return g_gemm256 != 0;
}

bool launch_gemm256_nt(const uint16_t* x, const uint16_t* W, const uint16_t* bias, uint16_t* y,
                       uint16_t* z, int T, int N, int K, int act, hipStream_t s) {
  if (!g256_enabled() || T % 256 || N % 256 || K % 128 || K < 128) return false;
  hipLaunchKernelGGL((g256::gemm256_kernel<false, false, g256::EPI_BIAS_ACT>),
                     dim3((T / 256) * (N / 256)), dim3(512), 0, s, (const bf16_t*)x, (int64_t)K,
                     (const bf16_t*)W, (int64_t)K, T, N, K / 64, K / 64, 1, (bf16_t*)y, (int64_t)N,
                     nullptr, (const bf16_t*)bias, act, (bf16_t*)z, nullptr);
  return true;
}

bool launch_gemm256_nn(const uint16_t* dy, const uint16_t* W, uint16_t* dx, int T, int N, int K,
                       hipStream_t s) {
  // dx[T][K] = dy[T][N] . W[N][K]: M = T, N' = K, reduction = N
  if (!g256_enabled() || T % 256 || K % 256 || N % 128 || N < 128) return false;
  hipLaunchKernelGGL((g256::gemm256_kernel<false, true, g256::EPI_BF16>),
                     dim3((T / 256) * (K / 256)), dim3(512), 0, s, (const bf16_t*)dy, (int64_t)N,
                     (const bf16_t*)W, (int64_t)K, T, K, N / 64, N / 64, 1, (bf16_t*)dx, (int64_t)K,
                     nullptr, nullptr, 0, nullptr, nullptr);
  return true;
}

bool launch_gemm256_nn_dact(const uint16_t* dy, const uint16_t* W, const uint16_t* aux,
                            uint16_t* dz, int T, int N, int K, int act, hipStream_t s) {
  // dz[T][K] = (dy[T][N] . W[N][K]) * act'(aux[T][K])
  if (!g256_enabled() || T % 256 || K % 256 || N % 128 || N < 128) return false;
  hipLaunchKernelGGL((g256::gemm256_kernel<false, true, g256::EPI_DACT>),
                     dim3((T / 256) * (K / 256)), dim3(512), 0, s, (const bf16_t*)dy, (int64_t)N,
                     (const bf16_t*)W, (int64_t)K, T, K, N / 64, N / 64, 1, (bf16_t*)dz, (int64_t)K,
                     nullptr, nullptr, act, (bf16_t*)aux, nullptr);
  return true;
}

// ---- persistent forward / data-gradient launchers ---------------------------
// Grid cap of the persistent kernels (0 = none): the overlapped micro-batch schedule caps the
// forward stream's GEMMs so the concurrent backward's kernels find free CUs.
static int g_gemmp_grid_cap = 0;
void set_gemmp_grid_cap(int cap) { g_gemmp_grid_cap = cap > 0 ? cap : 0; }
static int persistent_grid(int tiles, int ncu) {
  if (g_gemmp_grid_cap > 0 && g_gemmp_grid_cap < ncu) ncu = g_gemmp_grid_cap;
  return tiles < ncu ? tiles : ncu;
}

// Dynamic tile schedule of the persistent kernels (see gemmp_kernel): on when the
// compute stream shares the chip with collectives (the DDP engine turns it on for
// world > 1; DPA_GEMMP_DYNAMIC=0/1 overrides).  Queue counters: one small device buffer
// per device, zeroed on the stream before each launch (the GEMMs of a rank run on one
// stream, so launches never overlap on it).
static int g_gemmp_dynamic = -1;
void set_gemmp_dynamic(bool on) {
  const char* e = std::getenv("DPA_GEMMP_DYNAMIC");
  g_gemmp_dynamic = e ? (e[0] == '1' ? 1 : 0) : (on ? 1 : 0);
}
static int* gemmp_queue(hipStream_t s) {
  if (g_gemmp_dynamic < 0) set_gemmp_dynamic(false);
  if (!g_gemmp_dynamic) return nullptr;
  // one counter buffer per (device, stream): GEMMs on one stream never overlap, but the
  // overlapped micro-batch schedule runs GEMMs on two streams at once
  // A ring of NSLOT counter sets per (device, stream), zeroed once when created: every launch
  // leaves its counters zeroed (the kernel's last workgroup per queue resets them), so no
  // memset runs per launch (the reference schedule issues ~3000 GEMMs per step) and a captured
  // HIP graph replays with valid counters.
  constexpr int NSLOT = 256, SLOT_INTS = 8 * 16;
  struct Q { int dev; hipStream_t s; int* buf; int cursor; };
  static Q qs[64];
  static int nq = 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  Q* q = nullptr;
  for (int i = 0; i < nq; ++i)
    if (qs[i].dev == dev && qs[i].s == s) q = &qs[i];
  if (!q) {
    // a stream first seen while it is being captured (the graph's capture stream) keeps the
    // static schedule: no allocation inside a capture
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    int* buf = nullptr;
    if (nq >= 64 || hipMalloc(&buf, (size_t)NSLOT * SLOT_INTS * sizeof(int)) != hipSuccess) return nullptr;
    if (hipMemsetAsync(buf, 0, (size_t)NSLOT * SLOT_INTS * sizeof(int), s) != hipSuccess) return nullptr;
    qs[nq] = Q{dev, s, buf, 0};
    q = &qs[nq++];
  }
  int* slot = q->buf + (size_t)q->cursor * SLOT_INTS;
  q->cursor = (q->cursor + 1) % NSLOT;
  return slot;
}

template <bool B_TR, int EPI, int ACT, int POL = 0, int GM = 1, bool HMT = false>
static void gemmp_launch(const uint16_t* a, int64_t lda, const uint16_t* b, int64_t ldb, int M, int N, int K,
                         uint16_t* c, const uint16_t* bias, uint16_t* z, int ncu, hipStream_t s,
                         float* colpart, int hm, const g256::EpiArgs& ea) {
  const int tiles = (M / (HMT ? 128 : 256)) * (N / 256);
  const int grid = persistent_grid(tiles, ncu);
  int* q = (tiles > grid && grid >= 8) ? gemmp_queue(s) : nullptr;
  hipLaunchKernelGGL((g256::gemmp_kernel<B_TR, EPI, ACT, POL, GM, 0, 0, HMT>), dim3(grid), dim3(512), 0, s,
                     (const bf16_t*)a, lda, (const bf16_t*)b, ldb, M, N, K / 64, (bf16_t*)c, (int64_t)N,
                     (const bf16_t*)bias, (bf16_t*)z, colpart, q, hm, ea);
}

// The two GELU-side GEMMs (EPI 6: y and act' stored; EPI 4: times act' plus column sums) of
// wide layers (>= 8 column tiles) walk tiles in groups of 8 tile rows with non-temporal
// epilogue stores: 2.1% / 2.6% faster on the 3072-wide MLP GEMMs at T = 262144 (gemm_lab
// "policy" study, profiles/gemm_lab_r3_policy.txt); neither helps the narrow GEMMs.
// 128 x 256 tiles when the launch finishes sooner with them: R rounds of 256-row tiles over the
// grid against ceil(2 tiles / grid) rounds of half tiles, each costing ~HALF_COST of a full one
// (tools/probes/small_gemm.py).  At 8192 tokens every BERT-base GEMM gains (768 wide: 96 tiles
// for 256 CUs -> 192; 2304 / 3072 wide: 2 rounds -> 3 half rounds); at 262144 tokens none does.
// DPA_GEMMP_HALF: 0 off, 1 (default) by that rule, 2 wherever allowed (M % 256 == 0).
static int g_gemmp_half = -1;
void set_gemmp_half(int mode) { g_gemmp_half = mode < 0 ? -1 : mode; }  // -1: DPA_GEMMP_HALF / auto
static bool use_half_tiles(int M, int N, int ncu) {
  if (g_gemmp_half < 0) {
    const char* e = std::getenv("DPA_GEMMP_HALF");
    g_gemmp_half = e ? std::atoi(e) : 1;
  }
  const int mode = g_gemmp_half;
  constexpr double HALF_COST = 0.66;
  if (mode == 0 || M % 256) return false;
  if (mode >= 2) return true;
  const int g = persistent_grid(1 << 30, ncu);
  const int t = (M / 256) * (N / 256);
  const int rf = (t + g - 1) / g, rh = (2 * t + g - 1) / g;
  return rh * HALF_COST < rf * 0.97;
}

template <bool B_TR, int EPI, int ACT>
static void gemmp_go(const uint16_t* a, int64_t lda, const uint16_t* b, int64_t ldb, int M, int N, int K,
                     uint16_t* c, const uint16_t* bias, uint16_t* z, int ncu, hipStream_t s,
                     float* colpart = nullptr, int hm = 0, const g256::EpiArgs& ea = g256::EpiArgs{}) {
  if constexpr (EPI != 4) {
    if (use_half_tiles(M, N, ncu)) {
      gemmp_launch<B_TR, EPI, ACT, 0, 1, true>(a, lda, b, ldb, M, N, K, c, bias, z, ncu, s, colpart, hm, ea);
      return;
    }
  }
  if constexpr (EPI == 4 || EPI == 6 || EPI == 8) {
    if ((M / 256) % 8 == 0 && N / 256 >= 8) {
      gemmp_launch<B_TR, EPI, ACT, 1, 8>(a, lda, b, ldb, M, N, K, c, bias, z, ncu, s, colpart, hm, ea);
      return;
    }
  }
  gemmp_launch<B_TR, EPI, ACT>(a, lda, b, ldb, M, N, K, c, bias, z, ncu, s, colpart, hm, ea);
}

// y[T][N] = act(x[T][K] . W[N][K]^T + bias); z (nullable, act != 0) = the pre-activation,
// or act'(pre-activation) when zderiv (the backward then multiplies: act code 4).
bool launch_gemmp_nt(const uint16_t* x, const uint16_t* W, const uint16_t* bias, uint16_t* y,
                     uint16_t* z, int T, int N, int K, int act, int ncu, hipStream_t s, bool zderiv, int hm,
                     bool z8) {
  if (!g256_enabled() || T % 256 || N % 256 || K % 128 || K < 128 || act < 0 || act > 3 || N >= (1 << 24))
    return false;  // (output width < 2^24: the epilogue's 24-bit row multiply)
  if (hm && (act != 0 || hm < 7 || hm > 30 || (T & ((1 << hm) - 1)) || N % 64)) return false;
  if (z8 && (act == 0 || z == nullptr || !zderiv)) return false;
  if (act == 0) gemmp_go<false, 0, 0>(x, K, W, K, T, N, K, y, bias, nullptr, ncu, s, nullptr, hm);
  else if (z8) {
    if (act == 1) gemmp_go<false, 8, 1>(x, K, W, K, T, N, K, y, bias, z, ncu, s);
    else if (act == 2) gemmp_go<false, 8, 2>(x, K, W, K, T, N, K, y, bias, z, ncu, s);
    else gemmp_go<false, 8, 3>(x, K, W, K, T, N, K, y, bias, z, ncu, s);
  } else if (z != nullptr && zderiv) {
    if (act == 1) gemmp_go<false, 6, 1>(x, K, W, K, T, N, K, y, bias, z, ncu, s);
    else if (act == 2) gemmp_go<false, 6, 2>(x, K, W, K, T, N, K, y, bias, z, ncu, s);
    else gemmp_go<false, 6, 3>(x, K, W, K, T, N, K, y, bias, z, ncu, s);
  } else if (z == nullptr) {
    if (act == 1) gemmp_go<false, 1, 1>(x, K, W, K, T, N, K, y, bias, nullptr, ncu, s);
    else if (act == 2) gemmp_go<false, 1, 2>(x, K, W, K, T, N, K, y, bias, nullptr, ncu, s);
    else gemmp_go<false, 1, 3>(x, K, W, K, T, N, K, y, bias, nullptr, ncu, s);
  } else {
    if (act == 1) gemmp_go<false, 2, 1>(x, K, W, K, T, N, K, y, bias, z, ncu, s);
    else if (act == 2) gemmp_go<false, 2, 2>(x, K, W, K, T, N, K, y, bias, z, ncu, s);
    else gemmp_go<false, 2, 3>(x, K, W, K, T, N, K, y, bias, z, ncu, s);
  }
  return true;
}

// dx[T][K] = dy[T][N] . W[N][K]  (act != 0: times act'(aux[T][K]); colpart != nullptr:
// also the per-tile column-sum partials [(T/256)*2][K] of the result)
// dx[T][K] = dy[T][N] . W[N][K] + dx[T][K]  (in place, bf16)
// h[T][N] = res[T][N] + dropout_p(x[T][K] . W[N][K]^T + bias): the post-LN sublayer's residual
// branch folded into the GEMM epilogue (the LayerNorm then reads h alone and writes no h copy);
// the dropout bits are pair_hash(seed, offset) ones, regenerated by add_ln_bwd's pair-hash mode
bool launch_gemmp_nt_res(const uint16_t* x, const uint16_t* W, const uint16_t* bias, const uint16_t* res,
                         uint16_t* h, int T, int N, int K, int ncu, hipStream_t s, float p, uint32_t seed,
                         uint32_t offset) {
  if (!g256_enabled() || T % 256 || N % 256 || K % 128 || K < 128 || !(p >= 0.f && p < 1.f) || N >= (1 << 24))
    return false;
  g256::EpiArgs ea;
  ea.seed = seed;
  ea.offset = offset;
  ea.thr16 = pair_thr16(p);
  ea.scale = 1.f / (1.f - p);
  gemmp_go<false, 7, 0>(x, K, W, K, T, N, K, h, bias, const_cast<uint16_t*>(res), ncu, s, nullptr, 0, ea);
  return true;
}

// Data-gradient GEMMs dx[T][K] = dy[T][N] . W[N][K]: with WT (= W^T [K][N], the transposed bf16
// shadow) through the row-form kernel - the forward's operand path, no transposed LDS reads, 3-5%
// faster per call (tools/probes/dgrad_layout.py) - else reading W itself transposed.
template <int EPI, int ACT>
static void gemmp_dgrad(const uint16_t* dy, const uint16_t* W, const uint16_t* WT, int T, int N, int K,
                        uint16_t* dx, uint16_t* z, int ncu, hipStream_t s, float* colpart = nullptr) {
  if (WT != nullptr)
    gemmp_go<false, EPI, ACT>(dy, N, WT, N, T, K, N, dx, nullptr, z, ncu, s, colpart);
  else
    gemmp_go<true, EPI, ACT>(dy, N, W, K, T, K, N, dx, nullptr, z, ncu, s, colpart);
}

bool launch_gemmp_nn_acc(const uint16_t* dy, const uint16_t* W, uint16_t* dx, int T, int N, int K, int ncu,
                         hipStream_t s, const uint16_t* WT) {
  if (!g256_enabled() || T % 256 || K % 256 || N % 128 || N < 128 || K >= (1 << 24)) return false;
  gemmp_dgrad<5, 0>(dy, W, WT, T, N, K, dx, dx, ncu, s);
  return true;
}

bool launch_gemmp_nn(const uint16_t* dy, const uint16_t* W, uint16_t* dx, const uint16_t* aux, int act,
                     int T, int N, int K, int ncu, hipStream_t s, float* colpart, const uint16_t* WT) {
  if (!g256_enabled() || T % 256 || K % 256 || N % 128 || N < 128 || act < 0 || act > 5 || K >= (1 << 24))
    return false;
  uint16_t* ax = const_cast<uint16_t*>(aux);
  if (act == 0 || aux == nullptr) {
    if (colpart) return false;
    gemmp_dgrad<0, 0>(dy, W, WT, T, N, K, dx, nullptr, ncu, s);
  } else if (act == 5) {  // aux: u8 act' codes in the tile-native layout of an EPI 8 forward
    if (colpart) gemmp_dgrad<4, 5>(dy, W, WT, T, N, K, dx, ax, ncu, s, colpart);
    else gemmp_dgrad<3, 5>(dy, W, WT, T, N, K, dx, ax, ncu, s);
  } else if (act == 4 && WT != nullptr) {  // aux: bf16 act' (EPI 6 forward)
    if (colpart) gemmp_dgrad<4, 4>(dy, W, WT, T, N, K, dx, ax, ncu, s, colpart);
    else gemmp_dgrad<3, 4>(dy, W, WT, T, N, K, dx, ax, ncu, s);
  } else if (colpart) {
    if (act == 1) gemmp_go<true, 4, 1>(dy, N, W, K, T, K, N, dx, nullptr, ax, ncu, s, colpart);
    else if (act == 2) gemmp_go<true, 4, 2>(dy, N, W, K, T, K, N, dx, nullptr, ax, ncu, s, colpart);
    else if (act == 3) gemmp_go<true, 4, 3>(dy, N, W, K, T, K, N, dx, nullptr, ax, ncu, s, colpart);
    else gemmp_go<true, 4, 4>(dy, N, W, K, T, K, N, dx, nullptr, ax, ncu, s, colpart);
  } else {
    if (act == 1) gemmp_go<true, 3, 1>(dy, N, W, K, T, K, N, dx, nullptr, ax, ncu, s);
    else if (act == 2) gemmp_go<true, 3, 2>(dy, N, W, K, T, K, N, dx, nullptr, ax, ncu, s);
    else if (act == 3) gemmp_go<true, 3, 3>(dy, N, W, K, T, K, N, dx, nullptr, ax, ncu, s);
    else gemmp_go<true, 3, 4>(dy, N, W, K, T, K, N, dx, nullptr, ax, ncu, s);
  }
  return true;
}

// Split-K plan of the weight gradient (one 128 KiB workgroup per CU): rounds of
// workgroups x (K-tiles per split x ~1.5 us + ~4 us fixed) plus the cost of merging the
// splits.  Two merges: fp32 atomics straight into the gradient (~1.2 TB/s chip-wide: the
// L2 does one 4-byte RMW per atomic) or plain 16-B stores of each split's partial into a
// workspace plus one reduce pass over it ((2 s + 2) x the gradient bytes at HBM rate).
// The old rule (fill two rounds regardless of T) split an 8192-token micro-batch 32
// ways: 54x atomic amplification, 107 us per call.
// nseg > 1: that many equal token segments (multi-segment launch, one slab per (segment, split)).
struct WgradPlan { int splits, kps; bool ws; };
static WgradPlan wgrad_plan(int T, int N, int K, int nseg = 1) {
  const int tiles = (N / 256) * (K / 256) * nseg;
  const int ktot = T / 64;
  const int ncu = device_cu_count();
  const double mb = (double)N * K * 4.0 / 1e6;  // gradient bytes, MB
  // merge through the workspace whenever K is split (measured faster at every encoder shape:
  // 8192 tokens -17%, 262144 tokens -2..5%, tools/wgrad_bench.py)
  constexpr int force_ws = 1, force_s = -1;
  constexpr double merge_cost = 1.0;
  WgradPlan best_p{1, ktot + (ktot & 1), false};
  double best = 1e30;
  const int smax = ktot / 2 < 1 ? 1 : ktot / 2;
  for (int sp = 1; sp <= smax; ++sp) {
    if (force_s > 0 && sp != force_s) continue;
    int kps = (ktot + sp - 1) / sp;
    kps += kps & 1;
    const int s_eff = (ktot + kps - 1) / kps;
    const int wgs = tiles * s_eff;
    const int rounds = (wgs + ncu - 1) / ncu;
    const double main = rounds * (kps * 1.5 + 4.0);
    const int slabs = s_eff * nseg;  // partials merged per gradient element
    for (int w = 0; w < 2; ++w) {
      if (w == 1 && slabs < 2) continue;
      if (force_ws >= 0 && w != force_ws && !(w == 0 && slabs < 2)) continue;
      const double t = w ? main + merge_cost * (2.0 * slabs + 2.0) * mb / 4.0 : fmax(main, wgs * 0.35);
      if (t < best * 0.98) {
        best = t;
        best_p = WgradPlan{s_eff, kps, w == 1};
      }
    }
    // search up to 8 rounds of workgroups: a large tile count (GPT-2's 591-tile LM-head
    // weight gradient) needs 3 splits (1773 workgroups: 6.9 rounds) to avoid a 60%-empty last
    // round, past the 4-round cap this search used to stop at
    if (wgs > 8 * ncu) break;
  }
  return best_p;
}

int64_t gemm256_wgrad_workspace_floats(int T, int N, int K, int nseg) {
  if (!g256_enabled() || N % 256 || K % 256 || T % 128 || T < 128 || nseg < 1 || nseg > g256::WG_MAXSEG)
    return 0;
  const WgradPlan p = wgrad_plan(T, N, K, nseg);
  return p.ws ? (int64_t)p.splits * nseg * ((int64_t)N * K + N) : 0;  // [slabs][N][K] + bias partials [slabs][N]
}

__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ ws, float* __restrict__ dW,
                                                           int64_t n4, int splits) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  f32x4 acc = reinterpret_cast<const f32x4*>(dW)[i];
  for (int s = 0; s < splits; ++s) acc += reinterpret_cast<const f32x4*>(ws)[s * n4 + i];
  reinterpret_cast<f32x4*>(dW)[i] = acc;
}

// db[m] += sum over slabs (in order) of the split-K bias partials [slabs][N]
__global__ void __launch_bounds__(256) wgrad_colsum_reduce_kernel(const float* __restrict__ part, float* __restrict__ db,
                                                                  int n, int slabs) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float a = db[i];
  for (int s = 0; s < slabs; ++s) a += part[(int64_t)s * n + i];
  db[i] = a;
}

// The one-wave-per-SIMD TR x TR kernel (csrc/wgrad4w.hip) takes every weight gradient whose bias
// gradient comes from elsewhere (db == nullptr: the encoder's biases are reduced by the LayerNorm,
// dact-GEMM and attention backwards) with the same split plan; the 8-phase kernel keeps the
// in-kernel bias column sums.  set_wgrad4w(false): the 8-phase kernel everywhere (A/B, tests).
static bool g_wgrad4w = false;  // on once measured (see the header comment of wgrad4w.hip)
void set_wgrad4w(bool on) { g_wgrad4w = on; }

static bool wgrad4w_go(const uint16_t* const* dys, const uint16_t* const* xs, int nseg, float* dW, int T, int N,
                       int K, const WgradPlan& p, float* wsp, hipStream_t s) {
  if (!g_wgrad4w || (wsp == nullptr && p.splits * nseg != 1)) return false;
  if (!launch_wgrad4w(dys, xs, nseg, T, N, K, p.splits, p.kps, dW, wsp, s)) return false;
  if (wsp) {
    const int64_t n4 = (int64_t)N * K / 4;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, wsp, dW, n4,
                       p.splits * nseg);
  }
  return true;
}

bool launch_gemm256_wgrad(const uint16_t* dy, const uint16_t* x, float* dW, float* db, int T,
                          int N, int K, hipStream_t s, float* ws) {
  // dW[N][K] += dy[T][N]^T . x[T][K]: M = N, N' = K, reduction = T split over workgroups
  if (!g256_enabled() || N % 256 || K % 256 || T % 128 || T < 128) return false;
  const int tiles = (N / 256) * (K / 256);
  const int ktot = T / 64;
  const WgradPlan p = wgrad_plan(T, N, K);
  float* wsp = (p.ws && ws != nullptr) ? ws : nullptr;
  if (db == nullptr && wgrad4w_go(&dy, &x, 1, dW, T, N, K, p, wsp, s)) return true;
  hipLaunchKernelGGL((g256::gemm256_kernel<true, true, g256::EPI_ATOMIC_F32>),
                     dim3(tiles * p.splits), dim3(512), 0, s, (const bf16_t*)dy, (int64_t)N,
                     (const bf16_t*)x, (int64_t)K, N, K, ktot, p.kps, p.splits, nullptr, (int64_t)K, dW,
                     nullptr, 0, nullptr, db, wsp);
  if (wsp) {
    const int64_t n4 = (int64_t)N * K / 4;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, wsp, dW, n4,
                       p.splits);
    if (db)
      hipLaunchKernelGGL(wgrad_colsum_reduce_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s,
                         wsp + (int64_t)p.splits * N * K, db, N, p.splits);
  }
  return true;
}

// dW[N][K] += sum_s dy_s[T][N]^T . x_s[T][K] over nseg equal token segments in ONE launch: the
// split-K plan sees nseg x the tiles, so each segment is split fewer ways (fewer fp32 partial
// slabs per token than nseg separate launches) and one reduce pass merges everything.
bool launch_gemm256_wgrad_multi(const uint16_t* const* dys, const uint16_t* const* xs, int nseg, float* dW,
                                float* db, int T, int N, int K, hipStream_t s, float* ws) {
  if (!g256_enabled() || N % 256 || K % 256 || T % 128 || T < 128 || nseg < 1 || nseg > g256::WG_MAXSEG)
    return false;
  if (nseg == 1) return launch_gemm256_wgrad(dys[0], xs[0], dW, db, T, N, K, s, ws);
  g256::WgSegs sg{};
  for (int i = 0; i < nseg; ++i) {
    sg.a[i] = (const bf16_t*)dys[i];
    sg.b[i] = (const bf16_t*)xs[i];
  }
  sg.n = nseg;
  const int tiles = (N / 256) * (K / 256);
  const int ktot = T / 64;
  const WgradPlan p = wgrad_plan(T, N, K, nseg);
  float* wsp = (p.ws && ws != nullptr) ? ws : nullptr;
  if (db == nullptr && wgrad4w_go(dys, xs, nseg, dW, T, N, K, p, wsp, s)) return true;
  hipLaunchKernelGGL((g256::gemm256_kernel<true, true, g256::EPI_ATOMIC_F32>),
                     dim3(tiles * p.splits * nseg), dim3(512), 0, s, sg.a[0], (int64_t)N, sg.b[0], (int64_t)K,
                     N, K, ktot, p.kps, p.splits, nullptr, (int64_t)K, dW, nullptr, 0, nullptr, db, wsp, sg);
  if (wsp) {
    const int64_t n4 = (int64_t)N * K / 4;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, wsp, dW, n4,
                       p.splits * nseg);
    if (db)
      hipLaunchKernelGGL(wgrad_colsum_reduce_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s,
                         wsp + (int64_t)p.splits * nseg * N * K, db, N, p.splits * nseg);
  }
  return true;
}

// Tile offsets of a grouped weight-gradient launch; -1 when a site does not tile (256-multiple
// sides, an even number of 64-token K-tiles per segment, 1..8 segments).
int wgrad_group_prepare(WgGroupSite* sites, int nsites) {
  if (!g256_enabled() || nsites < 1) return -1;
  int total = 0;
  for (int i = 0; i < nsites; ++i) {
    WgGroupSite& s = sites[i];
    if (s.M % 256 || s.N % 256 || s.M <= 0 || s.N <= 0 || s.nseg < 1 || s.nseg > g256::WG_MAXSEG ||
        s.ktiles < 2 || (s.ktiles & 1) || s.dW == nullptr)
      return -1;
    s.tile0 = total;
    total += (s.M / 256) * (s.N / 256);
  }
  return total;
}

bool launch_wgrad_group(const WgGroupSite* d_sites, int nsites, int ntiles, hipStream_t s) {
  if (ntiles <= 0 || nsites < 1) return false;
  hipLaunchKernelGGL(g256::wgrad_group_kernel, dim3((unsigned)ntiles), dim3(512), 0, s, d_sites, nsites, ntiles);
  return true;
}

DPA_RNG_BASE_EXPORT(gemm256)

}  // namespace dpa
