// Lab: 256 x 256 bf16 GEMM with ONE wave per SIMD (4 waves, 256 threads, 512 registers per
// wave: the 8 x 8 grid of 16x16 fp32 accumulators of a 128 x 128 wave tile = 256 AGPRs).
//
// Question (VERDICT r3 "Next" #1): can a single wave per SIMD keep the matrix pipe as busy as
// the two-wave 8-phase template (gemm256.hip) while issuing its own LDS-DMA pieces and
// fragment reads?  If so, the freed half of the register file can hold the previous tile's
// epilogue state and the epilogue can be spread through the next tile's main loop.
//
// Main loop (one K-tile = 64 deep = two k32 steps of 64 MFMAs each, 128 "slots"):
//  * LDS: 2 K-tile buffers x {A rows 0-127, A rows 128-255, B rows 0-127, B rows 128-255}
//    half images of 16 KiB (128 KiB), filled by buffer_load ... lds (4 pieces of 1 KiB per
//    wave per half image), XOR swizzle on the source address, undone on the read.
//  * wave w computes rows 128 (w >> 1) .. +127 and columns 128 (w & 1) .. +127: it reads ONE
//    A half image and ONE B half image (16 ds_read_b128 per k32 step).
//  * slot s of K-tile t: MFMA (i, j) = (s >> 3 & 7, s & 7) of step s >> 6, interleaved with
//      - step-1 fragment reads of K-tile t during step 0 (one per 4 slots),
//      - step-0 fragment reads of K-tile t + 1 during slots 80-127 (one per 3 slots),
//      - DMA pieces: K-tile t + 1's pieces 8-15 in slots 0-47, K-tile t + 2's pieces 0-7 in
//        slots 80-127 (one per 6 slots),
//    a `s_waitcnt vmcnt(0)` + barrier at slot 80 (K-tile t + 1 landed, and every wave is past
//    its step-0 reads of buffer t & 1, so K-tile t + 2 may overwrite it).
#include <hip/hip_runtime.h>

#include <utility>

#include "common.h"
#include "mfma.h"

namespace dpa {
namespace g4w {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_v;

constexpr int HALF = 16384;
constexpr int B_REGION = 65536;
__host__ __device__ constexpr int img_off(int buf, int h) { return buf * 2 * HALF + h * HALF; }

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_v, a),
                                                 __builtin_bit_cast(bf16x8_v, b), c, 0, 0, 0);
}
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) char*)p);
}
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }

// Row-form operand ([rows][k], k contiguous): a 256-row tile = two 128-row half images.
struct Op {
  const bf16_t* base;
  int64_t ld;
  uint32_t off[4];  // DMA byte offsets of this wave's 4 pieces of a half image
  uint32_t rd[2];   // fragment read bases (k32 step 0 / 1) in this wave's half image
  int wv;

  __device__ __forceinline__ void init(const bf16_t* p, int64_t ld_, int row0, int w, int lane,
                                       uint32_t img_base) {
    ld = ld_;
    wv = w;
    base = p + (int64_t)row0 * ld_;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = (w * 4 + j) * 8 + (lane >> 3), phys = lane & 7;
      off[j] = (uint32_t)(r * (int)ld_ + ((phys ^ ((r >> 1) & 7)) << 3)) * 2u;
    }
    const int g = lane >> 4, li = lane & 15, s = (li >> 1) & 7;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) rd[kk] = img_base + (uint32_t)(li * 128 + (((kk * 4 + g) ^ s) << 4));
  }
  // piece j of half image h of K-tile t into LDS at `img` (the half image's byte address):
  // one descriptor per half image, the K-tile as the scalar offset (t * 128 bytes)
  __device__ __forceinline__ void piece(char* img, int h, int t, int j) const {
    const bf16_t* src = base + (int64_t)h * 128 * ld;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(src), (short)0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(img + (wv * 4 + j) * 1024), 16, off[j], t * 128, 0, 0);
  }
  // 16-row block I of k32 step KK of the image at byte offset `img` (relative to rd's base)
  template <int I, int KK>
  __device__ __forceinline__ void frag(bf16x8& f, int img) const {
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f) : "v"(rd[KK] + (uint32_t)img), "i"(I * 2048));
  }
};

// DMA piece q (0..15) of K-tile t into buffer buf: half images {A0, A1, B0, B1} x 4 pieces
__device__ __forceinline__ void dma_piece(const Op& opA, const Op& opB, char* smem, int buf, int t, int q) {
  const int h = (q >> 2) & 1, j = q & 3;
  if (q < 8) opA.piece(smem + img_off(buf, h), h, t, j);
  else opB.piece(smem + B_REGION + img_off(buf, h), h, t, j);
}

// Per-slot work of the main loop, all indices compile-time (template slot S).
struct MainState {
  f32x4 (&acc)[8][8];
  bf16x8 (&fa0)[8];
  bf16x8 (&fb0)[8];
  bf16x8 (&fa1)[8];
  bf16x8 (&fb1)[8];
  const Op& opA;
  const Op& opB;
  char* smem;
  int t, cur, nxt;
};

template <int S, bool H1, bool H2>
__device__ __forceinline__ void slot(MainState& m) {
  constexpr int i = (S >> 3) & 7, j = S & 7;
  if constexpr (S < 64) m.acc[i][j] = mfma16(m.fa0[i], m.fb0[j], m.acc[i][j]);
  else m.acc[i][j] = mfma16(m.fa1[i], m.fb1[j], m.acc[i][j]);
  // step-1 fragments of this K-tile during step 0: slot 8r = A block r, slot 8r + 4 = B block r
  if constexpr (S < 64 && (S & 7) == 0) m.opA.template frag<(S >> 3), 1>(m.fa1[S >> 3], m.cur);
  if constexpr (S < 64 && (S & 7) == 4) m.opB.template frag<(S >> 3), 1>(m.fb1[S >> 3], m.cur);
  if constexpr (S == 63) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  // DMA: K-tile t + 1 pieces 8..15 in slots 0, 6, .., 42; K-tile t + 2 pieces 0..7 in 80, 86, .., 122
  if constexpr (S < 48 && S % 6 == 0) {
    if constexpr (H1) dma_piece(m.opA, m.opB, m.smem, (m.t + 1) & 1, m.t + 1, 8 + S / 6);
  }
  if constexpr (S >= 80 && (S - 80) % 6 == 0) {
    if constexpr (H2) dma_piece(m.opA, m.opB, m.smem, m.t & 1, m.t + 2, (S - 80) / 6);
  }
  if constexpr (S == 79) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();
  }
  // step-0 fragments of K-tile t + 1 during slots 80..127 (one per 3 slots, A and B alternating)
  if constexpr (S >= 80 && (S - 80) % 3 == 0) {
    constexpr int r = (S - 80) / 3;
    if constexpr (H1) {
      if constexpr ((r & 1) == 0) m.opA.template frag<(r >> 1), 0>(m.fa0[r >> 1], m.nxt);
      else m.opB.template frag<(r >> 1), 0>(m.fb0[r >> 1], m.nxt);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
}

template <bool H1, bool H2, int... S>
__device__ __forceinline__ void all_slots(MainState& m, std::integer_sequence<int, S...>) {
  (slot<S, H1, H2>(m), ...);
}

template <bool H1, bool H2>
__device__ __forceinline__ void ktile(MainState& m) {
  __builtin_amdgcn_s_setprio(1);
  all_slots<H1, H2>(m, std::make_integer_sequence<int, 128>{});
  __builtin_amdgcn_s_setprio(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int EPI>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
gemm4w_kernel(const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ B, int64_t ldb, int M,
              int N, int nk, bf16_t* __restrict__ C, int64_t ldc) {
  __shared__ __attribute__((aligned(1024))) char smem[131072];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int wm = w >> 1, wn = w & 1;
  const int NT = N / 256;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = tile / NT, nt = tile - (tile / NT) * NT;
  const uint32_t sbase = lds_u32(smem);

  Op opA, opB;
  opA.init(A, lda, mt * 256, w, lane, sbase + img_off(0, wm));
  opB.init(B, ldb, nt * 256, w, lane, sbase + B_REGION + img_off(0, wn));

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];

  // prologue: K-tile 0 -> buffer 0 (all pieces), wait, step-0 fragments; K-tile 1 -> buffer 1
  // pieces 0..7 (pieces 8..15 go out in K-tile 0's slots 0-47 like every later K-tile's)
#pragma unroll
  for (int q = 0; q < 16; ++q) dma_piece(opA, opB, smem, 0, 0, q);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  barrier();
  opA.frag<0, 0>(fa0[0], 0); opA.frag<1, 0>(fa0[1], 0); opA.frag<2, 0>(fa0[2], 0); opA.frag<3, 0>(fa0[3], 0);
  opA.frag<4, 0>(fa0[4], 0); opA.frag<5, 0>(fa0[5], 0); opA.frag<6, 0>(fa0[6], 0); opA.frag<7, 0>(fa0[7], 0);
  opB.frag<0, 0>(fb0[0], 0); opB.frag<1, 0>(fb0[1], 0); opB.frag<2, 0>(fb0[2], 0); opB.frag<3, 0>(fb0[3], 0);
  opB.frag<4, 0>(fb0[4], 0); opB.frag<5, 0>(fb0[5], 0); opB.frag<6, 0>(fb0[6], 0); opB.frag<7, 0>(fb0[7], 0);
#pragma unroll
  for (int q = 0; q < 8; ++q) dma_piece(opA, opB, smem, 1, 1, q);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  // nk >= 2 (host-checked): K-tiles 0 .. nk-3 with both prefetches, then the two tail K-tiles
  for (int t = 0; t < nk - 2; ++t) {
    MainState m{acc, fa0, fb0, fa1, fb1, opA, opB, smem, t, (t & 1) * 2 * HALF, ((t + 1) & 1) * 2 * HALF};
    ktile<true, true>(m);
  }
  {
    const int t = nk - 2;
    MainState m{acc, fa0, fb0, fa1, fb1, opA, opB, smem, t, (t & 1) * 2 * HALF, ((t + 1) & 1) * 2 * HALF};
    ktile<true, false>(m);
  }
  {
    const int t = nk - 1;
    MainState m{acc, fa0, fb0, fa1, fb1, opA, opB, smem, t, (t & 1) * 2 * HALF, ((t + 1) & 1) * 2 * HALF};
    ktile<false, false>(m);
  }

  if constexpr (EPI == 0) {
    // timing probe: keep the accumulators live (one store per lane of a checksum)
    float x = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) x += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (x == 1.2345f) C[threadIdx.x] = (bf16_t)1;
  } else {
    // plain per-element bf16 stores (correctness check): lane holds C[4 (lane >> 4) + r][lane & 15]
    const int64_t row0 = (int64_t)mt * 256 + wm * 128 + 4 * (lane >> 4);
    const int col0 = nt * 256 + wn * 128 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) C[(row0 + 16 * i + r) * ldc + col0 + 16 * j] = f2bf(acc[i][j][r]);
  }
}

}  // namespace g4w

// y[M][N] = A[M][K] . B[N][K]^T (both row form); M, N % 256, K % 64
inline void launch_gemm4w(const uint16_t* A, const uint16_t* B, uint16_t* C, int M, int N, int K, bool store,
                          hipStream_t s) {
  const int tiles = (M / 256) * (N / 256);
  if (store)
    hipLaunchKernelGGL(g4w::gemm4w_kernel<1>, dim3(tiles), dim3(256), 0, s, (const bf16_t*)A, (int64_t)K,
                       (const bf16_t*)B, (int64_t)K, M, N, K / 64, (bf16_t*)C, (int64_t)N);
  else
    hipLaunchKernelGGL(g4w::gemm4w_kernel<0>, dim3(tiles), dim3(256), 0, s, (const bf16_t*)A, (int64_t)K,
                       (const bf16_t*)B, (int64_t)K, M, N, K / 64, (bf16_t*)C, (int64_t)N);
}

}  // namespace dpa
