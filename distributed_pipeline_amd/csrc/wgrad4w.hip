// Weight gradient dW[M][N] += sum_t dy[t][m] x[t][n] with ONE wave per SIMD (gfx950).
//
// The Linear weight gradient reads both operands with the reduction dimension (tokens)
// outermost in memory, so both LDS images are transposed ([64 k][128 cols]) and every MFMA
// operand fragment is two ds_read_b64_tr_b16 instead of one ds_read_b128: twice the LDS
// read instructions of the forward / data-gradient GEMMs.  In the two-waves-per-SIMD 8-phase
// template (gemm256_kernel<true, true, 2>) those reads are issued in bursts at the start of a
// phase and rely on the partner wave's MFMAs to hide them; the burst of a TR x TR phase (24
// reads) outlasts the partner's 16 MFMAs, and the weight gradient ran at 1.19 PFLOP/s against
// 1.34-1.46 for the other products.
//
// Here (the structure of tools/gemm_lab/gemm4w.hip, measured within 1-5% of the 8-phase
// template on row-form operands) each wave owns a 128 x 128 quadrant of the 256 x 256 tile
// (64 accumulators of 16 x 16, 256 registers) and interleaves its own fragment reads and
// LDS-DMA pieces with its MFMAs slot by slot, so the transposed reads ride in the MFMA gaps
// (at most 2 ds_read_b64_tr_b16 per 16-cycle v_mfma_f32_16x16x32_bf16):
//  * LDS: 2 K-tile buffers x {A cols 0-127, A cols 128-255, B cols 0-127, B cols 128-255}
//    transposed half images of 16 KiB, filled by buffer_load ... lds (4 pieces of 1 KiB per
//    wave per half image: 4 k-rows of 256 B each), 16-B chunks XOR-swizzled by the k-row so
//    the transposed reads are conflict-free (the layout of gemm256.hip Operand<true>);
//  * K-tile t, slot s of 128: MFMA (i, j) = (s >> 3 & 7, s & 7) of k32 step s >> 6; step-1
//    fragments of t read during step 0, step-0 fragments of t + 1 during slots 80-127, DMA
//    pieces of t + 1 (B) in slots 0-47 and of t + 2 (A) in slots 80-127, one vmcnt(0) +
//    barrier per K-tile at slot 80;
//  * the MFMAs run transposed (B.A^T), so a lane holds 4 consecutive columns of one row: the
//    split-K partial goes out as 16-B stores into the fp32 workspace slab of its split (merged
//    by wgrad_reduce_kernel, gemm256.hip) or, unsplit (one workgroup per output tile), as a
//    16-B read-modify-write of the gradient;
//  * K is split over workgroups exactly as gemm256's wgrad_plan decides (same launch shape).
#include <utility>

#include "common.h"
#include "launchers.h"
#include "mfma.h"

namespace dpa {
namespace w4t {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_v;

constexpr int HALF = 16384;
constexpr int B_REGION = 65536;
__host__ __device__ constexpr int img_off(int buf, int h) { return buf * 2 * HALF + h * HALF; }

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_v, a), __builtin_bit_cast(bf16x8_v, b),
                                                 c, 0, 0, 0);
}
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) char*)p);
}
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }
// chunk XOR of a transposed image row (as gemm256.hip tr_x)
__device__ __forceinline__ int tr_x(int row) { return ((row & 3) << 1) | (((row >> 3) & 1) << 3); }

// One transposed operand: [T][ld] in memory, a 256-column tile = two 128-column half images.
struct OpT {
  const bf16_t* base;  // element (k = 0, column 0 of the tile)
  int64_t ld;
  uint32_t off[4];     // byte offsets of this wave's 4 DMA pieces within a half image
  uint32_t rd;         // fragment read base of column block 0 in this wave's half image; block c
                       // is rd ^ (c << 5) (the swizzle's block bits are bits 5-7 of the address)
  int wv;

  __device__ __forceinline__ void init(const bf16_t* p, int64_t ld_, int col0, int w, int lane, uint32_t img) {
    ld = ld_;
    wv = w;
    base = p + col0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = (w * 4 + j) * 4 + (lane >> 4), phys = lane & 15;
      const int lc = phys ^ tr_x(k);
      off[j] = (uint32_t)(k * (int)ld_ + lc * 8) * 2u;
    }
    // chunk of column block c: (2 c + (pp >> 1)) ^ x = ((c ^ (x >> 1)) << 1) | (pp >> 1) (x has no
    // bit 0), so the byte address is rd ^ (c << 5) with img 16 KiB-aligned
    const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
    const int x = (q << 1) | ((g & 1) << 3);
    rd = img + (uint32_t)((8 * g + q) * 256 + (((x >> 1) << 1) | (pp >> 1)) * 16 + (pp & 1) * 8);
  }
  // piece j of half image h (columns 128 h ..) of K-tile t into LDS at `img` (the half image)
  __device__ __forceinline__ void piece(char* img, int h, int t, int j) const {
    const bf16_t* src = base + (int64_t)t * 64 * ld + h * 128;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(src), (short)0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(img + (wv * 4 + j) * 1024), 16, off[j], 0, 0, 0);
  }
  // 16-column block I, k32 step KK, of the buffer at byte offset `buf`.  Issued from asm: the
  // compiler does not see an LDS access, so it inserts no vmcnt drain against the in-flight
  // LDS-DMA (the builtin read got one before every read); the slot schedule retires the reads
  // with its own lgkmcnt waits before the fragments are used, and the two halves land directly
  // in the fragment's register quad (checked in the ISA: no copies in the main loop)
  template <int I, int KK>
  __device__ __forceinline__ void frag(bf16x8& f, uint32_t buf) const {
    bf16x4 a, b;
    const uint32_t addr = (rd ^ (uint32_t)(I << 5)) + buf;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(a) : "v"(addr), "i"(KK * 32 * 256));
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(b) : "v"(addr), "i"(KK * 32 * 256 + 1024));
    f = cat44(a, b);
  }
};

// DMA piece q (0..15) of K-tile t into buffer buf: half images {A0, A1, B0, B1} x 4 pieces
__device__ __forceinline__ void dma_piece(const OpT& opA, const OpT& opB, char* smem, int buf, int t, int q) {
  const int h = (q >> 2) & 1, j = q & 3;
  if (q < 8) opA.piece(smem + img_off(buf, h), h, t, j);
  else opB.piece(smem + B_REGION + img_off(buf, h), h, t, j);
}

struct MainState {
  f32x4 (&acc)[8][8];
  bf16x8 (&fa0)[8];
  bf16x8 (&fb0)[8];
  bf16x8 (&fa1)[8];
  bf16x8 (&fb1)[8];
  const OpT& opA;
  const OpT& opB;
  char* smem;
  int t;
  uint32_t cur, nxt;  // byte offsets of the buffers of K-tiles t and t + 1
};

// slot S of K-tile t (all indices compile-time); H1: K-tile t + 1 exists, H2: t + 2 exists
template <int S, bool H1, bool H2>
__device__ __forceinline__ void slot(MainState& m) {
  constexpr int i = (S >> 3) & 7, j = S & 7;
  // transposed product (B . A^T): lane = row of dW, registers = 4 consecutive columns
  if constexpr (S < 64) m.acc[i][j] = mfma16(m.fb0[j], m.fa0[i], m.acc[i][j]);
  else m.acc[i][j] = mfma16(m.fb1[j], m.fa1[i], m.acc[i][j]);
  // step-1 fragments of this K-tile during step 0: slot 8r = A block r, slot 8r + 4 = B block r
  if constexpr (S < 64 && (S & 7) == 0) m.opA.template frag<(S >> 3), 1>(m.fa1[S >> 3], m.cur);
  if constexpr (S < 64 && (S & 7) == 4) m.opB.template frag<(S >> 3), 1>(m.fb1[S >> 3], m.cur);
  if constexpr (S == 63) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  // DMA: K-tile t + 1 pieces 8..15 (B) in slots 0, 6, .., 42; K-tile t + 2 pieces 0..7 (A) in 80, .., 122
  if constexpr (S < 48 && S % 6 == 0) {
    if constexpr (H1) dma_piece(m.opA, m.opB, m.smem, (m.t + 1) & 1, m.t + 1, 8 + S / 6);
  }
  if constexpr (S >= 80 && (S - 80) % 6 == 0) {
    if constexpr (H2) dma_piece(m.opA, m.opB, m.smem, m.t & 1, m.t + 2, (S - 80) / 6);
  }
  if constexpr (S == 79) {
    // K-tile t + 1 has landed (this wave's pieces; the barrier: everyone's), and every wave is
    // past its reads of buffer t & 1, which K-tile t + 2's A pieces overwrite from slot 80
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

constexpr int MAXSEG = 8;
struct Segs {
  const bf16_t* a[MAXSEG];
  const bf16_t* b[MAXSEG];
  int n;  // 0: the kernel's A / B are the only segment
};

// grid = (M / 256) * (N / 256) * splits * max(1, segs.n); ktiles_per_split even, >= 2
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
wgrad4w_kernel(const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ B, int64_t ldb, int M, int N,
               int ktiles_total, int ktiles_per_split, int splits, float* __restrict__ Cf, int64_t ldc,
               float* __restrict__ wsp, Segs segs) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * B_REGION];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int wm = w >> 1, wn = w & 1;
  const int MT = M / 256, NT = N / 256;
  const int nseg = segs.n > 0 ? segs.n : 1;
  const int tile = xcd_remap(blockIdx.x, MT * NT * splits * nseg);
  const int nt = tile % NT, mt = (tile / NT) % MT, z = tile / (NT * MT);
  const int zs = z % splits;
  if (segs.n > 0) {
    const int sg = z / splits;
#pragma unroll
    for (int i = 0; i < MAXSEG; ++i)  // uniform selects: no dynamic index into the kernarg struct
      if (sg == i) {
        A = segs.a[i];
        B = segs.b[i];
      }
  }
  const int t0 = zs * ktiles_per_split;
  const int nk = min(ktiles_total - t0, ktiles_per_split);
  const uint32_t sbase = lds_u32(smem);

  OpT opA, opB;
  opA.init(A + (int64_t)t0 * 64 * lda, lda, mt * 256, w, lane, sbase + img_off(0, wm));
  opB.init(B + (int64_t)t0 * 64 * ldb, ldb, nt * 256, w, lane, sbase + B_REGION + img_off(0, wn));

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];

  // prologue: K-tile 0 -> buffer 0 (all pieces), wait, step-0 fragments; K-tile 1 -> buffer 1
  // A pieces (its B pieces go out in K-tile 0's slots 0-47 like every later K-tile's)
#pragma unroll
  for (int q = 0; q < 16; ++q) dma_piece(opA, opB, smem, 0, 0, q);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  barrier();
  opA.frag<0, 0>(fa0[0], 0u); opA.frag<1, 0>(fa0[1], 0u); opA.frag<2, 0>(fa0[2], 0u); opA.frag<3, 0>(fa0[3], 0u);
  opA.frag<4, 0>(fa0[4], 0u); opA.frag<5, 0>(fa0[5], 0u); opA.frag<6, 0>(fa0[6], 0u); opA.frag<7, 0>(fa0[7], 0u);
  opB.frag<0, 0>(fb0[0], 0u); opB.frag<1, 0>(fb0[1], 0u); opB.frag<2, 0>(fb0[2], 0u); opB.frag<3, 0>(fb0[3], 0u);
  opB.frag<4, 0>(fb0[4], 0u); opB.frag<5, 0>(fb0[5], 0u); opB.frag<6, 0>(fb0[6], 0u); opB.frag<7, 0>(fb0[7], 0u);
#pragma unroll
  for (int q = 0; q < 8; ++q) dma_piece(opA, opB, smem, 1, 1, q);  // nk >= 2 (host-checked)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  for (int t = 0; t < nk - 2; ++t) {
    MainState m{acc, fa0, fb0, fa1, fb1, opA, opB, smem, t, (uint32_t)((t & 1) * 2 * HALF),
                (uint32_t)(((t + 1) & 1) * 2 * HALF)};
    ktile<true, true>(m);
  }
  {
    const int t = nk - 2;
    MainState m{acc, fa0, fb0, fa1, fb1, opA, opB, smem, t, (uint32_t)((t & 1) * 2 * HALF),
                (uint32_t)(((t + 1) & 1) * 2 * HALF)};
    ktile<true, false>(m);
  }
  {
    const int t = nk - 1;
    MainState m{acc, fa0, fb0, fa1, fb1, opA, opB, smem, t, (uint32_t)((t & 1) * 2 * HALF),
                (uint32_t)(((t + 1) & 1) * 2 * HALF)};
    ktile<false, false>(m);
  }

  // epilogue: acc[i][j] lane l = row 16 i + (l & 15), columns 16 j + 4 (l >> 4) .. +3 of the quadrant
  const int64_t row0 = (int64_t)mt * 256 + wm * 128 + (lane & 15);
  const int col0 = nt * 256 + wn * 128 + 4 * (lane >> 4);
  // split: this split's slab of the workspace (plain stores); unsplit (one workgroup per output
  // tile): read-modify-write of the gradient itself
  const bool ws = wsp != nullptr;
  float* dst = ws ? wsp + (int64_t)z * M * N : Cf;
  const int64_t ld = ws ? (int64_t)N : ldc;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      f32x4* q = reinterpret_cast<f32x4*>(dst + (row0 + 16 * i) * ld + col0 + 16 * j);
      *q = ws ? acc[i][j] : *q + acc[i][j];
    }
}

}  // namespace w4t

// dW[M][N] += sum_s A_s[T][M]^T . B_s[T][N] (nseg segments; nseg == 1: A / B), K split `splits`
// ways of kps K-tiles (kps even, >= 2), partials to ws [splits * nseg][M][N] (nullptr: added into
// dW in place, splits * nseg == 1 only).  The caller merges ws (wgrad_reduce_kernel).
bool launch_wgrad4w(const uint16_t* const* as, const uint16_t* const* bs, int nseg, int T, int M, int N, int splits,
                    int kps, float* dW, float* ws, hipStream_t s) {
  if (M % 256 || N % 256 || T % 128 || nseg < 1 || nseg > w4t::MAXSEG || kps < 2 || (kps & 1)) return false;
  if (ws == nullptr && splits * nseg != 1) return false;
  const int ktot = T / 64;
  if ((int64_t)(splits - 1) * kps >= ktot || (int64_t)splits * kps < ktot) return false;
  if (ktot - (splits - 1) * kps < 2 || ((ktot - (splits - 1) * kps) & 1)) return false;
  w4t::Segs sg{};
  for (int i = 0; i < nseg; ++i) {
    sg.a[i] = (const bf16_t*)as[i];
    sg.b[i] = (const bf16_t*)bs[i];
  }
  sg.n = nseg > 1 ? nseg : 0;
  const int tiles = (M / 256) * (N / 256) * splits * nseg;
  hipLaunchKernelGGL(w4t::wgrad4w_kernel, dim3(tiles), dim3(256), 0, s, sg.a[0], (int64_t)M, sg.b[0], (int64_t)N, M,
                     N, ktot, kps, splits, dW, (int64_t)N, ws, sg);
  return true;
}

}  // namespace dpa
