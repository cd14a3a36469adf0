// Attention for sequence length 128, head_dim 64, bidirectional (the DiffuSeq /
// BERT shape, SURVEY K-M8): persistent kernels that stream (batch, head) items
// through LDS with global_load_lds prefetch, so the HBM traffic of item i+1
// overlaps the matrix-core work of item i.
//
// Both kernels: grid = 2 x #CUs persistent workgroups of 256 threads (4 waves),
// two resident per CU so every SIMD holds one wave of each and hides the other's
// LDS / MFMA / load latencies; items (b, h) strided over the grid.  All LDS accesses are inline asm so
// hipcc never drains the in-flight LDS-DMA with a vmcnt(0) before them.
//
// Forward (per item): S^T = K Q^T with the keys of a 32-query block in the
//   accumulators (softmax statistics lane-local, exact single pass: all 128
//   keys fit), P with attention dropout fed from the accumulators as the A
//   operand of O = P V (V read transposed), O staged through LDS to 16-byte
//   row stores.  LSE saved for the backward.
//
// Backward (per item, one kernel, no atomics, nothing recomputed twice):
//   wave w owns keys 32w..32w+31 (K/V fragments in registers) and sweeps the 4
//   query tiles: S = Q K^T, dP = dO V^T, P from the saved LSE,
//   dV += dropout(P)^T dO and dK += dS^T Q straight from the accumulators;
//   dS^T goes to LDS; after a barrier wave w computes dQ for queries
//   32w..32w+31 as dS K (both operands read transposed).  delta = rowsum(dO*O)
//   is formed in-kernel from a register prefetch of O.  dQ/dK/dV are staged
//   through LDS and written as whole 128-byte rows of the packed dqkv.
// Dropout bits: the same per-(query, key-pair) hash as attention.hip.
#include <cstdlib>
#include <utility>

#include "common.h"
#include "launchers.h"
#include "mfma.h"

namespace dpa {
namespace a128 {

constexpr int L = 128, HD = 64;
constexpr float ATT_C = 1.4426950408889634f / 8.0f;  // log2(e) / sqrt(64)
constexpr float LN2f = 0.6931471805599453f;
constexpr float LOG2Ef = 1.4426950408889634f;
constexpr int IMG = L * HD * 2;  // 16 KiB: one [128][64] bf16 image

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void glob_void;

struct DropCfg {
  uint32_t seedmix, thr16;
  float scale;
  bool on;
};
__device__ __forceinline__ DropCfg make_drop(float p, uint32_t seed, uint32_t offset, uint32_t bh) {
  DropCfg d;
  d.on = p > 0.f;
  d.thr16 = (uint32_t)(p * 65536.f + 0.5f);
  d.scale = d.on ? 1.f / (1.f - p) : 1.f;
  d.seedmix = lowbias32(seed ^ lowbias32((offset + rng_base()) * 0xC2B2AE3Du ^ (bh * 0x27D4EB2Fu)));
  return d;
}
__device__ __forceinline__ uint32_t drop_hash(const DropCfg& d, int q, int key) {
  return mix32(d.seedmix ^ ((uint32_t)q * 0x9E3779B1u) ^ ((uint32_t)(key >> 1) * 0x85EBCA77u));
}
__device__ __forceinline__ bool keep_from(const DropCfg& d, uint32_t h, int key) {
  const uint32_t r = (key & 1) ? (h >> 16) : (h & 0xffffu);
  return r >= d.thr16;
}
// keep_from for a per-lane key parity: sh = 16 (even key: low half) or 0 (odd key: high half);
// (h << sh) >= thr16 << 16 is the same test in two ops instead of four (no select of halves)
__device__ __forceinline__ bool keep_sh(const DropCfg& d, uint32_t h, uint32_t sh) {
  return (h << sh) >= (d.thr16 << 16);
}
__device__ __forceinline__ bool keep_bit(const DropCfg& d, int q, int key) {
  return keep_from(d, drop_hash(d, q, key), key);
}

// ---- LDS access (inline asm) ------------------------------------------------
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) char*)p);
}
__device__ __forceinline__ bf16x8 rd128(uint32_t a) {
  bf16x8 f;
  asm volatile("ds_read_b128 %0, %1" : "=v"(f) : "v"(a));
  return f;
}
__device__ __forceinline__ bf16x4 rdtr(uint32_t a) {
  bf16x4 f;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(f) : "v"(a));
  return f;
}
__device__ __forceinline__ f32x4 rd_f4(uint32_t a) {
  f32x4 f;
  asm volatile("ds_read_b128 %0, %1" : "=v"(f) : "v"(a));
  return f;
}
__device__ __forceinline__ void wr_b16(uint32_t a, uint16_t v) {
  asm volatile("ds_write_b16 %0, %1" ::"v"(a), "v"((uint32_t)v) : "memory");
}
__device__ __forceinline__ void wr_b32(uint32_t a, uint32_t v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void wr_b64(uint32_t a, uint32_t lo, uint32_t hi) {
  typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
  u32x2 v = {lo, hi};
  asm volatile("ds_write_b64 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void wr_f4(uint32_t a, const f32x4& v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ float rd_f1(uint32_t a) {
  float f;
  asm volatile("ds_read_b32 %0, %1" : "=v"(f) : "v"(a));
  return f;
}
__device__ __forceinline__ void lgkm0() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
// s_waitcnt vmcnt(n) for the counts the pipelines use (immediate operand).
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 17: asm volatile("s_waitcnt vmcnt(17)" ::: "memory"); break;
    case 22: asm volatile("s_waitcnt vmcnt(22)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

__device__ __forceinline__ void barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// [128][64] row-form image, 128-B rows, chunk XOR (row >> 1) & 7
__device__ __forceinline__ uint32_t off_r(int row, int ch) {
  return (uint32_t)(row * 128 + ((ch ^ ((row >> 1) & 7)) << 4));
}
// [128][128] image (dS^T), 256-B rows; XOR serving transposed reads conflict-free
__device__ __forceinline__ uint32_t off_s(int row, int ch) {
  return (uint32_t)(row * 256 + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4));
}

// Row-form fragment: A/B operand rows r0 + (lane & 31), k = 16s + 8h + j
__device__ __forceinline__ bf16x8 frag_r(uint32_t img, int r0, int s, int lane) {
  return rd128(img + off_r(r0 + (lane & 31), 2 * s + (lane >> 5)));
}
// Transposed read (k along image rows), permuted k order for accumulator
// operands: rows r0 + 4h + q and r0 + 8 + 4h + q, column col0 + (lane & 31).
__device__ __forceinline__ bf16x8 frag_tp(uint32_t img, int r0, int col0, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3, h = lane >> 5;
  const int col = col0 + 16 * (g & 1) + 4 * p;
  const int ra = r0 + 4 * h + q;
  return cat44(rdtr(img + off_r(ra, col >> 3) + (col & 7) * 2),
               rdtr(img + off_r(ra + 8, col >> 3) + (col & 7) * 2));
}
// Transposed read, natural k order: rows r0 + 8h + q and r0 + 8h + 4 + q.
__device__ __forceinline__ bf16x8 frag_tn_r(uint32_t img, int r0, int col0, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3, h = lane >> 5;
  const int col = col0 + 16 * (g & 1) + 4 * p;
  const int ra = r0 + 8 * h + q;
  return cat44(rdtr(img + off_r(ra, col >> 3) + (col & 7) * 2),
               rdtr(img + off_r(ra + 4, col >> 3) + (col & 7) * 2));
}
__device__ __forceinline__ bf16x8 frag_tn_s(uint32_t img, int r0, int col0, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3, h = lane >> 5;
  const int col = col0 + 16 * (g & 1) + 4 * p;
  const int ra = r0 + 8 * h + q;
  return cat44(rdtr(img + off_s(ra, col >> 3) + (col & 7) * 2),
               rdtr(img + off_s(ra + 4, col >> 3) + (col & 7) * 2));
}

// DMA a [128 rows][64] bf16 tile (row stride ld elements) into a row-form image:
// 16 pieces of 8 rows; wave w issues pieces 4w..4w+3.
__device__ __forceinline__ void dma_img(char* img, const bf16_t* src, int64_t ld, int w, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int pc = w * 4 + i;
    const int row = pc * 8 + (lane >> 3), phys = lane & 7;
    // 32-bit lane offset (row < 128, ld < 2^24: one full-rate 24-bit multiply) on the uniform
    // base, not a 64-bit product per piece
    const uint32_t off = __umul24((uint32_t)row, (uint32_t)ld) + (uint32_t)((phys ^ ((row >> 1) & 7)) << 3);
    const bf16_t* g = src + off;
    __builtin_amdgcn_global_load_lds((glob_void*)g, (lds_void*)(img + pc * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ float bflo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bfhi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// Where Q / K / V of (batch b, head h) live: element (l, d) of Q at
// qkv + b sb + h sh + l ld + d, K and V at + sw and + 2 sw.
//  token-major (the Linear output [B, L, 3, H, HD]): rows of 3 H HD elements, a head's
//    128-byte row segments strided by the whole token row;
//  head-major [B, 3 H, L, HD] (the QKV GEMM's head-major epilogue store): every [L][HD] head
//    block is 16 KiB contiguous.
struct QkvLayout {
  int64_t sb, sh, sw, ld;
};
__device__ __forceinline__ QkvLayout qkv_layout(int H, int hmaj) {
  QkvLayout q;
  q.sb = 3LL * H * L * HD;
  if (hmaj) {
    q.sh = (int64_t)L * HD;
    q.sw = (int64_t)H * L * HD;
    q.ld = HD;
  } else {
    q.sh = HD;
    q.sw = (int64_t)H * HD;
    q.ld = 3LL * H * HD;
  }
  return q;
}

// ---- immediate-offset LDS access (per-lane base VGPR + compile-time offset) --
template <int IMM>
__device__ __forceinline__ bf16x8 rd128o(uint32_t a) {
  bf16x8 f;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f) : "v"(a), "i"(IMM));
  return f;
}
template <int IMM>
__device__ __forceinline__ f32x4 rdf4o(uint32_t a) {
  f32x4 f;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f) : "v"(a), "i"(IMM));
  return f;
}
template <int IMM>
__device__ __forceinline__ bf16x4 rdtro(uint32_t a) {
  bf16x4 f;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(f) : "v"(a), "i"(IMM));
  return f;
}
template <int IMM>
__device__ __forceinline__ void wr16o(uint32_t a, uint16_t v) {
  asm volatile("ds_write_b16 %0, %1 offset:%2" ::"v"(a), "v"((uint32_t)v), "i"(IMM) : "memory");
}

// ============================================================================
// forward
// ============================================================================
// DROP: attention dropout on (p > 0) at compile time (no per-score wave-uniform branch).
template <bool DROP>
__global__ void __launch_bounds__(256, 2) attn128_fwd_kernel(const bf16_t* __restrict__ qkv,
                                                            bf16_t* __restrict__ out,
                                                            float* __restrict__ lse, int B, int H,
                                                            float p, uint32_t seed, uint32_t offset,
                                                            int hmaj) {
  // two workgroups per CU (8 waves: one wave of each on every SIMD hides the
  // other's latencies); per workgroup 2 stages at s * 32K: K, V images.  Q goes
  // straight to fragment registers (each wave needs only its 32 queries).
  __shared__ __attribute__((aligned(1024))) char smem[2 * 2 * IMG];
  const int w = threadIdx.x >> 6;
  const int nitems = B * H;
  const QkvLayout lay = qkv_layout(H, hmaj);
  const int64_t ld = lay.ld, ldo = (int64_t)H * HD;
  const uint32_t sb = lds_u32(smem);

  bf16x8 qpf[4];
  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;
  auto issue = [&](int item, int stg) {
    const int b = item / H, hd = item - b * H;
    const bf16_t* qb = qkv + (int64_t)b * lay.sb + (int64_t)hd * lay.sh;
    char* base = smem + stg * 2 * IMG;
    dma_img(base, qb + lay.sw, ld, w, lane);
    dma_img(base + IMG, qb + 2 * lay.sw, ld, w, lane);
    const bf16_t* qrow = qb + (int64_t)(w * 32 + (lane & 31)) * ld;
#pragma unroll
    for (int s = 0; s < 4; ++s) qpf[s] = ld_frag(qrow + 16 * s + 8 * hf);
  };

  const int G = gridDim.x;
  int item = blockIdx.x;
  if (item < nitems) issue(item, 0);
#pragma unroll 1
  for (int k = 0; item < nitems; ++k, item += G) {
    const int cur = k & 1;
    // This item's K/V DMA and Q loads landed; only the previous item's 5 stores
    // (lse + 4 O rows) were issued after them (in-order retire).
    if (k == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    barrier();
    bf16x8 qf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = qpf[s];
    if (item + G < nitems) issue(item + G, cur ^ 1);
    const uint32_t ki = sb + cur * 2 * IMG, vi = ki + IMG;
    const int b = item / H, hd = item - b * H;
    const DropCfg dc = make_drop(p, seed, offset, (uint32_t)item);
    const int q = w * 32 + (lane & 31);
    // per-lane LDS fragment bases, derived once per item through an opaque zero (hoisted out of
    // the item loop they would stay live across it); every read is base + immediate
    uint32_t z0;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z0));
    const int ln = lane + (int)z0;
    uint32_t rb[4], tp;
    {
      const int r = ln & 31, sw_r = (r >> 1) & 7, h = ln >> 5;
#pragma unroll
      for (int s = 0; s < 4; ++s) rb[s] = (uint32_t)(r * 128 + (((2 * s + h) ^ sw_r) << 4));
      // transposed V fragment rows r0 + 4h + qq (+8), r0 % 16 == 0: swizzle (2h + qq/2); the
      // second column block is +64 bytes, the +8 rows' read +1024 + (1 - dt) * 64
      const int g = ln >> 4, li = ln & 15, qq = li >> 2, pp = li & 3;
      const int cp = 2 * (g & 1) + (pp >> 1), e = (pp & 1) * 8;
      tp = (uint32_t)((4 * h + qq) * 128 + ((cp ^ ((2 * h + (qq >> 1)) & 7)) << 4) + e);
    }

    // S^T (keys in registers, query on the lane)
    f32x16 acc[4];
#define DPA_FWD_S(T)                                                            \
  {                                                                            \
    bf16x8 kf[4];                                                              \
    kf[0] = rd128o<T * 4096>(ki + rb[0]);                                      \
    kf[1] = rd128o<T * 4096>(ki + rb[1]);                                      \
    kf[2] = rd128o<T * 4096>(ki + rb[2]);                                      \
    kf[3] = rd128o<T * 4096>(ki + rb[3]);                                      \
    lgkm0();                                                                   \
    acc[T] = zero16();                                                         \
    for (int s = 0; s < 4; ++s) acc[T] = mfma32(kf[s], qf[s], acc[T]);         \
  }
    DPA_FWD_S(0) DPA_FWD_S(1) DPA_FWD_S(2) DPA_FWD_S(3)
#undef DPA_FWD_S
    // max over the raw scores, the softmax scale folded into the exp's FMA
    float m = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) m = fmaxf(m, acc[t][i]);
    m = fmaxf(m, __shfl_xor(m, 32, 64)) * ATT_C;
    float l = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float e = fexp2(fmaf(acc[t][i], ATT_C, -m));
        acc[t][i] = e;
        l += e;
      }
    l += __shfl_xor(l, 32, 64);
    const float inv_l = 1.f / l;
    if (hf == 0) lse[(int64_t)item * L + q] = (m + log2f(l)) * LN2f;
    f32x16 o[2];
    o[0] = zero16();
    o[1] = zero16();
    // 1 / l and the kept probabilities' 1 / (1 - p) scale the scores here (queries on the lane;
    // the output's rows sit on registers and would need a cross-lane fetch per row)
    const float fk = DROP ? inv_l * dc.scale : inv_l;
    // key pair of register 2j of tile t: t * 16 + (j & 1) + 4 (j >> 1) + 2 hf
    const uint32_t hq = (uint32_t)q * 0x9E3779B1u, hk0 = (uint32_t)(2 * hf) * 0x85EBCA77u;
    const uint32_t sq = dc.seedmix ^ hq, c8000 = 0x80008000u, c15 = 0x000F000Fu;
    const uint32_t thr_h = min(dc.thr16, 65535u) ^ 0x8000u, ts2 = thr_h | (thr_h << 16);
    bf16x8 pfr[4][2];  // P (dropped) as A fragments: registers 2j, 2j + 1 = one key pair, one dword
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      uint32_t pk[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) pk[j] = pack_bf2(acc[t][2 * j] * fk, acc[t][2 * j + 1] * fk);
      if constexpr (DROP) {
#pragma unroll
        for (int j = 0; j < 8; ++j)  // drop_hash(dc, q, t * 32 + acc_row(2 j, hf)), per-lane terms hoisted
          pk[j] = drop_pair(pk[j], drop_hash_s(sq, hk0 + (uint32_t)(t * 16 + (j & 1) + 4 * (j >> 1)) * 0x85EBCA77u, c8000),
                            ts2, c15);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s)
        pfr[t][s] = __builtin_bit_cast(bf16x8, (u32x4){pk[4 * s], pk[4 * s + 1], pk[4 * s + 2], pk[4 * s + 3]});
    }
#define DPA_FWD_PV(T, S)                                                                            \
  {                                                                                                \
    const bf16x8 af = pfr[T][S];                                                                   \
    constexpr int R0 = (T * 32 + 16 * S) * 128;                                                    \
    const bf16x8 v0 = cat44(rdtro<IMG + R0>(ki + tp), rdtro<IMG + R0 + 1024 + 64>(ki + tp));       \
    const bf16x8 v1 = cat44(rdtro<IMG + R0 + 64>(ki + tp), rdtro<IMG + R0 + 1024>(ki + tp));       \
    lgkm0();                                                                                       \
    o[0] = mfma32(af, v0, o[0]);                                                                   \
    o[1] = mfma32(af, v1, o[1]);                                                                   \
  }
    DPA_FWD_PV(0, 0) DPA_FWD_PV(0, 1) DPA_FWD_PV(1, 0) DPA_FWD_PV(1, 1)
    DPA_FWD_PV(2, 0) DPA_FWD_PV(2, 1) DPA_FWD_PV(3, 0) DPA_FWD_PV(3, 1)
#undef DPA_FWD_PV
    // stage O (rows = queries) unswizzled in the K image (dead: every wave passed its S^T):
    // row 32w + 4h + (i&3) + 8(i>>2), column dt*32 + (lane&31) - all but the lane part immediate
    barrier();
    const uint32_t qi = ki;
    {
      const uint32_t ost = qi + (uint32_t)((32 * w + 4 * hf) * 128 + (ln & 31) * 2);
#define DPA_FWD_ST(I)                                                        \
  wr16o<((I & 3) + 8 * (I >> 2)) * 128>(ost, f2bf(o[0][I]));                 \
  wr16o<((I & 3) + 8 * (I >> 2)) * 128 + 64>(ost, f2bf(o[1][I]));
      DPA_FWD_ST(0) DPA_FWD_ST(1) DPA_FWD_ST(2) DPA_FWD_ST(3) DPA_FWD_ST(4) DPA_FWD_ST(5)
      DPA_FWD_ST(6) DPA_FWD_ST(7) DPA_FWD_ST(8) DPA_FWD_ST(9) DPA_FWD_ST(10) DPA_FWD_ST(11)
      DPA_FWD_ST(12) DPA_FWD_ST(13) DPA_FWD_ST(14) DPA_FWD_ST(15)
#undef DPA_FWD_ST
    }
    barrier();
    bf16_t* ob = out + (int64_t)b * L * ldo + (int64_t)hd * HD;
    {
      const uint32_t cpy = qi + (uint32_t)((tid >> 3) * 128 + (tid & 7) * 16);
      const bf16x8 c0 = rd128o<0>(cpy), c1 = rd128o<4096>(cpy), c2 = rd128o<8192>(cpy), c3 = rd128o<12288>(cpy);
      lgkm0();
      bf16_t* orow = ob + __umul24((uint32_t)(tid >> 3), (uint32_t)ldo) + (tid & 7) * 8;
      const int64_t r32 = 32 * ldo;
      *reinterpret_cast<bf16x8*>(orow) = c0;
      *reinterpret_cast<bf16x8*>(orow + r32) = c1;
      *reinterpret_cast<bf16x8*>(orow + 2 * r32) = c2;
      *reinterpret_cast<bf16x8*>(orow + 3 * r32) = c3;
    }
  }
}

// ============================================================================
// backward
// ============================================================================
// LDS (one stage per workgroup, two workgroups per CU so that one's loads
// overlap the other's math): Q, dO, K images; then lse2[128], delta[128].  V never
// goes through LDS: each wave needs only its 32 keys' V rows (fragment registers).
// Every fragment read is one of a handful of per-lane base addresses plus an
// immediate: the XOR swizzles are chosen so the tile offsets never interact
// with the lane bits (derivations at the bases below).
constexpr int BWD_BUF = 3 * IMG;
constexpr int BWD_STATS = BWD_BUF;
constexpr int I_Q = 0, I_DO = IMG, I_K = 2 * IMG;

struct BwdBases {
  uint32_t rb[4];     // row-form fragment, k-step s: row (lane & 31), chunk 2s + h
  uint32_t tp;        // transposed (permuted k) fragment of a Q / dO image, r0 = 0, dt = 0
  uint32_t tn1[2], tn2[2];  // transposed (natural k) fragment of the K image, per dt
  uint32_t ts1, ts2;  // transposed (natural k) fragment of the dS^T image, this wave's queries
  uint32_t stat;      // lse2 / delta rows 4h..: + 4 * (32t + 8g)
  uint32_t ost;       // unswizzled output staging: row 32w + 4h, col lane & 31
  uint32_t cpy;       // copy-out: row tid >> 3, chunk tid & 7 (unswizzled)
};

__device__ __forceinline__ BwdBases bwd_bases(int lane, int w, int tid) {
  BwdBases B;
  const int h = lane >> 5, g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int cp = 2 * (g & 1) + (p >> 1);  // chunk within a 32-column block
  const int e = (p & 1) * 8;
  const int r = lane & 31, sw_r = (r >> 1) & 7;
#pragma unroll
  for (int s = 0; s < 4; ++s) B.rb[s] = (uint32_t)(r * 128 + (((2 * s + h) ^ sw_r) << 4));
  // frag_tp rows r0 + 4h + q (+8): swizzle (2h + q/2) for r0 % 16 == 0; dt -> +64 /
  // second read +1024 + (1 - dt) * 64
  B.tp = (uint32_t)((4 * h + q) * 128 + ((cp ^ ((2 * h + (q >> 1)) & 7)) << 4) + e);
  // frag_tn (K) rows r0 + 8h + q and +4: swizzle (4h + q/2) and (4h + 2 + q/2)
#pragma unroll
  for (int dt = 0; dt < 2; ++dt) {
    B.tn1[dt] = (uint32_t)((8 * h + q) * 128 + (((4 * dt + cp) ^ ((4 * h + (q >> 1)) & 7)) << 4) + e);
    B.tn2[dt] = (uint32_t)((8 * h + q + 4) * 128 + (((4 * dt + cp) ^ ((4 * h + 2 + (q >> 1)) & 7)) << 4) + e);
  }
  // dS^T image (256-B rows, XOR ((row&3)<<2)|((row>>2)&3)), rows r0 + 8h + q (+4),
  // columns 32w + 16(g&1) + 4p
  B.ts1 = (uint32_t)((8 * h + q) * 256 + (((4 * w + cp) ^ ((q << 2) | (2 * h))) << 4) + e);
  B.ts2 = (uint32_t)((8 * h + q + 4) * 256 + (((4 * w + cp) ^ ((q << 2) | (2 * h + 1))) << 4) + e);
  B.stat = (uint32_t)(BWD_STATS + 16 * h);
  B.ost = (uint32_t)((32 * w + 4 * h) * 128 + (lane & 31) * 2);
  B.cpy = (uint32_t)((tid >> 3) * 128 + (tid & 7) * 16);
  return B;
}

// S = Q K^T and dP = dO V^T for query tile T (this wave's 32 keys on the lane)
template <int T, int S>
__device__ __forceinline__ void bwd_sdp_step(f32x16& sacc, f32x16& dpacc, uint32_t base,
                                             const BwdBases& B, uint32_t kbase,
                                             const bf16x8 (&vf)[4]) {
  const bf16x8 qf = rd128o<I_Q + T * 32 * 128>(base + B.rb[S]);
  const bf16x8 df = rd128o<I_DO + T * 32 * 128>(base + B.rb[S]);
  const bf16x8 kf = rd128o<I_K>(kbase + B.rb[S]);  // this wave's keys (re-read: VGPR budget)
  lgkm0();
  sacc = mfma32(qf, kf, sacc);
  dpacc = mfma32(df, vf[S], dpacc);
}

// dV += dropout(P)^T dO and dK += dS^T Q for k-step S of tile T, output columns DT
template <int T, int S, int DT>
__device__ __forceinline__ void bwd_dkv_step(f32x16 (&dv)[2], f32x16 (&dk)[2], const bf16x8& pf,
                                             const bf16x8& sf, uint32_t base, const BwdBases& B) {
  constexpr int R0 = (T * 32 + 16 * S) * 128;
  const bf16x8 tdo = cat44(rdtro<I_DO + R0 + DT * 64>(base + B.tp),
                           rdtro<I_DO + R0 + 1024 + (1 - DT) * 64>(base + B.tp));
  const bf16x8 tq = cat44(rdtro<I_Q + R0 + DT * 64>(base + B.tp),
                          rdtro<I_Q + R0 + 1024 + (1 - DT) * 64>(base + B.tp));
  lgkm0();
  dv[DT] = mfma32(pf, tdo, dv[DT]);
  dk[DT] = mfma32(sf, tq, dk[DT]);
}

// Per-lane dropout hash terms of one item: hq = (4 hf + (key & 1)) * C_Q and hk = (key >> 1) * C_K.
// The query of a hash is T*32 + 8G + 2j + 4hf + (key & 1) with T, G, j compile-time, so its
// product with C_Q is hq plus an immediate (mod 2^32): no quarter-rate v_mul_lo_u32 per hash.
struct HashTerms {
  uint32_t hq, hk, sh;  // sh: keep_sh shift of this lane's key parity
  int par;
};

template <int T, int G, bool DROP>
__device__ __forceinline__ void bwd_pds(f32x16& sacc, f32x16& dpacc, uint32_t base,
                                        const BwdBases& B, const DropCfg& dc, const HashTerms& ht) {
  const f32x4 lv = rdf4o<T * 128 + G * 32>(base + B.stat);
  const f32x4 dl = rdf4o<T * 128 + G * 32 + 512>(base + B.stat);
  lgkm0();
  // keys key and key^1 sit on adjacent lanes and need the same (query, key pair)
  // hashes: each lane computes two of the four and swaps for the rest (DPP)
  uint32_t hh[4];
  if constexpr (DROP) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      constexpr uint32_t CQ = 0x9E3779B1u;
      const uint32_t qt = ht.hq + (uint32_t)(T * 32 + 8 * G + 2 * j) * CQ;
      const uint32_t mine = mix32(dc.seedmix ^ qt ^ ht.hk);
      const uint32_t other = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mine, 0xB1, 0xF, 0xF, true);
      hh[2 * j] = ht.par ? other : mine;
      hh[2 * j + 1] = ht.par ? mine : other;
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = 4 * G + r;
    const float pr = fexp2(fmaf(sacc[i], ATT_C, -lv[r]));
    if constexpr (DROP) {
      // one select per score: the kept-and-scaled multiplier serves P and dP
      const float m = keep_sh(dc, hh[r], ht.sh) ? dc.scale : 0.f;
      sacc[i] = pr * m;
      dpacc[i] = pr * fmaf(dpacc[i], m, -dl[r]);
    } else {
      // no dropout: dS carries the 1/sqrt(64) gradient scale (exact in bf16, a power of two)
      // in the same FMA, so dQ / dK need no scaling pass; dl is delta / 8 here
      sacc[i] = pr;
      dpacc[i] = pr * fmaf(dpacc[i], 0.125f, -dl[r]);
    }
  }
}

template <int T, bool DROP>
__device__ __forceinline__ void bwd_tile(f32x16 (&dv)[2], f32x16 (&dk)[2], uint4 (&dsb)[2],
                                         uint32_t base, const BwdBases& B, uint32_t kbase,
                                         const bf16x8 (&vf)[4], const DropCfg& dc, const HashTerms& ht) {
  f32x16 sacc = zero16(), dpacc = zero16();
  bwd_sdp_step<T, 0>(sacc, dpacc, base, B, kbase, vf);
  bwd_sdp_step<T, 1>(sacc, dpacc, base, B, kbase, vf);
  bwd_sdp_step<T, 2>(sacc, dpacc, base, B, kbase, vf);
  bwd_sdp_step<T, 3>(sacc, dpacc, base, B, kbase, vf);
  // P, dS on this lane's query rows 32T + 8g + 4h + r (statistics read per group g)
  bwd_pds<T, 0, DROP>(sacc, dpacc, base, B, dc, ht);
  bwd_pds<T, 1, DROP>(sacc, dpacc, base, B, dc, ht);
  bwd_pds<T, 2, DROP>(sacc, dpacc, base, B, dc, ht);
  bwd_pds<T, 3, DROP>(sacc, dpacc, base, B, dc, ht);
  {
    const bf16x8 pf = acc_to_frag(sacc, 0), sf = acc_to_frag(dpacc, 0);
    dsb[0] = __builtin_bit_cast(uint4, sf);
    bwd_dkv_step<T, 0, 0>(dv, dk, pf, sf, base, B);
    bwd_dkv_step<T, 0, 1>(dv, dk, pf, sf, base, B);
  }
  {
    const bf16x8 pf = acc_to_frag(sacc, 1), sf = acc_to_frag(dpacc, 1);
    dsb[1] = __builtin_bit_cast(uint4, sf);
    bwd_dkv_step<T, 1, 0>(dv, dk, pf, sf, base, B);
    bwd_dkv_step<T, 1, 1>(dv, dk, pf, sf, base, B);
  }
}

template <int KS>
__device__ __forceinline__ void bwd_dq_step(f32x16 (&dq)[2], uint32_t base, const BwdBases& B) {
  const bf16x8 af = cat44(rdtro<KS * 16 * 256>(base + B.ts1), rdtro<KS * 16 * 256>(base + B.ts2));
  const bf16x8 b0 = cat44(rdtro<I_K + KS * 16 * 128>(base + B.tn1[0]),
                          rdtro<I_K + KS * 16 * 128>(base + B.tn2[0]));
  const bf16x8 b1 = cat44(rdtro<I_K + KS * 16 * 128>(base + B.tn1[1]),
                          rdtro<I_K + KS * 16 * 128>(base + B.tn2[1]));
  lgkm0();
  dq[0] = mfma32(af, b0, dq[0]);
  dq[1] = mfma32(af, b1, dq[1]);
}

// One b16 LDS write per register (converting registers in pairs and writing the high half
// with ds_write_b16_d16_hi saves 48 conversions per item but made the compiler allocate 256
// VGPRs and spill).  Row of register i: 32w + 4h + (i&3) + 8(i>>2), column DT*32 + (lane&31): all but the lane
// part immediate.
template <int X, int DT, int M>
__device__ __forceinline__ void bwd_stage_pair(const f32x16& acc, float scale, uint32_t a) {
  constexpr int I0 = 2 * M, I1 = 2 * M + 1;
  wr16o<X * IMG + ((I0 & 3) + 8 * (I0 >> 2)) * 128 + DT * 64>(a, f2bf(acc[I0] * scale));
  wr16o<X * IMG + ((I1 & 3) + 8 * (I1 >> 2)) * 128 + DT * 64>(a, f2bf(acc[I1] * scale));
}

template <int X, int DT, int... M>
__device__ __forceinline__ void bwd_stage_out_seq(const f32x16& acc, float scale, uint32_t a,
                                                  std::integer_sequence<int, M...>) {
  (bwd_stage_pair<X, DT, M>(acc, scale, a), ...);
}

template <int X, int DT>
__device__ __forceinline__ void bwd_stage_out(const f32x16& acc, float scale, uint32_t a) {
  bwd_stage_out_seq<X, DT>(acc, scale, a, std::make_integer_sequence<int, 8>{});
}

// DROP: attention dropout on (p > 0), a template parameter so the per-score dropout work
// carries no wave-uniform branch (~130 scalar branches and their exec bookkeeping per item)
template <bool DROP>
__global__ void __launch_bounds__(256, 2) attn128_bwd_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ out, const bf16_t* __restrict__ dout,
    const float* __restrict__ lse, bf16_t* __restrict__ dqkv, float* __restrict__ colpart, int B,
    int H, float p, uint32_t seed, uint32_t offset, int hmaj) {
  __shared__ __attribute__((aligned(1024))) char smem[BWD_STATS + 2 * L * 4];
  const int nitems = B * H;
  const QkvLayout lay = qkv_layout(H, hmaj);
  // qkv is read in its own layout; dqkv is always written token-major [B, L, 3 H HD]
  const int64_t ld = 3LL * H * HD, ldo = (int64_t)H * HD;
  const uint32_t sb = lds_u32(smem);
  const int w = threadIdx.x >> 6;
  const int kb = w * 32;

  const int G = gridDim.x;
  for (int item = blockIdx.x; item < nitems; item += G) {
    // Every lane-dependent quantity is derived from the thread id through an
    // opaque zero, once per item: otherwise LICM hoists ~150 per-lane constants
    // (fragment addresses, DMA offsets, per-query hash terms) out of the item
    // loop, where they overflow the 256-VGPR budget of 2 waves/SIMD and spill.
    uint32_t z0;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z0));
    const int tid = (int)(threadIdx.x + z0), lane = tid & 63, hf = lane >> 5;
    const int key = kb + (lane & 31);
    const BwdBases BB = bwd_bases(lane, w, tid);
    const uint32_t base = sb;
    const int b = item / H, hd = item - b * H;
    const bf16_t* qb = qkv + (int64_t)b * lay.sb + (int64_t)hd * lay.sh;
    dma_img(smem + I_Q, qb, lay.ld, w, lane);
    dma_img(smem + I_DO, dout + (int64_t)b * L * ldo + (int64_t)hd * HD, ldo, w, lane);
    dma_img(smem + I_K, qb + lay.sw, lay.ld, w, lane);
    uint4 opf[4];
    {
      const bf16_t* orow = out + ((int64_t)b * L * ldo + (int64_t)hd * HD) +
                           (__umul24((uint32_t)(tid >> 1), (uint32_t)ldo) + (uint32_t)(tid & 1) * 32);
#pragma unroll
      for (int c = 0; c < 4; ++c) opf[c] = *reinterpret_cast<const uint4*>(orow + c * 8);
    }
    bf16x8 vf[4];
    {
      const bf16_t* vrow = (qb + 2 * lay.sw) + __umul24((uint32_t)key, (uint32_t)lay.ld);
#pragma unroll
      for (int s = 0; s < 4; ++s) vf[s] = ld_frag(vrow + 16 * s + 8 * hf);
    }
    const float lpf = tid < L ? lse[(int64_t)item * L + tid] : 0.f;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();
    // delta = rowsum(dO * O) and lse (log2 units) -> LDS
    {
      const int row = tid >> 1, half = tid & 1;
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const bf16x8 dv = rd128(base + I_DO + off_r(row, half * 4 + c));
        lgkm0();
        const uint32_t ow[4] = {opf[c].x, opf[c].y, opf[c].z, opf[c].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t dw = (uint32_t)(uint16_t)dv[2 * e] | ((uint32_t)(uint16_t)dv[2 * e + 1] << 16);
          s += bflo(dw) * bflo(ow[e]) + bfhi(dw) * bfhi(ow[e]);
        }
      }
      s += __shfl_xor(s, 1, 64);
      if (half == 0) wr_b32(base + BWD_STATS + 512 + row * 4, __float_as_uint(DROP ? s : s * 0.125f));
      if (tid < L) wr_b32(base + BWD_STATS + tid * 4, __float_as_uint(lpf * LOG2Ef));
    }
    barrier();

    const DropCfg dc = make_drop(p, seed, offset, (uint32_t)item);
    HashTerms ht;
    ht.par = key & 1;
    ht.sh = ht.par ? 0u : 16u;
    ht.hq = (uint32_t)(4 * hf + ht.par) * 0x9E3779B1u;
    ht.hk = (uint32_t)(key >> 1) * 0x85EBCA77u;
    const uint32_t kbase = base + kb * 128;
    f32x16 dk[2], dv[2];
    uint4 dsb[4][2];  // dS as bf16 (the exact A-operand packing), 8 registers per tile
    dk[0] = zero16(); dk[1] = zero16(); dv[0] = zero16(); dv[1] = zero16();
    bwd_tile<0, DROP>(dv, dk, dsb[0], base, BB, kbase, vf, dc, ht);
    bwd_tile<1, DROP>(dv, dk, dsb[1], base, BB, kbase, vf, dc, ht);
    bwd_tile<2, DROP>(dv, dk, dsb[2], base, BB, kbase, vf, dc, ht);
    bwd_tile<3, DROP>(dv, dk, dsb[3], base, BB, kbase, vf, dc, ht);
    // dS^T -> LDS over Q + dO (dead once every wave is here): [128 keys][128 q], 256-B rows
    barrier();
    {
      const int fk = ((key & 3) << 2) | ((key >> 2) & 3);
      const uint32_t rowa = base + key * 256 + 8 * hf;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const uint4 v = dsb[t][g >> 1];
          const uint32_t lo = (g & 1) ? v.z : v.x, hi = (g & 1) ? v.w : v.y;
          wr_b64(rowa + (((4 * t + g) ^ fk) << 4), lo, hi);
        }
    }
    barrier();
    // dQ for queries 32w..32w+31: sum over keys of dS[q][key] K[key][d]
    f32x16 dq[2];
    dq[0] = zero16();
    dq[1] = zero16();
    bwd_dq_step<0>(dq, base, BB); bwd_dq_step<1>(dq, base, BB);
    bwd_dq_step<2>(dq, base, BB); bwd_dq_step<3>(dq, base, BB);
    bwd_dq_step<4>(dq, base, BB); bwd_dq_step<5>(dq, base, BB);
    bwd_dq_step<6>(dq, base, BB); bwd_dq_step<7>(dq, base, BB);
    // stage dQ (rows = queries of wave w), dK, dV (rows = keys of wave w), unswizzled
    barrier();
    const uint32_t oa = base + BB.ost;
    constexpr float gs = DROP ? 0.125f : 1.f;  // without dropout dS already carried the 1/8
    bwd_stage_out<0, 0>(dq[0], gs, oa); bwd_stage_out<0, 1>(dq[1], gs, oa);
    bwd_stage_out<1, 0>(dk[0], gs, oa); bwd_stage_out<1, 1>(dk[1], gs, oa);
    bwd_stage_out<2, 0>(dv[0], 1.f, oa);    bwd_stage_out<2, 1>(dv[1], 1.f, oa);
    barrier();
    bf16_t* gb = dqkv + (int64_t)b * L * ld + (int64_t)hd * HD;
    const uint32_t ca = base + BB.cpy;
    const int crow = tid >> 3, cch = tid & 7;
    // this thread's row segment once; the 12 stores add wave-uniform offsets (no per-store
    // 64-bit multiply of the row index by ld)
    const uint32_t roff = __umul24((uint32_t)crow, (uint32_t)ld) + (uint32_t)cch * 8;
    const int64_t s32 = 32 * ld, sq = (int64_t)H * HD;
    // Column sums of the bf16 dQ/dK/dV this item writes (the qkv bias gradient,
    // so the wgrad GEMM needs no column-sum pass): each thread sums its 4 rows.
    float cs[3][8];
#define DPA_CP(C)                                                                         \
  {                                                                                       \
    const bf16x8 v = rd128o<(C >> 2) * IMG + (C & 3) * 4096>(ca);                         \
    lgkm0();                                                                              \
    *reinterpret_cast<bf16x8*>((gb + ((C & 3) * s32 + (C >> 2) * sq)) + roff) = v;         \
    _Pragma("unroll") for (int j = 0; j < 8; ++j) {                                       \
      const float f = __uint_as_float((uint32_t)(uint16_t)v[j] << 16);                    \
      cs[C >> 2][j] = (C & 3) ? cs[C >> 2][j] + f : f;                                    \
    }                                                                                     \
  }
    DPA_CP(0) DPA_CP(1) DPA_CP(2) DPA_CP(3) DPA_CP(4) DPA_CP(5)
    DPA_CP(6) DPA_CP(7) DPA_CP(8) DPA_CP(9) DPA_CP(10) DPA_CP(11)
#undef DPA_CP
    barrier();  // staging fully read before the next item's DMA lands on it
    if (colpart != nullptr) {
      // [32 row groups][192 columns] fp32 partials over the (now free) staging area
      const uint32_t pa = base + (uint32_t)(crow * 192 + cch * 8) * 4;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        wr_f4(pa + q * 256, f32x4{cs[q][0], cs[q][1], cs[q][2], cs[q][3]});
        wr_f4(pa + q * 256 + 16, f32x4{cs[q][4], cs[q][5], cs[q][6], cs[q][7]});
      }
      barrier();
      if (tid < 192) {
        // inline-asm LDS reads carry no implicit wait: load all, lgkmcnt(0), then add
        float v[32];
#pragma unroll
        for (int r = 0; r < 32; ++r) v[r] = rd_f1(base + (uint32_t)(r * 192 + tid) * 4);
        lgkm0();
        float t = 0.f;
#pragma unroll
        for (int r = 0; r < 32; ++r) t += v[r];
        colpart[(int64_t)item * 192 + tid] = t;
      }
      barrier();
    }
  }
}

// ============================================================================
// forward, head_dim 128 (DiffuSeq-XL: 2048 / 16 heads), token-major qkv
// ============================================================================
// Same item stream as attn128_fwd_kernel, with [128][128] K / V images (256-B rows, the
// swz_x256 chunk XOR: conflict-free for both the row-form ds_read_b128 S^T operand and the
// transposed V reads).  Two stages of 64 KiB fill the LDS, so ONE workgroup per CU (4 waves,
// up to 512 registers each): the next item's K / V DMA and Q loads are always in flight
// while this item computes; at ~8.4 MFLOP per 128 KiB of traffic the kernel is HBM-bound.
// Dropout / LSE / output conventions are those of the general kernels in attention.hip,
// whose backward it pairs with.
constexpr int HD2 = 128;
constexpr int IMG2 = L * HD2 * 2;  // 32 KiB
constexpr float ATT_C2 = 1.4426950408889634f * 0.08838834764831845f;  // log2(e) / sqrt(128)

__device__ __forceinline__ uint32_t off2(int row, int ch) {
  return (uint32_t)(row * 256 + ((ch ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 4));
}
// Row-form fragment of a [128][128] image: rows r0 + (lane & 31), k = 16s + 8h + j (s < 8)
__device__ __forceinline__ bf16x8 frag_r2(uint32_t img, int r0, int s, int lane) {
  return rd128(img + off2(r0 + (lane & 31), 2 * s + (lane >> 5)));
}
// Transposed read, permuted k order (accumulator operand): rows r0 + 4h + q and r0 + 8 + 4h + q
__device__ __forceinline__ bf16x8 frag_tp2(uint32_t img, int r0, int col0, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3, h = lane >> 5;
  const int col = col0 + 16 * (g & 1) + 4 * p;
  const int ra = r0 + 4 * h + q;
  return cat44(rdtr(img + off2(ra, col >> 3) + (col & 7) * 2),
               rdtr(img + off2(ra + 8, col >> 3) + (col & 7) * 2));
}
// DMA a [128 rows][128] bf16 tile (row stride ld elements): 32 pieces of 4 rows, wave w issues 8w..8w+7
// (32-bit row offsets: 128 rows x ld < 2^31 elements; 64-bit products were hoisted out of the
// item loop and spilled)
__device__ __forceinline__ void dma_img2(char* img, const bf16_t* src, int ld, int w, int lane) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int pc = w * 8 + i;
    const int row = pc * 4 + (lane >> 4), phys = lane & 15;
    const bf16_t* g = src + (row * ld + ((phys ^ (((row & 3) << 2) | ((row >> 2) & 3))) << 3));
    __builtin_amdgcn_global_load_lds((glob_void*)g, (lds_void*)(img + pc * 1024), 16, 0, 0);
  }
}

__global__ void __launch_bounds__(256, 1) attn128_fwd_d128_kernel(const bf16_t* __restrict__ qkv,
                                                                 bf16_t* __restrict__ out,
                                                                 float* __restrict__ lse, int B, int H,
                                                                 float p, uint32_t seed, uint32_t offset) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * 2 * IMG2];
  const int w = threadIdx.x >> 6;
  const int nitems = B * H;
  const int64_t ld = 3LL * H * HD2, ldo = (int64_t)H * HD2, sb = 3LL * H * L * HD2;
  const uint32_t sbase = lds_u32(smem);
  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;

  bf16x8 qpf[8];
  auto issue = [&](int item, int stg) {
    const int b = item / H, hd = item - b * H;
    const bf16_t* qb = qkv + (int64_t)b * sb + (int64_t)hd * HD2;
    char* base = smem + stg * 2 * IMG2;
    dma_img2(base, qb + (int64_t)H * HD2, (int)ld, w, lane);
    dma_img2(base + IMG2, qb + 2LL * H * HD2, (int)ld, w, lane);
    const bf16_t* qrow = qb + (int64_t)(w * 32 + (lane & 31)) * ld;
#pragma unroll
    for (int s = 0; s < 8; ++s) qpf[s] = ld_frag(qrow + 16 * s + 8 * hf);
  };

  const int G = gridDim.x;
  int item = blockIdx.x;
  if (item < nitems) issue(item, 0);
  for (int k = 0; item < nitems; ++k, item += G) {
    const int cur = k & 1;
    // this item's K/V DMA and Q loads landed; only the previous item's 9 stores (lse + 8 O
    // chunks) were issued after them (in-order retire)
    if (k == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
    barrier();
    bf16x8 qf[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) qf[s] = qpf[s];
    if (item + G < nitems) issue(item + G, cur ^ 1);
    const uint32_t ki = sbase + cur * 2 * IMG2, vi = ki + IMG2;
    const int b = item / H, hd = item - b * H;
    const DropCfg dc = make_drop(p, seed, offset, (uint32_t)item);
    const int q = w * 32 + (lane & 31);

    // S^T (keys in registers, query on the lane)
    f32x16 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      acc[t] = zero16();
#pragma unroll
      for (int hs = 0; hs < 2; ++hs) {
        bf16x8 kf[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) kf[s] = frag_r2(ki, t * 32, 4 * hs + s, lane);
        lgkm0();
#pragma unroll
        for (int s = 0; s < 4; ++s) acc[t] = mfma32(kf[s], qf[4 * hs + s], acc[t]);
      }
    }
    float m = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        acc[t][i] *= ATT_C2;
        m = fmaxf(m, acc[t][i]);
      }
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float l = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float e = fexp2(acc[t][i] - m);
        acc[t][i] = e;
        l += e;
      }
    l += __shfl_xor(l, 32, 64);
    const float inv_l = 1.f / l;
    const float fk = dc.on ? inv_l * dc.scale : inv_l;
    // key pair of register 2j of tile t: t * 16 + (j & 1) + 4 (j >> 1) + 2 hf
    const uint32_t hq = (uint32_t)q * 0x9E3779B1u, hk0 = (uint32_t)(2 * hf) * 0x85EBCA77u;
    const uint32_t sq = dc.seedmix ^ hq, c8000 = 0x80008000u, c15 = 0x000F000Fu;
    const uint32_t thr_h = min(dc.thr16, 65535u) ^ 0x8000u, ts2 = thr_h | (thr_h << 16);
    f32x16 o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] = zero16();
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      // registers 2j, 2j + 1 = one key pair = one packed dword, dropped as a pair (drop_pair)
      uint32_t pk[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) pk[j] = pack_bf2(acc[t][2 * j] * fk, acc[t][2 * j + 1] * fk);
      if (dc.on) {
#pragma unroll
        for (int j = 0; j < 8; ++j)  // drop_hash(dc, q, t * 32 + acc_row(2 j, hf)), per-lane terms hoisted
          pk[j] = drop_pair(pk[j], drop_hash_s(sq, hk0 + (uint32_t)(t * 16 + (j & 1) + 4 * (j >> 1)) * 0x85EBCA77u, c8000),
                            ts2, c15);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 af = __builtin_bit_cast(bf16x8, (u32x4){pk[4 * s], pk[4 * s + 1], pk[4 * s + 2], pk[4 * s + 3]});
        bf16x8 vf[4];
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) vf[dt] = frag_tp2(vi, t * 32 + 16 * s, dt * 32, lane);
        lgkm0();
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) o[dt] = mfma32(af, vf[dt], o[dt]);
      }
    }
    if (hf == 0) lse[(int64_t)item * L + q] = (m + log2f(l)) * LN2f;
    // stage O (rows = queries) in the K image (dead: every wave passed its S^T)
    barrier();
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = w * 32 + acc_row(i, hf), col = dt * 32 + (lane & 31);
        wr_b16(ki + off2(row, col >> 3) + (col & 7) * 2, f2bf(o[dt][i]));
      }
    barrier();
    bf16_t* ob = out + (int64_t)b * L * ldo + (int64_t)hd * HD2;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int idx = tid + c * 256, row = idx >> 4, ch = idx & 15;
      const bf16x8 v = rd128(ki + off2(row, ch));
      lgkm0();
      *reinterpret_cast<bf16x8*>(ob + (int64_t)row * ldo + ch * 8) = v;
    }
  }
}

// ============================================================================
// backward, head_dim 128 (DiffuSeq-XL), token-major qkv / dqkv: two persistent kernels
// ============================================================================
// The computation of the general kernels (attention.hip attn_bwd_q_kernel, then
// attn_bwd_kv_kernel; same dropout hashes, same delta hand-off), restructured for L = 128:
// one workgroup per CU walks (b, h) items; the item's operand images for all 128 rows come
// into one of two 64 KiB LDS stages by DMA while the previous item computes, and the next
// item's register operands are loaded one item ahead.  Outputs are staged through the dead
// stage image and written as 16-B row chunks (the general kernels store 2 B per lane).
// wave-uniform vmcnt(N) for the counts used below
__device__ __forceinline__ void wait_vm2(int n) {
  switch (n) {
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// column sums of one item's 128 x 128 output block (bf16-rounded, scaled) -> dst[128]: lane sums
// over the wave's 16 rows per register column, the two lane halves, then the 4 waves via LDS
__device__ __forceinline__ void item_colsum128(const f32x16 (&v)[4], float scale, float* red, float* dst, int w,
                                               int lane, int tid) {
  const int hf = lane >> 5;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    float cs = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) cs += bf2f(f2bf(v[dt][i] * scale));
    cs += __shfl_xor(cs, 32, 64);
    if (hf == 0) red[w * HD2 + dt * 32 + (lane & 31)] = cs;
  }
  __syncthreads();
  if (tid < HD2) dst[tid] = red[tid] + red[HD2 + tid] + red[2 * HD2 + tid] + red[3 * HD2 + tid];
  __syncthreads();
}

// dQ (and delta = rowsum(dO * O), published for the dK/dV kernel).  Wave w owns queries
// 32w .. 32w + 31 (Q, dO fragments in registers); K, V images [128][128] per stage.
__global__ void __launch_bounds__(256, 1) attn128_bwd_q_d128_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ out, const bf16_t* __restrict__ dout,
    const float* __restrict__ lse, float* __restrict__ delta, bf16_t* __restrict__ dqkv, int B, int H, float p,
    uint32_t seed, uint32_t offset, float* __restrict__ colpart) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * 2 * IMG2];
  __shared__ float cred[4 * HD2];
  const int w = threadIdx.x >> 6;
  const int nitems = B * H;
  const int64_t ld = 3LL * H * HD2, ldo = (int64_t)H * HD2, sb = 3LL * H * L * HD2;
  const uint32_t sbase = lds_u32(smem);
  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;
  const int q = w * 32 + (lane & 31);

  bf16x8 qn[8], dn[8], on[8];
  auto issue = [&](int item, int stg) {
    const int b = item / H, hd = item - b * H;
    const bf16_t* qb = qkv + (int64_t)b * sb + (int64_t)hd * HD2;
    char* base = smem + stg * 2 * IMG2;
    dma_img2(base, qb + (int64_t)H * HD2, (int)ld, w, lane);
    dma_img2(base + IMG2, qb + 2LL * H * HD2, (int)ld, w, lane);
    const bf16_t* qrow = qb + (int64_t)q * ld;
    const bf16_t* drow = dout + ((int64_t)b * L + q) * ldo + (int64_t)hd * HD2;
    const bf16_t* orow = out + ((int64_t)b * L + q) * ldo + (int64_t)hd * HD2;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      qn[s] = ld_frag(qrow + 16 * s + 8 * hf);
      dn[s] = ld_frag(drow + 16 * s + 8 * hf);
      on[s] = ld_frag(orow + 16 * s + 8 * hf);
    }
  };

  const int G = gridDim.x;
  int item = blockIdx.x;
  if (item < nitems) issue(item, 0);
  for (int k = 0; item < nitems; ++k, item += G) {
    const int cur = k & 1;
    // this item's DMA and register loads landed; only the previous item's 8 dq stores are younger
    wait_vm2(k == 0 ? 0 : 8);
    barrier();
    bf16x8 qf[8], df[8];
    float dlt = 0.f;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      qf[s] = qn[s];
      df[s] = dn[s];
#pragma unroll
      for (int j = 0; j < 8; ++j) dlt += bf2f(df[s][j]) * bf2f(on[s][j]);
    }
    dlt += __shfl_xor(dlt, 32, 64);
    if (item + G < nitems) issue(item + G, cur ^ 1);
    const int b = item / H, hd = item - b * H;
    const int64_t lrow = (int64_t)item * L;
    if (hf == 0) delta[lrow + q] = dlt;
    const float lse2 = lse[lrow + q] * 1.4426950408889634f;
    const uint32_t ki = sbase + cur * 2 * IMG2, vi = ki + IMG2;
    const DropCfg dc = make_drop(p, seed, offset, (uint32_t)item);
    const uint32_t qterm = (uint32_t)q * 0x9E3779B1u;
    f32x16 dq[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[dt] = zero16();
#pragma unroll 1
    for (int t = 0; t < 4; ++t) {
      f32x16 sacc = zero16(), dpacc = zero16();
#pragma unroll
      for (int hs = 0; hs < 2; ++hs) {
        bf16x8 kf[4], vf[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          kf[s] = frag_r2(ki, t * 32, 4 * hs + s, lane);
          vf[s] = frag_r2(vi, t * 32, 4 * hs + s, lane);
        }
        lgkm0();
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          sacc = mfma32(kf[s], qf[4 * hs + s], sacc);
          dpacc = mfma32(vf[s], df[4 * hs + s], dpacc);
        }
      }
      uint32_t hh[8];
      if (dc.on) {
        const uint32_t kt0 = (uint32_t)((t * 32 + 4 * hf) >> 1) * 0x85EBCA77u;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          hh[j] = mix32(dc.seedmix ^ qterm ^ (kt0 + (uint32_t)(((2 * j & 3) + 8 * (j >> 1)) >> 1) * 0x85EBCA77u));
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) sacc[i] = fexp2(fmaf(sacc[i], ATT_C2, -lse2));
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float dpd = dpacc[i];
        if (dc.on) dpd = keep_from(dc, hh[i >> 1], i & 1) ? dpd * dc.scale : 0.f;
        sacc[i] = sacc[i] * (dpd - dlt);
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 sf = acc_to_frag(sacc, s);
        bf16x8 kt[4];
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) kt[dt] = frag_tp2(ki, t * 32 + 16 * s, dt * 32, lane);
        lgkm0();
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) dq[dt] = mfma32(sf, kt[dt], dq[dt]);
      }
    }
    // stage dq (rows = queries, scaled by 1/sqrt(D)) in the K image, then 16-B row stores
    barrier();
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = w * 32 + acc_row(i, hf), col = dt * 32 + (lane & 31);
        wr_b16(ki + off2(row, col >> 3) + (col & 7) * 2, f2bf(dq[dt][i] * 0.08838834764831845f));
      }
    barrier();
    bf16_t* db = dqkv + (int64_t)b * L * ld + (int64_t)hd * HD2;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int idx = tid + c * 256, row = idx >> 4, ch = idx & 15;
      const bf16x8 v = rd128(ki + off2(row, ch));
      lgkm0();
      *reinterpret_cast<bf16x8*>(db + (int64_t)row * ld + ch * 8) = v;
    }
    if (colpart) item_colsum128(dq, 0.08838834764831845f, cred, colpart + (int64_t)item * 3 * HD2, w, lane, tid);
  }
}

// dK, dV.  Wave w owns keys 32w .. 32w + 31 (K, V fragments in registers); Q, dO images
// [128][128] plus the item's scaled LSE and delta per stage.
__global__ void __launch_bounds__(256, 1) attn128_bwd_kv_d128_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, bf16_t* __restrict__ dqkv, int B, int H, float p, uint32_t seed,
    uint32_t offset, float* __restrict__ colpart) {
  constexpr int STG = 2 * IMG2 + 1024;  // Q, dO images + lse[128] + delta[128]
  __shared__ __attribute__((aligned(1024))) char smem[2 * STG];
  __shared__ float cred[4 * HD2];
  const int w = threadIdx.x >> 6;
  const int nitems = B * H;
  const int64_t ld = 3LL * H * HD2, ldo = (int64_t)H * HD2, sb = 3LL * H * L * HD2;
  const uint32_t sbase = lds_u32(smem);
  const int tid = threadIdx.x, lane = tid & 63, hf = lane >> 5;
  const int key = w * 32 + (lane & 31);

  bf16x8 kf[8], vf[8];
  // this wave's K / V rows of `item` into kf / vf (issued for the next item once the current
  // item's last S / dP products have consumed them: no second register set)
  auto load_kv = [&](int item) {
    const int b = item / H, hd = item - b * H;
    const bf16_t* krow = qkv + (int64_t)b * sb + (int64_t)hd * HD2 + (int64_t)key * ld + (int64_t)H * HD2;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      kf[s] = ld_frag(krow + 16 * s + 8 * hf);
      vf[s] = ld_frag(krow + (int64_t)H * HD2 + 16 * s + 8 * hf);
    }
  };
  auto issue = [&](int item, int stg) {
    const int b = item / H, hd = item - b * H;
    const bf16_t* qb = qkv + (int64_t)b * sb + (int64_t)hd * HD2;
    char* base = smem + stg * STG;
    dma_img2(base, qb, (int)ld, w, lane);
    dma_img2(base + IMG2, dout + (int64_t)b * L * ldo + (int64_t)hd * HD2, (int)ldo, w, lane);
    // stats: wave 0/1 the LSE halves, wave 2/3 the delta halves (4 B per lane, one DMA each)
    const float* st = (w < 2 ? lse : delta) + (int64_t)item * L + (w & 1) * 64 + lane;
    __builtin_amdgcn_global_load_lds((glob_void*)st, (lds_void*)(base + 2 * IMG2 + w * 256), 4, 0, 0);
  };

  const int G = gridDim.x;
  int item = blockIdx.x;
  if (item < nitems) {
    issue(item, 0);
    load_kv(item);
  }
  for (int k = 0; item < nitems; ++k, item += G) {
    const int cur = k & 1;
    // this item's DMA (issued first) and K/V loads (issued after it) landed; only the previous
    // item's 16 dk/dv stores are younger
    wait_vm2(k == 0 ? 0 : 16);
    barrier();
    const bool has_next = item + G < nitems;
    if (has_next) issue(item + G, cur ^ 1);
    const int b = item / H, hd = item - b * H;
    const uint32_t qi = sbase + cur * STG, doi = qi + IMG2, sti = qi + 2 * IMG2;
    const DropCfg dc = make_drop(p, seed, offset, (uint32_t)item);
    f32x16 dk[4], dv[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) { dk[dt] = zero16(); dv[dt] = zero16(); }
    const int par = lane & 1;
    const uint32_t kt = (uint32_t)(key >> 1) * 0x85EBCA77u;
#pragma unroll 1
    for (int qt = 0; qt < 4; ++qt) {
      f32x16 sacc = zero16(), dpacc = zero16();
#pragma unroll
      for (int hs = 0; hs < 4; ++hs) {
        bf16x8 qa[2], da[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          qa[s] = frag_r2(qi, qt * 32, 2 * hs + s, lane);
          da[s] = frag_r2(doi, qt * 32, 2 * hs + s, lane);
        }
        lgkm0();
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          sacc = mfma32(qa[s], kf[2 * hs + s], sacc);
          dpacc = mfma32(da[s], vf[2 * hs + s], dpacc);
        }
      }
      if (qt == 3 && has_next) load_kv(item + G);  // kf / vf are dead for this item now
      // this lane's key, register i's query qt*32 + acc_row(i, hf) = rows 8G + 4hf + (0..3) of
      // group G: its LSE and delta as one 16-B LDS read each; dropout hashes per key pair
      // (lanes key, key^1 share them: each computes two of four and swaps the rest by DPP)
#pragma unroll
      for (int G = 0; G < 4; ++G) {
        const f32x4 lv = rd_f4(sti + (uint32_t)(qt * 32 + 8 * G + 4 * hf) * 4);
        const f32x4 dl = rd_f4(sti + 512 + (uint32_t)(qt * 32 + 8 * G + 4 * hf) * 4);
        uint32_t hh[4];
        if (dc.on) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const uint32_t qq = (uint32_t)(qt * 32 + 8 * G + 4 * hf + 2 * j + par);
            const uint32_t mine = mix32(dc.seedmix ^ (qq * 0x9E3779B1u) ^ kt);
            const uint32_t other = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mine, 0xB1, 0xF, 0xF, true);
            hh[2 * j] = par ? other : mine;
            hh[2 * j + 1] = par ? mine : other;
          }
        }
        lgkm0();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 4 * G + r;
          const float pr = fexp2(fmaf(sacc[i], ATT_C2, -lv[r] * 1.4426950408889634f));
          if (dc.on) {  // one select per score (see bwd_pds)
            const float m = keep_sh(dc, hh[r], (key & 1) ? 0u : 16u) ? dc.scale : 0.f;
            sacc[i] = pr * m;
            dpacc[i] = pr * fmaf(dpacc[i], m, -dl[r]);
          } else {
            sacc[i] = pr;
            dpacc[i] = pr * (dpacc[i] - dl[r]);
          }
        }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pf = acc_to_frag(sacc, s);
        const bf16x8 sf = acc_to_frag(dpacc, s);
#pragma unroll
        for (int dh = 0; dh < 2; ++dh) {
          bf16x8 tdo[2], tq[2];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            tdo[e] = frag_tp2(doi, qt * 32 + 16 * s, (2 * dh + e) * 32, lane);
            tq[e] = frag_tp2(qi, qt * 32 + 16 * s, (2 * dh + e) * 32, lane);
          }
          lgkm0();
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            dv[2 * dh + e] = mfma32(pf, tdo[e], dv[2 * dh + e]);
            dk[2 * dh + e] = mfma32(sf, tq[e], dk[2 * dh + e]);
          }
        }
      }
    }
    // stage dK (scaled by 1/sqrt(D)) in the Q image and dV in the dO image, 16-B row stores
    barrier();
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = w * 32 + acc_row(i, hf), col = dt * 32 + (lane & 31);
        wr_b16(qi + off2(row, col >> 3) + (col & 7) * 2, f2bf(dk[dt][i] * 0.08838834764831845f));
        wr_b16(doi + off2(row, col >> 3) + (col & 7) * 2, f2bf(dv[dt][i]));
      }
    barrier();
    bf16_t* kb = dqkv + (int64_t)b * L * ld + (int64_t)H * HD2 + (int64_t)hd * HD2;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int idx = tid + c * 256, row = idx >> 4, ch = idx & 15;
      const bf16x8 vk = rd128(qi + off2(row, ch));
      const bf16x8 vv = rd128(doi + off2(row, ch));
      lgkm0();
      *reinterpret_cast<bf16x8*>(kb + (int64_t)row * ld + ch * 8) = vk;
      *reinterpret_cast<bf16x8*>(kb + (int64_t)H * HD2 + (int64_t)row * ld + ch * 8) = vv;
    }
    if (colpart) {
      float* cp = colpart + (int64_t)item * 3 * HD2;
      item_colsum128(dk, 0.08838834764831845f, cred, cp + HD2, w, lane, tid);
      item_colsum128(dv, 1.f, cred, cp + 2 * HD2, w, lane, tid);
    }
  }
}

// db[q*H*64 + h*64 + d] += sum_b colpart[(b*H + h)*192 + q*64 + d] in two fixed-order passes (no
// fp32 atomics): grid (H*3, chunks of B) stores each chunk's sum over its first row in place,
// then colpart_final_kernel adds the chunk sums in order
__global__ void __launch_bounds__(256) colpart_reduce_kernel(float* __restrict__ colpart, int B, int H, int bchunk) {
  __shared__ float red[4][64];
  const int hq = blockIdx.x, h = hq / 3, q = hq - 3 * h;
  const int d = threadIdx.x & 63, r = threadIdx.x >> 6;
  const int b0 = blockIdx.y * bchunk, b1 = min(B, b0 + bchunk);
  float t = 0.f;
  for (int b = b0 + r; b < b1; b += 4) t += colpart[((int64_t)b * H + h) * 192 + q * 64 + d];
  red[r][d] = t;
  __syncthreads();
  if (r == 0 && b0 < b1)
    colpart[((int64_t)b0 * H + h) * 192 + q * 64 + d] = (red[0][d] + red[1][d]) + (red[2][d] + red[3][d]);
}

__global__ void __launch_bounds__(64) colpart_final_kernel(const float* __restrict__ colpart, float* __restrict__ db,
                                                           int B, int H, int bchunk) {
  const int hq = blockIdx.x, h = hq / 3, q = hq - 3 * h, d = threadIdx.x;
  float t = 0.f;
  for (int b0 = 0; b0 < B; b0 += bchunk) t += colpart[((int64_t)b0 * H + h) * 192 + q * 64 + d];
  db[q * H * HD + h * HD + d] += t;
}

static bool enabled() { return true; }

static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

}  // namespace a128

bool launch_attn128_fwd(const uint16_t* qkv, uint16_t* out, float* lse, int B, int Lq, int H,
                        float p, bool causal, uint32_t seed, uint32_t offset, hipStream_t s, bool head_major) {
  if (Lq != a128::L || causal || (!a128::enabled() && !head_major)) return false;
  const int items = B * H, slots = 2 * a128::num_cus();
  const int grid = items < slots ? items : slots;
  if (p > 0.f)
    hipLaunchKernelGGL(a128::attn128_fwd_kernel<true>, dim3(grid), dim3(256), 0, s, (const bf16_t*)qkv,
                       (bf16_t*)out, lse, B, H, p, seed, offset, head_major ? 1 : 0);
  else
    hipLaunchKernelGGL(a128::attn128_fwd_kernel<false>, dim3(grid), dim3(256), 0, s, (const bf16_t*)qkv,
                       (bf16_t*)out, lse, B, H, p, seed, offset, head_major ? 1 : 0);
  return true;
}

bool attn128_supports(int L, int D, bool causal) { return L == a128::L && D == a128::HD && !causal; }

// L = 128, head_dim 128, bidirectional, token-major (DiffuSeq-XL): the persistent backward
// (dQ + delta, then dK / dV), one workgroup per CU each
bool launch_attn128_bwd_d128(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout, const float* lse,
                             float* delta, uint16_t* dqkv, int B, int Lq, int H, float p, bool causal,
                             uint32_t seed, uint32_t offset, hipStream_t s, float* colpart) {
  if (Lq != a128::L || causal || !a128::enabled()) return false;
  const int items = B * H, slots = a128::num_cus();
  const int grid = items < slots ? items : slots;
  hipLaunchKernelGGL(a128::attn128_bwd_q_d128_kernel, dim3(grid), dim3(256), 0, s, (const bf16_t*)qkv,
                     (const bf16_t*)out, (const bf16_t*)dout, lse, delta, (bf16_t*)dqkv, B, H, p, seed, offset,
                     colpart);
  hipLaunchKernelGGL(a128::attn128_bwd_kv_d128_kernel, dim3(grid), dim3(256), 0, s, (const bf16_t*)qkv,
                     (const bf16_t*)dout, lse, (const float*)delta, (bf16_t*)dqkv, B, H, p, seed, offset,
                     colpart);
  return true;
}

// L = 128, head_dim 128, bidirectional, token-major (DiffuSeq-XL): persistent forward, one
// workgroup per CU; paired with the general backward kernels (same dropout / LSE conventions)
bool launch_attn128_fwd_d128(const uint16_t* qkv, uint16_t* out, float* lse, int B, int Lq, int H,
                             float p, bool causal, uint32_t seed, uint32_t offset, hipStream_t s) {
  if (Lq != a128::L || causal || !a128::enabled()) return false;
  const int items = B * H, slots = a128::num_cus();
  const int grid = items < slots ? items : slots;
  hipLaunchKernelGGL(a128::attn128_fwd_d128_kernel, dim3(grid), dim3(256), 0, s, (const bf16_t*)qkv,
                     (bf16_t*)out, lse, B, H, p, seed, offset);
  return true;
}

bool launch_attn128_bwd(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout,
                        const float* lse, uint16_t* dqkv, float* colpart, float* dbias, int B,
                        int Lq, int H, float p, bool causal, uint32_t seed, uint32_t offset,
                        hipStream_t s, bool head_major, bool db_accumulate, bool defer_reduce) {
  if (Lq != a128::L || causal || (!a128::enabled() && !head_major)) return false;
  const int items = B * H, slots = 2 * a128::num_cus();
  const int grid = items < slots ? items : slots;
  if (p > 0.f)
    hipLaunchKernelGGL(a128::attn128_bwd_kernel<true>, dim3(grid), dim3(256), 0, s, (const bf16_t*)qkv,
                       (const bf16_t*)out, (const bf16_t*)dout, lse, (bf16_t*)dqkv,
                       dbias ? colpart : nullptr, B, H, p, seed, offset, head_major ? 1 : 0);
  else
    hipLaunchKernelGGL(a128::attn128_bwd_kernel<false>, dim3(grid), dim3(256), 0, s, (const bf16_t*)qkv,
                       (const bf16_t*)out, (const bf16_t*)dout, lse, (bf16_t*)dqkv,
                       dbias ? colpart : nullptr, B, H, p, seed, offset, head_major ? 1 : 0);
  if (dbias && !defer_reduce) {  // deferred: the caller reduces several calls' partials at once
    const int bchunk = 64, nch = (B + bchunk - 1) / bchunk;
    if (!db_accumulate) (void)hipMemsetAsync(dbias, 0, sizeof(float) * 3 * H * a128::HD, s);
    hipLaunchKernelGGL(a128::colpart_reduce_kernel, dim3(3 * H, nch), dim3(256), 0, s, colpart, B, H, bchunk);
    hipLaunchKernelGGL(a128::colpart_final_kernel, dim3(3 * H), dim3(64), 0, s, (const float*)colpart, dbias, B, H,
                       bchunk);
  }
  return true;
}

DPA_RNG_BASE_EXPORT(attention128)

}  // namespace dpa
