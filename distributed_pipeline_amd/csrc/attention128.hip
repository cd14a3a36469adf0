// Attention for sequence length 128, head_dim 64, bidirectional (the DiffuSeq /
// BERT shape, SURVEY K-M8): persistent kernels that stream (batch, head) items
// through LDS with global_load_lds prefetch, so the HBM traffic of item i+1
// overlaps the matrix-core work of item i.
//
// Both kernels: grid = #CUs, 256 threads (4 waves), items (b, h) strided over
// the grid, two LDS buffers (ping-pong).  All LDS accesses are inline asm so
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
  d.seedmix = lowbias32(seed ^ lowbias32(offset * 0xC2B2AE3Du ^ (bh * 0x27D4EB2Fu)));
  return d;
}
__device__ __forceinline__ bool keep_bit(const DropCfg& d, int q, int key) {
  const uint32_t h = lowbias32(d.seedmix ^ ((uint32_t)q * 0x9E3779B1u) ^ ((uint32_t)(key >> 1) * 0x85EBCA77u));
  const uint32_t r = (key & 1) ? (h >> 16) : (h & 0xffffu);
  return r >= d.thr16;
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
__device__ __forceinline__ void lgkm0() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
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
    const bf16_t* g = src + (int64_t)row * ld + ((phys ^ ((row >> 1) & 7)) << 3);
    __builtin_amdgcn_global_load_lds((glob_void*)g, (lds_void*)(img + pc * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ float bflo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bfhi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// ============================================================================
// forward
// ============================================================================
__global__ void __launch_bounds__(256) attn128_fwd_kernel(const bf16_t* __restrict__ qkv,
                                                         bf16_t* __restrict__ out,
                                                         float* __restrict__ lse, int B, int H,
                                                         float p, uint32_t seed, uint32_t offset) {
  // buffer b at b * 48K: Q, K, V images
  __shared__ __attribute__((aligned(1024))) char smem[2 * 3 * IMG];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hf = lane >> 5;
  const int nitems = B * H;
  const int64_t ld = 3LL * H * HD, ldo = (int64_t)H * HD;
  const uint32_t sb = lds_u32(smem);

  auto issue = [&](int item, int buf) {
    const int b = item / H, hd = item - b * H;
    const bf16_t* qb = qkv + (int64_t)b * L * ld + (int64_t)hd * HD;
    char* base = smem + buf * 3 * IMG;
    dma_img(base, qb, ld, w, lane);
    dma_img(base + IMG, qb + (int64_t)H * HD, ld, w, lane);
    dma_img(base + 2 * IMG, qb + 2LL * H * HD, ld, w, lane);
  };

  int item = blockIdx.x;
  if (item < nitems) issue(item, 0);
  for (int k = 0; item < nitems; ++k, item += gridDim.x) {
    const int cur = k & 1;
    // this item's DMA landed; the previous item's 5 stores (lse + 4 O rows) may
    // still be in flight (issued last, retired in order)
    if (k == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    barrier();
    if (item + (int)gridDim.x < nitems) issue(item + gridDim.x, cur ^ 1);
    const uint32_t qi = sb + cur * 3 * IMG, ki = qi + IMG, vi = qi + 2 * IMG;
    const int b = item / H, hd = item - b * H;
    const DropCfg dc = make_drop(p, seed, offset, (uint32_t)item);
    const int q = w * 32 + (lane & 31);

    // S^T (keys in registers, query on the lane)
    bf16x8 qf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = frag_r(qi, w * 32, s, lane);
    f32x16 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      bf16x8 kf[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) kf[s] = frag_r(ki, t * 32, s, lane);
      lgkm0();
      acc[t] = zero16();
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[t] = mfma32(kf[s], qf[s], acc[t]);
    }
    float m = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        acc[t][i] *= ATT_C;
        m = fmaxf(m, acc[t][i]);
      }
    m = fmaxf(m, __shfl_xor(m, 32, 64));
    float l = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float e = exp2f(acc[t][i] - m);
        acc[t][i] = e;
        l += e;
      }
    l += __shfl_xor(l, 32, 64);
    const float inv_l = 1.f / l;
    if (hf == 0) lse[(int64_t)item * L + q] = (m + log2f(l)) * LN2f;
    f32x16 o[2];
    o[0] = zero16();
    o[1] = zero16();
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float pr = acc[t][i] * inv_l;
        if (dc.on) pr = keep_bit(dc, q, t * 32 + acc_row(i, hf)) ? pr * dc.scale : 0.f;
        acc[t][i] = pr;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 af = acc_to_frag(acc[t], s);
        bf16x8 vf[2];
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) vf[dt] = frag_tp(vi, t * 32 + 16 * s, dt * 32, lane);
        lgkm0();
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) o[dt] = mfma32(af, vf[dt], o[dt]);
      }
    }
    // stage O (rows = queries) in the Q image (dead: every wave passed its reads)
    barrier();
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = w * 32 + acc_row(i, hf), col = dt * 32 + (lane & 31);
        wr_b16(qi + off_r(row, col >> 3) + (col & 7) * 2, f2bf(o[dt][i]));
      }
    barrier();
    bf16_t* ob = out + (int64_t)b * L * ldo + (int64_t)hd * HD;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int idx = tid + c * 256, row = idx >> 3, ch = idx & 7;
      const bf16x8 v = rd128(qi + off_r(row, ch));
      lgkm0();
      *reinterpret_cast<bf16x8*>(ob + (int64_t)row * ldo + ch * 8) = v;
    }
  }
}

// ============================================================================
// backward
// ============================================================================
// LDS: buffers b = 0, 1 at b * 64K: Q, K, V, dO images; at 128K: lse2[128], delta[128]
constexpr int BWD_BUF = 4 * IMG;
constexpr int BWD_STATS = 2 * BWD_BUF;

__global__ void __launch_bounds__(256) attn128_bwd_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ out, const bf16_t* __restrict__ dout,
    const float* __restrict__ lse, bf16_t* __restrict__ dqkv, int B, int H, float p, uint32_t seed,
    uint32_t offset) {
  __shared__ __attribute__((aligned(1024))) char smem[BWD_STATS + 2 * L * 4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hf = lane >> 5;
  const int nitems = B * H;
  const int64_t ld = 3LL * H * HD, ldo = (int64_t)H * HD;
  const uint32_t sb = lds_u32(smem);
  const uint32_t s_lse = sb + BWD_STATS, s_del = s_lse + L * 4;

  // register prefetch of O (delta) and LSE: thread -> row tid >> 1, half tid & 1
  uint4 opf[4];
  float lpf = 0.f;
  auto prefetch = [&](int item) {
    const int b = item / H, hd = item - b * H;
    const bf16_t* orow = out + ((int64_t)b * L + (tid >> 1)) * ldo + (int64_t)hd * HD + (tid & 1) * 32;
#pragma unroll
    for (int c = 0; c < 4; ++c) opf[c] = *reinterpret_cast<const uint4*>(orow + c * 8);
    if (tid < L) lpf = lse[(int64_t)item * L + tid];
  };
  auto issue = [&](int item, int buf) {
    const int b = item / H, hd = item - b * H;
    const bf16_t* qb = qkv + (int64_t)b * L * ld + (int64_t)hd * HD;
    char* base = smem + buf * BWD_BUF;
    dma_img(base, qb, ld, w, lane);
    dma_img(base + IMG, qb + (int64_t)H * HD, ld, w, lane);
    dma_img(base + 2 * IMG, qb + 2LL * H * HD, ld, w, lane);
    dma_img(base + 3 * IMG, dout + (int64_t)b * L * ldo + (int64_t)hd * HD, ldo, w, lane);
  };

  int item = blockIdx.x;
  if (item < nitems) {
    issue(item, 0);
    prefetch(item);
  }
  for (int k = 0; item < nitems; ++k, item += gridDim.x) {
    const int cur = k & 1;
    const uint32_t qi = sb + cur * BWD_BUF, ki = qi + IMG, vi = qi + 2 * IMG, di = qi + 3 * IMG;
    // this item's DMA + O/LSE prefetch landed; the previous item's 12 output
    // stores (issued last, retired in order) may still be in flight
    if (k == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    barrier();
    // delta = rowsum(dO * O) and lse (log2 units) -> LDS
    {
      const int row = tid >> 1, half = tid & 1;
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const bf16x8 dv = rd128(di + off_r(row, half * 4 + c));
        lgkm0();
        const uint32_t ow[4] = {opf[c].x, opf[c].y, opf[c].z, opf[c].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t dw = (uint32_t)(uint16_t)dv[2 * e] | ((uint32_t)(uint16_t)dv[2 * e + 1] << 16);
          s += bflo(dw) * bflo(ow[e]) + bfhi(dw) * bfhi(ow[e]);
        }
      }
      s += __shfl_xor(s, 1, 64);
      if (half == 0) wr_b32(s_del + row * 4, __float_as_uint(s));
      if (tid < L) wr_b32(s_lse + tid * 4, __float_as_uint(lpf * LOG2Ef));
    }
    const int nxt = item + gridDim.x;
    if (nxt < nitems) {
      issue(nxt, cur ^ 1);
      prefetch(nxt);
    }
    barrier();

    const int b = item / H, hd = item - b * H;
    const DropCfg dc = make_drop(p, seed, offset, (uint32_t)item);
    const int kb = w * 32, key = kb + (lane & 31);
    bf16x8 kf[4], vf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kf[s] = frag_r(ki, kb, s, lane);
      vf[s] = frag_r(vi, kb, s, lane);
    }
    lgkm0();
    f32x16 dk[2], dv[2];
    uint4 dsb[4][2];  // dS as bf16 (the exact A-operand packing), 8 registers per tile
    dk[0] = zero16(); dk[1] = zero16(); dv[0] = zero16(); dv[1] = zero16();
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x16 sacc = zero16(), dpacc = zero16();
      {
        bf16x8 qf[4], df[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          qf[s] = frag_r(qi, t * 32, s, lane);
          df[s] = frag_r(di, t * 32, s, lane);
        }
        lgkm0();
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          sacc = mfma32(qf[s], kf[s], sacc);
          dpacc = mfma32(df[s], vf[s], dpacc);
        }
      }
      // lse2 / delta of this lane's query rows 32t + 8g + 4h + r (r = 0..3)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 lv = rd_f4(s_lse + (t * 32 + 8 * g + 4 * hf) * 4);
        const f32x4 dl = rd_f4(s_del + (t * 32 + 8 * g + 4 * hf) * 4);
        lgkm0();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = 4 * g + r;
          const int qq = t * 32 + 8 * g + 4 * hf + r;
          const float pr = exp2f(sacc[i] * ATT_C - lv[r]);
          float pd = pr, dpd = dpacc[i];
          if (dc.on) {
            const bool kp = keep_bit(dc, qq, key);
            pd = kp ? pr * dc.scale : 0.f;
            dpd = kp ? dpd * dc.scale : 0.f;
          }
          sacc[i] = pd;
          dpacc[i] = pr * (dpd - dl[r]);
        }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pf = acc_to_frag(sacc, s);
        const bf16x8 sf = acc_to_frag(dpacc, s);
        dsb[t][s] = __builtin_bit_cast(uint4, sf);
        bf16x8 tdo[2], tq[2];
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          tdo[dt] = frag_tp(di, t * 32 + 16 * s, dt * 32, lane);
          tq[dt] = frag_tp(qi, t * 32 + 16 * s, dt * 32, lane);
        }
        lgkm0();
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) {
          dv[dt] = mfma32(pf, tdo[dt], dv[dt]);
          dk[dt] = mfma32(sf, tq[dt], dk[dt]);
        }
      }
    }
    // dS^T -> LDS (over V / dO of this buffer, dead once every wave is here)
    barrier();
    const uint32_t si = vi;  // [128 keys][128 queries], 256-B rows (32 KiB: V + dO)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        // group g = registers 4g..4g+3 = elements 4(g&1).. of fragment g>>1
        const int q0 = t * 32 + 8 * g + 4 * hf;
        const uint4 v = dsb[t][g >> 1];
        const uint32_t lo = (g & 1) ? v.z : v.x, hi = (g & 1) ? v.w : v.y;
        wr_b64(si + off_s(key, q0 >> 3) + (q0 & 7) * 2, lo, hi);
      }
    barrier();
    // dQ for queries 32w..32w+31: sum over keys of dS[q][key] K[key][d]
    f32x16 dq[2];
    dq[0] = zero16();
    dq[1] = zero16();
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const bf16x8 af = frag_tn_s(si, ks * 16, w * 32, lane);
      bf16x8 bk[2];
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) bk[dt] = frag_tn_r(ki, ks * 16, dt * 32, lane);
      lgkm0();
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) dq[dt] = mfma32(af, bk[dt], dq[dt]);
    }
    // stage dQ (rows = queries of wave w), dK, dV (rows = keys of wave w) in Q/K/V images
    barrier();
#pragma unroll
    for (int dt = 0; dt < 2; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = w * 32 + acc_row(i, hf), col = dt * 32 + (lane & 31);
        const uint32_t o = off_r(row, col >> 3) + (col & 7) * 2;
        wr_b16(qi + o, f2bf(dq[dt][i] * 0.125f));
        wr_b16(ki + o, f2bf(dk[dt][i] * 0.125f));
        wr_b16(vi + o, f2bf(dv[dt][i]));
      }
    barrier();
    bf16_t* gb = dqkv + (int64_t)b * L * ld + (int64_t)hd * HD;
#pragma unroll
    for (int c = 0; c < 12; ++c) {
      const int idx = tid + c * 256;          // 3 tensors x 128 rows x 8 chunks
      const int x = idx >> 10, row = (idx >> 3) & 127, ch = idx & 7;
      const bf16x8 v = rd128(qi + x * IMG + off_r(row, ch));
      lgkm0();
      *reinterpret_cast<bf16x8*>(gb + (int64_t)row * ld + (int64_t)x * H * HD + ch * 8) = v;
    }
  }
}

static bool enabled() {
  static int on = -1;
  if (on < 0) {
    const char* e = std::getenv("DPA_ATTN128");
    on = (e && e[0] == '0') ? 0 : 1;
  }
  return on != 0;
}

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
                        float p, bool causal, uint32_t seed, uint32_t offset, hipStream_t s) {
  if (Lq != a128::L || causal || !a128::enabled()) return false;
  const int items = B * H;
  const int grid = items < a128::num_cus() ? items : a128::num_cus();
  hipLaunchKernelGGL(a128::attn128_fwd_kernel, dim3(grid), dim3(256), 0, s, (const bf16_t*)qkv,
                     (bf16_t*)out, lse, B, H, p, seed, offset);
  return true;
}

bool launch_attn128_bwd(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout,
                        const float* lse, uint16_t* dqkv, int B, int Lq, int H, float p, bool causal,
                        uint32_t seed, uint32_t offset, hipStream_t s) {
  if (Lq != a128::L || causal || !a128::enabled()) return false;
  const int items = B * H;
  const int grid = items < a128::num_cus() ? items : a128::num_cus();
  hipLaunchKernelGGL(a128::attn128_bwd_kernel, dim3(grid), dim3(256), 0, s, (const bf16_t*)qkv,
                     (const bf16_t*)out, (const bf16_t*)dout, lse, (bf16_t*)dqkv, B, H, p, seed,
                     offset);
  return true;
}

}  // namespace dpa
