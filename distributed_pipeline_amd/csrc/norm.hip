// Fused residual / embedding-sum + LayerNorm (SURVEY K-M6/K-M9/K-M10):
//
//   s   = y + pos[row % L] + temb[row / L]   (pos, temb optional row-broadcast terms)
//   h   = dropout_p(s) + residual            (pre-dropout; residual optional)
//   out = LayerNorm(h) * gamma + beta        -> bf16; saves h (bf16), mean, rstd
//   post mode: h = s + residual, out = dropout_p(LayerNorm(h) * gamma + beta)
//
// Uses: BERT post-LN sublayers (y = branch output, residual = x); the DiffuSeq input
// block (y = up-proj, pos, temb = time embedding, post dropout: reference model's
// Dropout(LayerNorm(...))); GPT-2 pre-LN residual streams (h is the new residual
// stream, out the next sublayer's LN input; the backward adds h's own incoming
// gradient dh_in).  Backward (dy, dresidual, dgamma, dbeta) in one pass per row.  One
// wave64 owns a row: D/64 elements per lane (D = 768 -> 12) in groups of 8 (16-byte
// vectors) or 4 (8-byte) interleaved over the lanes (RowMap), so every load/store
// instruction covers 512 B - 1 KiB of the row contiguously, and both reductions
// are a single wave-wide shuffle tree (no LDS, no barriers).
// The dropout mask is never stored: it is regenerated from the counter-based
// Philox stream (seed, offset, row, column) in the backward.
//
// dgamma/dbeta: each block accumulates its rows' contributions in registers,
// reduces its 4 waves through LDS and adds one fp32 atomic per column.
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "launchers.h"

namespace dpa {

// Element -> lane map of a D = 64 * VEC row: lane `ln` holds VEC / CH groups of CH consecutive
// elements, group g at column g * 64 * CH + ln * CH, so one load instruction of a wave covers
// 64 * CH contiguous elements (1 KiB for CH = 8) instead of 64 strided VEC-element runs.
template <int VEC>
struct RowMap {
  static constexpr int CH = VEC % 8 == 0 ? 8 : VEC % 4 == 0 ? 4 : VEC;
  static constexpr int NG = VEC / CH;
  __device__ __forceinline__ static int col(int ln, int i) { return (i / CH) * 64 * CH + ln * CH + i % CH; }
};

template <int VEC>
struct RowIO {
  using M = RowMap<VEC>;
  // load this lane's VEC elements of a row (16-B vectors for CH = 8, 8-B for CH = 4)
  __device__ __forceinline__ static void load(const bf16_t* row, int ln, float* v) {
#pragma unroll
    for (int g = 0; g < M::NG; ++g) {
      const bf16_t* p = row + g * 64 * M::CH + ln * M::CH;
      float* o = v + g * M::CH;
      if constexpr (M::CH == 8) {
        const uint4 raw = *reinterpret_cast<const uint4*>(p);
        const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          o[2 * k] = __uint_as_float(w[k] << 16);
          o[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
        }
      } else if constexpr (M::CH == 4) {
        const uint2 raw = *reinterpret_cast<const uint2*>(p);
        o[0] = __uint_as_float(raw.x << 16);
        o[1] = __uint_as_float(raw.x & 0xffff0000u);
        o[2] = __uint_as_float(raw.y << 16);
        o[3] = __uint_as_float(raw.y & 0xffff0000u);
      } else {
#pragma unroll
        for (int c = 0; c < M::CH; ++c) o[c] = bf2f(p[c]);
      }
    }
  }
  __device__ __forceinline__ static void store(bf16_t* row, int ln, const float* v) {
#pragma unroll
    for (int g = 0; g < M::NG; ++g) {
      bf16_t* p = row + g * 64 * M::CH + ln * M::CH;
      const float* o = v + g * M::CH;
      if constexpr (M::CH == 8) {
        *reinterpret_cast<uint4*>(p) = make_uint4(pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3]),
                                                  pack_bf2(o[4], o[5]), pack_bf2(o[6], o[7]));
      } else if constexpr (M::CH == 4) {
        *reinterpret_cast<uint2*>(p) = make_uint2(pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3]));
      } else {
#pragma unroll
        for (int c = 0; c < M::CH; ++c) p[c] = f2bf(o[c]);
      }
    }
  }
};

// keep-mask bits for this lane's VEC elements of `row`: element (row, col) keeps iff word
// col & 3 of the Philox block (row, col >> 2) is >= p * 2^32 - one call per 4 aligned columns
// (a function of (row, col) only, whatever the element -> lane map).
template <int VEC>
__device__ __forceinline__ void dropout_keep(uint32_t seed, uint32_t offset, int64_t row, int ln,
                                             float p, bool* keep) {
  using M = RowMap<VEC>;
  const uint32_t thr = (uint32_t)(p * 4294967296.0);
  if constexpr (M::CH % 4 == 0) {
#pragma unroll
    for (int c = 0; c < VEC / 4; ++c) {
      const int col = M::col(ln, 4 * c);
      uint32_t r[4];
      philox4(seed, 0x5bd1e995u, (uint32_t)row, (uint32_t)(row >> 32) ^ (uint32_t)(col >> 2), offset + rng_base(),
              0xdeadbeefu, r);
#pragma unroll
      for (int k = 0; k < 4; ++k) keep[4 * c + k] = r[k] >= thr;
    }
  } else {
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      const int col = M::col(ln, i);
      uint32_t r[4];
      philox4(seed, 0x5bd1e995u, (uint32_t)row, (uint32_t)(row >> 32) ^ (uint32_t)(col >> 2), offset + rng_base(),
              0xdeadbeefu, r);
      keep[i] = r[col & 3] >= thr;
    }
  }
}

// keep bits of the pair-hash mode (common.h pair_hash): the post-LN sublayers whose residual +
// dropout run in the producing GEMM's epilogue (gemm256.hip EPI 7) regenerate them here.
template <int VEC>
__device__ __forceinline__ void dropout_keep_pair(uint32_t sm, uint32_t thr16, int64_t row, int ln, bool* keep) {
  using M = RowMap<VEC>;
  if constexpr (M::CH % 2 == 0) {
#pragma unroll
    for (int i = 0; i < VEC; i += 2) {  // elements i, i + 1 are columns 2j, 2j + 1 of one pair
      const uint32_t h = pair_hash(sm, (uint32_t)row, (uint32_t)M::col(ln, i));
      keep[i] = (h & 0xffffu) >= thr16;
      keep[i + 1] = (h >> 16) >= thr16;
    }
  } else {
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      const uint32_t col = (uint32_t)M::col(ln, i);
      keep[i] = pair_keep(pair_hash(sm, (uint32_t)row, col), col, thr16);
    }
  }
}

// 1 / gamma for the output-based backward (xhat = (o - b) / gamma, the "memory-efficient"
// LayerNorm backward; used only when every |gamma| >= LN_XO_GMIN, so never 0 there).
__device__ __forceinline__ float inv_gamma(float g) { return g != 0.f ? 1.f / g : 0.f; }
// Guard of the output-based backward.  o = xhat * g + b is rounded to bf16 (relative error
// e of |o|), so xhat = (o - b) / g carries an absolute error e * (|xhat| + |b| / |g|), against
// e * (|xhat| + |mean| * rstd) for the h copy: the reconstruction is as exact as the h copy
// only while |b| / |g| stays O(1) and g is not tiny.  A LayerNorm with any column where
// |g| < LN_XO_GMIN or |b| > LN_XO_BRATIO * |g| keeps the exact h-copy path: its forward writes
// the h copy (hguard) and its backward reads it.  Both kernels evaluate the same predicate on
// the same gamma and beta (the optimizer runs after the backward), so no flag travels between
// them and nothing syncs with the host.
constexpr float LN_XO_GMIN = 0.125f;
constexpr float LN_XO_BRATIO = 1.0f;
__device__ __forceinline__ bool xo_unsafe(float g, float b) {
  return fabsf(g) < LN_XO_GMIN || fabsf(b) > LN_XO_BRATIO * fabsf(g);
}

template <int VEC>
__global__ void __launch_bounds__(256) add_ln_fwd_kernel(
    const bf16_t* __restrict__ y, const bf16_t* __restrict__ res, const bf16_t* __restrict__ gamma,
    const bf16_t* __restrict__ beta, bf16_t* __restrict__ out, bf16_t* __restrict__ hsave,
    float* __restrict__ mean_out, float* __restrict__ rstd_out, int64_t R, float p, float eps,
    uint32_t seed, uint32_t offset, const bf16_t* __restrict__ pos, const bf16_t* __restrict__ temb,
    int L, int post, int hguard) {
  constexpr int D = VEC * 64;
  const int lane = threadIdx.x & 63;
  // grid-stride over rows (4 per block per pass): gamma / beta are loaded once per wave instead
  // of once per row, and a capped grid replaces R / 4 short-lived blocks
  float g[VEC], b[VEC];
  RowIO<VEC>::load(gamma, lane, g);
  RowIO<VEC>::load(beta, lane, b);
  bool write_h0 = hsave != nullptr;
  if (write_h0 && hguard) {
    // output-based backward unless some |gamma| is small (the row holds all of gamma)
    bool small = false;
#pragma unroll
    for (int i = 0; i < VEC; ++i) small |= xo_unsafe(g[i], b[i]);
    write_h0 = __builtin_amdgcn_ballot_w64(small) != 0;
  }
  const bool write_h = write_h0;
  for (int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); row < R;
       row += (int64_t)gridDim.x * (blockDim.x >> 6)) {
  float h[VEC];
  RowIO<VEC>::load(y + row * D, lane, h);
  if (pos) {
    float t[VEC];
    RowIO<VEC>::load(pos + (row % L) * D, lane, t);
#pragma unroll
    for (int i = 0; i < VEC; ++i) h[i] += t[i];
  }
  if (temb) {
    float t[VEC];
    RowIO<VEC>::load(temb + (row / L) * D, lane, t);
#pragma unroll
    for (int i = 0; i < VEC; ++i) h[i] += t[i];
  }
  if (p > 0.f && !post) {
    bool keep[VEC];
    dropout_keep<VEC>(seed, offset, row, lane, p, keep);
    const float sc = 1.f / (1.f - p);
#pragma unroll
    for (int i = 0; i < VEC; ++i) h[i] = keep[i] ? h[i] * sc : 0.f;
  }
  if (res) {
    float r[VEC];
    RowIO<VEC>::load(res + row * D, lane, r);
#pragma unroll
    for (int i = 0; i < VEC; ++i) h[i] += r[i];
  }
  // round h to bf16 first so the backward (which reloads the bf16 copy) is consistent
#pragma unroll
  for (int i = 0; i < VEC; ++i) h[i] = bf2f(f2bf(h[i]));
  float o[VEC];
  if (write_h) RowIO<VEC>::store(hsave + row * D, lane, h);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VEC; ++i) s += h[i];
  const float mean = wave_sum(s) * (1.f / D);
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < VEC; ++i) { const float d = h[i] - mean; v += d * d; }
  const float rstd = rsqrtf(wave_sum(v) * (1.f / D) + eps);
#pragma unroll
  for (int i = 0; i < VEC; ++i) o[i] = (h[i] - mean) * rstd * g[i] + b[i];
  if (p > 0.f && post) {
    bool keep[VEC];
    dropout_keep<VEC>(seed, offset, row, lane, p, keep);
    const float sc = 1.f / (1.f - p);
#pragma unroll
    for (int i = 0; i < VEC; ++i) o[i] = keep[i] ? o[i] * sc : 0.f;
  }
  RowIO<VEC>::store(out + row * D, lane, o);
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
  }
}

// grid-stride over rows; block = 4 waves; partial dgamma/dbeta per block.
// POST at compile time (the two dropout placements share no loop body) and <= 128 VGPRs
// (4 waves per SIMD: the LDS reduction buffer allows 4 blocks per CU); D > 768 keeps
// 6 x VEC live accumulator/row floats: 4 waves per SIMD up to D = 768, 2-3 up to D = 1024.
// D >= 1536 takes add_ln_bwd_rowblk_kernel (one row per block) instead.
// HK: the dy dropout bits come from the pair hash (pre-dropout placement only)
// NW waves per block (4, or 8 for the small-R two-stage shapes: the same waves per CU with half the
// blocks, so half the column-sum partials to store and re-read)
template <int VEC, bool POST, bool XO, bool HK = false, int NW = 4>
__global__ void __launch_bounds__(NW * 64, (VEC <= 12 ? 4 : VEC <= 16 ? 2 : 1) * 4 / NW) add_ln_bwd_kernel(
    const bf16_t* __restrict__ dout, const bf16_t* __restrict__ hsave,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const bf16_t* __restrict__ gamma, bf16_t* __restrict__ dres, bf16_t* __restrict__ dy,
    float* __restrict__ dyb, float* __restrict__ part_dg, float* __restrict__ part_db, int64_t R,
    float p, uint32_t seed, uint32_t offset, const bf16_t* __restrict__ dh_in, float* __restrict__ part,
    bool part_acc, const bf16_t* __restrict__ beta, const bf16_t* __restrict__ hcopy) {
  constexpr int D = VEC * 64;
  __shared__ float red[NW][D];  // reused for dgamma, dbeta, dyb in turn
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float g[VEC], adg[VEC], adb[VEC], ady[VEC];
  RowIO<VEC>::load(gamma, lane, g);
  // XO: `hsave` is the LN output o = xhat * g + b (kept alive anyway as the next sublayer's
  // input), so xhat = (o - b) / g and the forward writes no h copy.  beta and 1 / gamma sit
  // in LDS (read per row: in registers they would spill the 128-VGPR budget at D = 768)
  __shared__ float cst[XO ? 2 : 1][XO ? D : 1];
  bool xo = false;  // wave-uniform: every wave holds all of gamma
  if constexpr (XO) {
    float bb[VEC];
    RowIO<VEC>::load(beta, lane, bb);
    bool small = false;
#pragma unroll
    for (int i = 0; i < VEC; ++i) small |= xo_unsafe(g[i], bb[i]);
    xo = __builtin_amdgcn_ballot_w64(small) == 0;
    for (int c = threadIdx.x; c < D; c += blockDim.x) {
      cst[0][c] = bf2f(beta[c]);
      cst[1][c] = inv_gamma(bf2f(gamma[c]));
    }
    __syncthreads();
  }
  const bf16_t* const hsrc = XO && !xo ? hcopy : hsave;
#pragma unroll
  for (int i = 0; i < VEC; ++i) { adg[i] = 0.f; adb[i] = 0.f; ady[i] = 0.f; }
  const float sc = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const uint32_t hsm = HK ? pair_seedmix(seed, offset + rng_base()) : 0u, hthr = pair_thr16(p);
  for (int64_t row = (int64_t)blockIdx.x * NW + w; row < R; row += (int64_t)gridDim.x * NW) {
    float h[VEC], d[VEC];
    RowIO<VEC>::load(hsrc + row * D, lane, h);
    RowIO<VEC>::load(dout + row * D, lane, d);
    // pair-hash mode: every load of the row issued before any math, the keep bits computed
    // under their latency (left to itself the scheduler interleaved the cheap hash with the
    // loads and waited on each: 0.40 vs 0.31 ms per call at 262144 x 768)
    uint32_t kbits = 0;
    float mean_h = 0.f, rstd_h = 0.f;
    if constexpr (HK) {
      mean_h = mean_in[row];
      rstd_h = rstd_in[row];
      __builtin_amdgcn_sched_barrier(0);
      if (p > 0.f) {
        bool keep[VEC];
        dropout_keep_pair<VEC>(hsm, hthr, row, lane, keep);
#pragma unroll
        for (int i = 0; i < VEC; ++i) kbits |= keep[i] ? (1u << i) : 0u;
      }
    }
    if (POST && p > 0.f) {
      bool keep[VEC];
      dropout_keep<VEC>(seed, offset, row, lane, p, keep);
#pragma unroll
      for (int i = 0; i < VEC; ++i) d[i] = keep[i] ? d[i] * sc : 0.f;
    }
    const float mean = HK ? mean_h : (XO && xo ? 0.f : mean_in[row]), rstd = HK ? rstd_h : rstd_in[row];
    // opaque zero per row: keeps the loop-invariant LDS reads of cst inside the row loop
    int zo = 0;
    if constexpr (XO) asm volatile("v_mov_b32 %0, 0" : "=v"(zo));
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      float xh;
      if (XO && xo) {
        const int c = RowMap<VEC>::col(lane, i) + zo;
        xh = (h[i] - cst[0][c]) * cst[1][c];
      } else {
        xh = (h[i] - mean) * rstd;
      }
      adg[i] += d[i] * xh;
      adb[i] += d[i];
      const float gx = d[i] * g[i];
      h[i] = xh;
      d[i] = gx;
      s1 += gx;
      s2 += gx * xh;
    }
    s1 = wave_sum(s1) * (1.f / D);
    s2 = wave_sum(s2) * (1.f / D);
#pragma unroll
    for (int i = 0; i < VEC; ++i) d[i] = rstd * (d[i] - s1 - h[i] * s2);
    if (dh_in) {
      float e[VEC];
      RowIO<VEC>::load(dh_in + row * D, lane, e);
#pragma unroll
      for (int i = 0; i < VEC; ++i) d[i] += e[i];
    }
    if (dres) RowIO<VEC>::store(dres + row * D, lane, d);
    if (dy) {
      if (!POST && p > 0.f) {
        if constexpr (HK) {
#pragma unroll
          for (int i = 0; i < VEC; ++i) d[i] = ((kbits >> i) & 1u) ? d[i] * sc : 0.f;
        } else {
          bool keep[VEC];
          dropout_keep<VEC>(seed, offset, row, lane, p, keep);
#pragma unroll
          for (int i = 0; i < VEC; ++i) d[i] = keep[i] ? d[i] * sc : 0.f;
        }
      }
      RowIO<VEC>::store(dy + row * D, lane, d);
      if (dyb) {
        // bias gradient of the layer that produced y: column sums of the bf16 dy
#pragma unroll
        for (int i = 0; i < VEC; ++i) ady[i] += bf2f(f2bf(d[i]));
      }
    }
  }
  // per block and accumulator: one fp32 atomic per column (dg/db/dyb zeroed by the
  // launcher or accumulated onto the parameter grads), or - part != nullptr - a plain
  // store of the block's column sums into part[block][3][D] (ln_colreduce_kernel adds them)
  float* const dst[3] = {part_dg, part_db, dyb};
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    if (a == 2 && !dyb) break;
    if (a) __syncthreads();  // previous accumulator's columns have been read
#pragma unroll
    for (int i = 0; i < VEC; ++i) red[w][RowMap<VEC>::col(lane, i)] = a == 0 ? adg[i] : a == 1 ? adb[i] : ady[i];
    __syncthreads();
    if (part) {
      float* pr = part + ((int64_t)blockIdx.x * 3 + a) * D;
      for (int c = threadIdx.x; c < D; c += blockDim.x) {
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < NW; ++k) v += red[k][c];
        pr[c] = part_acc ? pr[c] + v : v;  // part_acc: partials summed over micro-batches
      }
    } else {
      for (int c = threadIdx.x; c < D; c += blockDim.x) {
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < NW; ++k) v += red[k][c];
        atomicAdd(dst[a] + c, v);
      }
    }
  }
}

// Wide rows (D = 1536, 2048): one row per 256-thread block, VT = D / 256 elements per thread in
// groups of CH interleaved over the threads (a load instruction covers 256 CH contiguous
// elements).  A thread owns the same VT columns for every row, so its column accumulators are
// 3 VT registers (24 at D = 2048, vs 96 for the wave-per-row kernel, which held D = 2048 at 256
// VGPRs - one wave per SIMD), and the block's column sums need no cross-wave reduction.  The two
// row sums cross the 4 waves through LDS (double-buffered by row parity: one barrier per row).
// Column sums always two-stage: part[block][3][D].
template <int D, bool POST, bool XO, bool HK = false>
__global__ void __launch_bounds__(256) add_ln_bwd_rowblk_kernel(
    const bf16_t* __restrict__ dout, const bf16_t* __restrict__ hsave,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const bf16_t* __restrict__ gamma, bf16_t* __restrict__ dres, bf16_t* __restrict__ dy,
    bool want_dyb, int64_t R, float p, uint32_t seed, uint32_t offset, const bf16_t* __restrict__ dh_in,
    float* __restrict__ part, bool part_acc, const bf16_t* __restrict__ beta,
    const bf16_t* __restrict__ hcopy) {
  constexpr int VT = D / 256;
  constexpr int CH = VT % 8 == 0 ? 8 : VT % 4 == 0 ? 4 : VT % 2 == 0 ? 2 : 1;
  constexpr int NG = VT / CH;
  static_assert(VT * 256 == D && CH % 2 == 0, "rowblk: D = 256 * even");
  __shared__ float rsum[2][4][2];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  auto col = [&](int i) { return (i / CH) * 256 * CH + t * CH + i % CH; };
  auto ld = [&](const bf16_t* row, float* v) {
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
      const bf16_t* q = row + gi * 256 * CH + t * CH;
      uint32_t wv[CH / 2];
      if constexpr (CH == 8) {
        const uint4 r = *reinterpret_cast<const uint4*>(q);
        wv[0] = r.x; wv[1] = r.y; wv[2] = r.z; wv[3] = r.w;
      } else if constexpr (CH == 4) {
        const uint2 r = *reinterpret_cast<const uint2*>(q);
        wv[0] = r.x; wv[1] = r.y;
      } else {
        wv[0] = *reinterpret_cast<const uint32_t*>(q);
      }
#pragma unroll
      for (int k = 0; k < CH / 2; ++k) {
        v[gi * CH + 2 * k] = __uint_as_float(wv[k] << 16);
        v[gi * CH + 2 * k + 1] = __uint_as_float(wv[k] & 0xffff0000u);
      }
    }
  };
  auto st = [&](bf16_t* row, const float* v) {
#pragma unroll
    for (int gi = 0; gi < NG; ++gi) {
      bf16_t* q = row + gi * 256 * CH + t * CH;
      const float* o = v + gi * CH;
      if constexpr (CH == 8) {
        *reinterpret_cast<uint4*>(q) = make_uint4(pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3]),
                                                  pack_bf2(o[4], o[5]), pack_bf2(o[6], o[7]));
      } else if constexpr (CH == 4) {
        *reinterpret_cast<uint2*>(q) = make_uint2(pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3]));
      } else {
        *reinterpret_cast<uint32_t*>(q) = pack_bf2(o[0], o[1]);
      }
    }
  };
  // same (row, col) -> Philox word map as dropout_keep (HK: the pair hash of dropout_keep_pair)
  const uint32_t hsm = HK ? pair_seedmix(seed, offset + rng_base()) : 0u, hthr = pair_thr16(p);
  auto keep_mask = [&](int64_t row, bool* keep) {
    if constexpr (HK) {
#pragma unroll
      for (int i = 0; i < VT; i += 2) {  // CH even: elements i, i + 1 are one column pair
        const uint32_t h = pair_hash(hsm, (uint32_t)row, (uint32_t)col(i));
        keep[i] = (h & 0xffffu) >= hthr;
        keep[i + 1] = (h >> 16) >= hthr;
      }
      return;
    }
    const uint32_t thr = (uint32_t)(p * 4294967296.0);
#pragma unroll
    for (int i = 0; i < VT; i += 2) {
      const int c = col(i);  // pairs never straddle a 4-column Philox block (c even)
      uint32_t r[4];
      if (CH >= 4 && (i % 4) != 0) continue;
      philox4(seed, 0x5bd1e995u, (uint32_t)row, (uint32_t)(row >> 32) ^ (uint32_t)(c >> 2), offset + rng_base(),
              0xdeadbeefu, r);
      if constexpr (CH >= 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k) keep[i + k] = r[k] >= thr;
      } else {
        keep[i] = r[c & 3] >= thr;
        keep[i + 1] = r[(c & 3) + 1] >= thr;
      }
    }
  };
  float g[VT], adg[VT], adb[VT], ady[VT];
  ld(gamma, g);
  float bt[XO ? VT : 1], rg[XO ? VT : 1];
  __shared__ int nsmall;
  bool xo = false;  // block-uniform (the threads hold different columns of gamma)
  if constexpr (XO) {
    ld(beta, bt);
    bool small = false;
#pragma unroll
    for (int i = 0; i < VT; ++i) {
      rg[i] = inv_gamma(g[i]);
      small |= xo_unsafe(g[i], bt[i]);
    }
    if (t == 0) nsmall = 0;
    __syncthreads();
    if (small) nsmall = 1;
    __syncthreads();
    xo = nsmall == 0;
  }
  const bf16_t* const hsrc = XO && !xo ? hcopy : hsave;
#pragma unroll
  for (int i = 0; i < VT; ++i) { adg[i] = 0.f; adb[i] = 0.f; ady[i] = 0.f; }
  const float sc = p > 0.f ? 1.f / (1.f - p) : 1.f;
  int par = 0;
  for (int64_t row = blockIdx.x; row < R; row += gridDim.x, par ^= 1) {
    float h[VT], d[VT];
    ld(hsrc + row * D, h);
    ld(dout + row * D, d);
    if (POST && p > 0.f) {
      bool keep[VT];
      keep_mask(row, keep);
#pragma unroll
      for (int i = 0; i < VT; ++i) d[i] = keep[i] ? d[i] * sc : 0.f;
    }
    const float mean = mean_in[row], rstd = rstd_in[row];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VT; ++i) {
      float xh;
      if (XO && xo) xh = (h[i] - bt[i]) * rg[i]; else xh = (h[i] - mean) * rstd;
      adg[i] += d[i] * xh;
      adb[i] += d[i];
      const float gx = d[i] * g[i];
      h[i] = xh;
      d[i] = gx;
      s1 += gx;
      s2 += gx * xh;
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    if (lane == 0) {
      rsum[par][w][0] = s1;
      rsum[par][w][1] = s2;
    }
    __syncthreads();  // the other parity's slots were read before this barrier (previous row)
    s1 = (rsum[par][0][0] + rsum[par][1][0] + rsum[par][2][0] + rsum[par][3][0]) * (1.f / D);
    s2 = (rsum[par][0][1] + rsum[par][1][1] + rsum[par][2][1] + rsum[par][3][1]) * (1.f / D);
#pragma unroll
    for (int i = 0; i < VT; ++i) d[i] = rstd * (d[i] - s1 - h[i] * s2);
    if (dh_in) {
      float e[VT];
      ld(dh_in + row * D, e);
#pragma unroll
      for (int i = 0; i < VT; ++i) d[i] += e[i];
    }
    if (dres) st(dres + row * D, d);
    if (dy) {
      if (!POST && p > 0.f) {
        bool keep[VT];
        keep_mask(row, keep);
#pragma unroll
        for (int i = 0; i < VT; ++i) d[i] = keep[i] ? d[i] * sc : 0.f;
      }
      st(dy + row * D, d);
      if (want_dyb) {
#pragma unroll
        for (int i = 0; i < VT; ++i) ady[i] += bf2f(f2bf(d[i]));
      }
    }
  }
  float* pr = part + (int64_t)blockIdx.x * 3 * D;
#pragma unroll
  for (int i = 0; i < VT; ++i) {
    if (part_acc) {
      adg[i] += pr[col(i)];
      adb[i] += pr[D + col(i)];
      if (want_dyb) ady[i] += pr[2 * D + col(i)];
    }
    pr[col(i)] = adg[i];
    pr[D + col(i)] = adb[i];
    if (want_dyb) pr[2 * D + col(i)] = ady[i];
  }
}

// Second stage of the two-stage column sums, in two fixed-order passes (no fp32 atomics: the
// LayerNorm / bias gradients are bitwise reproducible).  Pass 1, grid (D / 64, #accumulators,
// NSEG): a block sums column chunk x of accumulator y over its segment of the nb block partials
// (64 columns x 4 row lanes, coalesced 256-B rows) and stores the segment sum IN PLACE, over its
// segment's first partial row (a row no other block reads).  Pass 2 (ln_colfinal_kernel) adds the
// NSEG segment sums in segment order onto the destination.
__global__ void __launch_bounds__(256) ln_colreduce_kernel(float* __restrict__ part, int nb, int D, int astride) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), rl = threadIdx.x >> 6, a = blockIdx.y;
  const int per = (nb + gridDim.z - 1) / gridDim.z;
  const int r0 = blockIdx.z * per, r1 = min(nb, r0 + per);
  float t = 0.f;
  if (c < D)
    for (int r = r0 + rl; r < r1; r += 4) t += part[((int64_t)r * astride + a) * D + c];
  red[rl][threadIdx.x & 63] = t;
  __syncthreads();
  if (rl == 0 && r0 < r1 && c < D)
    part[((int64_t)r0 * astride + a) * D + c] =
        (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
}

// grid (D / 64, #accumulators), 64 threads: dst_a[c] += sum over segments (in order) of pass 1's sums
__global__ void __launch_bounds__(64) ln_colfinal_kernel(const float* __restrict__ part, int nb, int D, int astride,
                                                        int nseg, float* __restrict__ d0, float* __restrict__ d1,
                                                        float* __restrict__ d2) {
  const int c = blockIdx.x * 64 + threadIdx.x, a = blockIdx.y;
  if (c >= D) return;
  const int per = (nb + nseg - 1) / nseg;
  float t = 0.f;
  for (int sg = 0; sg < nseg && sg * per < nb; ++sg) t += part[((int64_t)sg * per * astride + a) * D + c];
  float* dst = a == 0 ? d0 : a == 1 ? d1 : d2;
  dst[c] += t;
}

static void colsum_two_pass(float* part, int nb, int D, int astride, int nacc, float* d0, float* d1, float* d2,
                            hipStream_t s) {
  const int nseg = nb >= 256 ? 16 : nb >= 32 ? 4 : 1;
  const unsigned cb = (unsigned)((D + 63) / 64);
  hipLaunchKernelGGL(ln_colreduce_kernel, dim3(cb, nacc, nseg), dim3(256), 0, s, part, nb, D, astride);
  hipLaunchKernelGGL(ln_colfinal_kernel, dim3(cb, nacc), dim3(64), 0, s, (const float*)part, nb, D, astride,
                     nseg, d0, d1, d2);
}

#define DPA_LN_DISPATCH(D, FN, ...)                      \
  switch (D) {                                           \
    case 64: FN<1>(__VA_ARGS__); break;                  \
    case 128: FN<2>(__VA_ARGS__); break;                 \
    case 256: FN<4>(__VA_ARGS__); break;                 \
    case 512: FN<8>(__VA_ARGS__); break;                 \
    case 768: FN<12>(__VA_ARGS__); break;                \
    case 1024: FN<16>(__VA_ARGS__); break;               \
    case 1536: FN<24>(__VA_ARGS__); break;               \
    case 2048: FN<32>(__VA_ARGS__); break;               \
    default: return false;                               \
  }

template <int VEC>
static void ln_fwd_impl(const uint16_t* y, const uint16_t* res, const uint16_t* g, const uint16_t* b,
                        uint16_t* out, uint16_t* hsave, float* mean, float* rstd, int64_t R, float p,
                        float eps, uint32_t seed, uint32_t off, const uint16_t* pos, const uint16_t* temb,
                        int L, bool post, bool hguard, hipStream_t s) {
  // a few resident waves per SIMD, each walking rows: R / 32 blocks (8 rows per wave) clamped to
  // [4, 32] blocks per CU.  Interleaved
  // A/Bs: 262144 rows best at 8192 blocks (profiles/wt_shadow_r5.txt); 32768 rows (seq 512 x 64)
  // and 8192 rows (the 32 x 64 schedule) -0.25% each at 1024 blocks vs 8192 / 2048
  // (profiles/ln_bwd_blocks_r5.txt)
  int64_t nb = (R + 3) / 4;
  const int64_t cu = device_cu_count();
  const int64_t cap = std::min(std::max((R + 31) / 32, cu * 4), cu * 32);
  if (nb > cap) nb = cap;
  const unsigned grid = (unsigned)nb;
  hipLaunchKernelGGL(add_ln_fwd_kernel<VEC>, dim3(grid), dim3(256), 0, s, (const bf16_t*)y,
                     (const bf16_t*)res, (const bf16_t*)g, (const bf16_t*)b, (bf16_t*)out,
                     (bf16_t*)hsave, mean, rstd, R, p, eps, seed, off, (const bf16_t*)pos,
                     (const bf16_t*)temb, L < 1 ? 1 : L, post ? 1 : 0, hguard ? 1 : 0);
}

bool launch_add_ln_fwd(const uint16_t* y, const uint16_t* res, const uint16_t* g, const uint16_t* b,
                       uint16_t* out, uint16_t* hsave, float* mean, float* rstd, int64_t R, int D,
                       float p, float eps, uint32_t seed, uint32_t off, hipStream_t s, const uint16_t* pos,
                       const uint16_t* temb, int L, bool post, bool hguard) {
  if ((pos || temb) && (L < 1 || R % L)) return false;
  DPA_LN_DISPATCH(D, ln_fwd_impl, y, res, g, b, out, hsave, mean, rstd, R, p, eps, seed, off, pos, temb, L,
                  post, hguard, s)
  return true;
}

// at least 32 rows per block: the per-block column-sum atomics (3 x D per block) stay a
// small share at small R (8192-row micro-batch: 256 blocks instead of 512; same-box A/B
// on the reference 32 x 64 schedule 327.2 -> 324.0 ms/step); large R is capped at 512 blocks
int ln_bwd_blocks(int64_t R) {
  int64_t nb = (R + 31) / 32;
  return (int)(nb < 512 ? nb : 512);
}

// Small R (a 64-sample micro-batch of the reference schedule is 8192 rows): 32 rows per
// block left 4 waves per CU, each walking 8 rows back to back - latency-bound at ~1.7 TB/s
// (29 us per call).  Two rows per wave instead (8 per block), with the block column sums
// stored as partials (9.4 MB at 8192 x 768, plain 16-byte stores) and reduced by a second
// kernel - more blocks would otherwise cost one fp32 atomic per column per block.
constexpr int64_t LN_SMALL_R = 65536;
// rows per block of the small-R kernel: 8 waves x 2 rows (was 4 x 2: the 8192 x 768 partials were
// 9.4 MB written and, deferred, re-read per call against ~38 MB of row traffic)
#ifndef DPA_LN_SMALL_NW
#define DPA_LN_SMALL_NW 8
#endif
constexpr int LN_SMALL_NW = DPA_LN_SMALL_NW;
constexpr int LN_SMALL_ROWS = 2 * LN_SMALL_NW;
// wide rows (D >= 1536, add_ln_bwd_rowblk_kernel): always two-stage, up to 1024 blocks (the
// partials are 3 x D floats per block; the second stage reads them once)
constexpr int LN_WIDE_D = 1536;
// The small-R kernel grid-strides, so its block count is capped at one 8-wave block per CU
// a 32768-row micro-batch (seq 512 x 64) walks 16 rows
// per wave and stores 2.4 MB of partials instead of 18.9 MB, 8192 rows 4 per wave.  Interleaved
// A/Bs (profiles/ln_bwd_blocks_r5.txt): seq512 8 x 64 -1.1% at 1024 blocks and -0.2% more at
// 256; the 32 x 64 schedule -0.75% at 256 vs 1024 (= the old 512 at 8192 rows), +0.3% at 128.
// Large R (> LN_SMALL_R): the 4-wave grid of ln_bwd_blocks, its block partials summed in two
// ordered passes too (4.7 MB at 512 blocks x 3 x 768) instead of one fp32 atomic per column per
// block - the reduction is deterministic at every R.
static int64_t ln_bwd_two_stage_blocks(int64_t R, int D) {
  if (D >= LN_WIDE_D) return R < 1024 ? R : 1024;  // add_ln_bwd_rowblk_kernel: one row per block at a time
  const int64_t cap = device_cu_count();
  if (R <= LN_SMALL_R) {
    const int64_t nb = (R + LN_SMALL_ROWS - 1) / LN_SMALL_ROWS;
    return cap > 0 && nb > cap ? cap : nb;
  }
  return ln_bwd_blocks(R);
}
int64_t ln_bwd_ws_floats(int64_t R, int D) { return ln_bwd_two_stage_blocks(R, D) * 3 * D; }

// Second stage of the two-stage column sums: part[nb][3][D] -> dg, db (, dyb) (+=); the partials
// are consumed (pass 1 stores its segment sums over them)
static void ln_colreduce_launch(float* part, int nb, int D, float* dg, float* db, float* dyb, hipStream_t s) {
  colsum_two_pass(part, nb, D, 3, dyb ? 3 : 2, dg, db, dyb, s);
}

// part_mode (two-stage shapes only, ws = a caller-owned partial buffer of ln_bwd_ws_floats):
// 0 the partials are reduced onto dg / db / dyb right away; 1 they are stored and 2 added
// onto the buffer's previous contents, with no reduction - the caller runs
// launch_ln_colreduce once over the sum of several micro-batches' partials.
template <int VEC>
static void ln_bwd_impl(const uint16_t* dout, const uint16_t* hsave, const float* mean,
                        const float* rstd, const uint16_t* g, uint16_t* dres, uint16_t* dy,
                        float* dyb, float* dg, float* db, int64_t R, float p, uint32_t seed,
                        uint32_t off, const uint16_t* dh_in, bool post, int zero_mask, hipStream_t s,
                        float* ws, int part_mode, const uint16_t* beta, const uint16_t* hcopy, bool hk) {
  constexpr int D = VEC * 64;
  const int64_t nb2 = ln_bwd_two_stage_blocks(R, D);
  const bool two_stage = ws != nullptr && nb2 > 0;
  const int nb = two_stage ? (int)nb2 : ln_bwd_blocks(R);
  const bool pacc = two_stage && part_mode == 2, reduce = !two_stage || part_mode == 0;
  // zero the accumulators that are scratch (zero_mask bits: 1 dg, 2 db, 4 dyb); the others
  // are parameter .grad buffers the kernel accumulates onto.  One memset when the scratch
  // ones are consecutive rows of one buffer (the binding allocates them so).
  const bool zg = zero_mask & 1, zb = zero_mask & 2, zy = dyb && (zero_mask & 4);
  if (zg && zb && db == dg + D && (!dyb || !zy || dyb == dg + 2 * D)) {
    (void)hipMemsetAsync(dg, 0, sizeof(float) * D * (zy ? 3 : 2), s);
  } else {
    if (zg) (void)hipMemsetAsync(dg, 0, sizeof(float) * D, s);
    if (zb) (void)hipMemsetAsync(db, 0, sizeof(float) * D, s);
    if (zy) (void)hipMemsetAsync(dyb, 0, sizeof(float) * D, s);
  }
  float* part = two_stage ? ws : nullptr;
  float* const dyb_k = dy ? dyb : nullptr;
  // beta != nullptr: `hsave` is the LN output (pre-dropout placement only: a post-dropout
  // output has zeroed elements and cannot be inverted)
  const bool xo = beta != nullptr && hcopy != nullptr && !post;
  const bf16_t* bt = (const bf16_t*)beta;
  if constexpr (D >= LN_WIDE_D) {
    if (two_stage) {
#define DPA_LN_ROWBLK(P, X, H)                                                                              \
  hipLaunchKernelGGL((add_ln_bwd_rowblk_kernel<D, P, X, H>), dim3(nb), dim3(256), 0, s, (const bf16_t*)dout, \
                     (const bf16_t*)hsave, mean, rstd, (const bf16_t*)g, (bf16_t*)dres, (bf16_t*)dy,      \
                     dyb_k != nullptr, R, p, seed, off, (const bf16_t*)dh_in, part, pacc, bt,    \
                     (const bf16_t*)hcopy)
      if (post) DPA_LN_ROWBLK(true, false, false);
      else if (hk) DPA_LN_ROWBLK(false, false, true);
      else if (xo) DPA_LN_ROWBLK(false, true, false);
      else DPA_LN_ROWBLK(false, false, false);
#undef DPA_LN_ROWBLK
      if (reduce) ln_colreduce_launch(part, nb, D, dg, db, dyb_k, s);
      return;
    }
  }
#define DPA_LN_BWD_NW(P, X, H, NWV)                                                                          \
  hipLaunchKernelGGL((add_ln_bwd_kernel<VEC, P, X, H, NWV>), dim3(nb), dim3(NWV * 64), 0, s,                  \
                     (const bf16_t*)dout, (const bf16_t*)hsave, mean, rstd, (const bf16_t*)g, (bf16_t*)dres,  \
                     (bf16_t*)dy, dyb_k, dg, db, R, p, seed, off, (const bf16_t*)dh_in, part, pacc, bt,       \
                     (const bf16_t*)hcopy)
#define DPA_LN_BWD(P, X, H)                             \
  do {                                                  \
    if constexpr (D < LN_WIDE_D) {                      \
      if (two_stage && R <= LN_SMALL_R) {               \
        DPA_LN_BWD_NW(P, X, H, LN_SMALL_NW);            \
        break;                                          \
      }                                                 \
    }                                                   \
    DPA_LN_BWD_NW(P, X, H, 4);                          \
  } while (0)
  if (post) DPA_LN_BWD(true, false, false);
  else if (hk) DPA_LN_BWD(false, false, true);
  else if (xo) DPA_LN_BWD(false, true, false);
  else DPA_LN_BWD(false, false, false);
#undef DPA_LN_BWD
#undef DPA_LN_BWD_NW
  if (two_stage && reduce) ln_colreduce_launch(part, nb, D, dg, db, dyb_k, s);
}

bool launch_ln_colreduce(float* part, int64_t R, int D, float* dg, float* db, float* dyb, hipStream_t s) {
  const int64_t nb = ln_bwd_two_stage_blocks(R, D);
  if (nb <= 0 || D % 64) return false;
  ln_colreduce_launch(part, (int)nb, D, dg, db, dyb, s);
  return true;
}

// dst[c] += sum_r part[r][c] (fp32 [rows][cols] partials, cols % 64 == 0): the bias
// gradient of a fused epilogue's per-tile column sums, accumulated straight onto the
// parameter's fp32 .grad (no ATen reduce + autograd add per micro-batch)
bool launch_colsum_acc(float* part, int rows, int cols, float* dst, hipStream_t s) {
  if (cols <= 0 || rows <= 0) return false;
  colsum_two_pass(part, rows, cols, 1, 1, dst, nullptr, nullptr, s);
  return true;
}

// Position- and sequence-sums of a [B][L][H] bf16 gradient in ONE read (the DiffuSeq input
// block's position-embedding and time-embedding gradients; two ATen reductions read it twice):
//   dtemb[b][h] = sum_l d[b][l][h]      (written here)
//   part[g][l][h] = sum_{b in group g} d[b][l][h]   (summed over g by colsum_acc afterwards)
// Workgroup = 16 sequences x 64 columns; thread (c, q) sums rows l = q + 4k of column c, so a
// wave reads 64 contiguous columns of one row; LQ = L / 4 position partials live in registers.
template <int LQ>
__global__ void __launch_bounds__(256) seq_pos_partial_kernel(const bf16_t* __restrict__ d, int B, int H,
                                                              float* __restrict__ dtemb,
                                                              float* __restrict__ part) {
  constexpr int L = 4 * LQ, BG = 16;
  __shared__ float red[4][64];
  const int c = blockIdx.y * 64 + (threadIdx.x & 63), q = threadIdx.x >> 6;
  const int g = blockIdx.x, b0 = g * BG;
  float pacc[LQ];
#pragma unroll
  for (int k = 0; k < LQ; ++k) pacc[k] = 0.f;
  for (int bi = 0; bi < BG && b0 + bi < B; ++bi) {
    const bf16_t* row = d + ((int64_t)(b0 + bi) * L + q) * H + c;
    float sb = 0.f;
#pragma unroll
    for (int k = 0; k < LQ; ++k) {
      const float v = bf2f(row[(int64_t)k * 4 * H]);
      pacc[k] += v;
      sb += v;
    }
    red[q][threadIdx.x & 63] = sb;
    __syncthreads();
    if (q == 0 && dtemb)
      dtemb[(int64_t)(b0 + bi) * H + c] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                                          red[3][threadIdx.x];
    __syncthreads();
  }
  if (part) {
    float* pg = part + (int64_t)g * L * H + c;
#pragma unroll
    for (int k = 0; k < LQ; ++k) pg[(int64_t)(q + 4 * k) * H] = pacc[k];
  }
}

int seq_pos_groups(int B) { return (B + 15) / 16; }

bool launch_seq_pos_sums(const uint16_t* d, int B, int L, int H, float* dpos, float* dtemb, float* part,
                         hipStream_t s) {
  if (H % 64 || B <= 0 || (L != 64 && L != 128 && L != 256)) return false;
  const dim3 grid((unsigned)seq_pos_groups(B), (unsigned)(H / 64));
  float* pp = dpos ? part : nullptr;
  switch (L) {
    case 64: hipLaunchKernelGGL(seq_pos_partial_kernel<16>, grid, dim3(256), 0, s, (const bf16_t*)d, B, H, dtemb, pp); break;
    case 128: hipLaunchKernelGGL(seq_pos_partial_kernel<32>, grid, dim3(256), 0, s, (const bf16_t*)d, B, H, dtemb, pp); break;
    default: hipLaunchKernelGGL(seq_pos_partial_kernel<64>, grid, dim3(256), 0, s, (const bf16_t*)d, B, H, dtemb, pp); break;
  }
  if (dpos) launch_colsum_acc(part, seq_pos_groups(B), L * H, dpos, s);  // dpos (zeroed) += sum_g part[g]
  return true;
}

bool launch_add_ln_bwd(const uint16_t* dout, const uint16_t* hsave, const float* mean,
                       const float* rstd, const uint16_t* g, uint16_t* dres, uint16_t* dy, float* dyb,
                       float* dg, float* db, int64_t R, int D, float p, uint32_t seed, uint32_t off,
                       hipStream_t s, const uint16_t* dh_in, bool post, int zero_mask, float* ws,
                       int part_mode, const uint16_t* beta, const uint16_t* hcopy, bool pair_hash) {
  if (beta && (post || !hcopy)) return false;  // a post-dropout output cannot be inverted
  if (pair_hash && (post || beta)) return false;  // the pair-hash bits are the pre-dropout GEMM epilogue's
  DPA_LN_DISPATCH(D, ln_bwd_impl, dout, hsave, mean, rstd, g, dres, dy, dyb, dg, db, R, p, seed,
                  off, dh_in, post, zero_mask, s, ws, part_mode, beta, hcopy, pair_hash)
  return true;
}

DPA_RNG_BASE_EXPORT(norm)

}  // namespace dpa
