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
// wave64 owns a row: D/64 contiguous elements per lane (D = 768 -> 12), loaded
// as 8-byte vectors, so a row is one fully coalesced 1.5 KiB transaction and
// both reductions are a single wave-wide shuffle tree (no LDS, no barriers).
// The dropout mask is never stored: it is regenerated from the counter-based
// Philox stream (seed, offset, row, column) in the backward.
//
// dgamma/dbeta: each block accumulates its rows' contributions in registers,
// reduces its 4 waves through LDS and adds one fp32 atomic per column.
#include "common.h"
#include "launchers.h"

namespace dpa {

template <int VEC>
struct RowIO {
  // load VEC bf16 (VEC % 4 == 0 uses 8-byte vectors)
  __device__ __forceinline__ static void load(const bf16_t* p, float* v) {
    if constexpr (VEC % 4 == 0) {
#pragma unroll
      for (int c = 0; c < VEC / 4; ++c) {
        uint2 raw = *reinterpret_cast<const uint2*>(p + 4 * c);
        v[4 * c + 0] = __uint_as_float(raw.x << 16);
        v[4 * c + 1] = __uint_as_float(raw.x & 0xffff0000u);
        v[4 * c + 2] = __uint_as_float(raw.y << 16);
        v[4 * c + 3] = __uint_as_float(raw.y & 0xffff0000u);
      }
    } else {
#pragma unroll
      for (int c = 0; c < VEC; ++c) v[c] = bf2f(p[c]);
    }
  }
  __device__ __forceinline__ static void store(bf16_t* p, const float* v) {
    if constexpr (VEC % 4 == 0) {
#pragma unroll
      for (int c = 0; c < VEC / 4; ++c) {
        uint2 raw;
        raw.x = pack_bf2(v[4 * c + 0], v[4 * c + 1]);
        raw.y = pack_bf2(v[4 * c + 2], v[4 * c + 3]);
        *reinterpret_cast<uint2*>(p + 4 * c) = raw;
      }
    } else {
#pragma unroll
      for (int c = 0; c < VEC; ++c) p[c] = f2bf(v[c]);
    }
  }
};

// keep-mask bits for this lane's VEC elements of `row`, from one Philox call per 4.
template <int VEC>
__device__ __forceinline__ void dropout_keep(uint32_t seed, uint32_t offset, int64_t row, int col0,
                                             float p, bool* keep) {
  const uint32_t thr = (uint32_t)(p * 4294967296.0);
#pragma unroll
  for (int c = 0; c < (VEC + 3) / 4; ++c) {
    uint32_t r[4];
    philox4(seed, 0x5bd1e995u, (uint32_t)row, (uint32_t)(row >> 32) ^ (uint32_t)((col0 >> 2) + c),
            offset, 0xdeadbeefu, r);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (4 * c + k < VEC) keep[4 * c + k] = r[k] >= thr;
  }
}

template <int VEC>
__global__ void __launch_bounds__(256) add_ln_fwd_kernel(
    const bf16_t* __restrict__ y, const bf16_t* __restrict__ res, const bf16_t* __restrict__ gamma,
    const bf16_t* __restrict__ beta, bf16_t* __restrict__ out, bf16_t* __restrict__ hsave,
    float* __restrict__ mean_out, float* __restrict__ rstd_out, int64_t R, float p, float eps,
    uint32_t seed, uint32_t offset, const bf16_t* __restrict__ pos, const bf16_t* __restrict__ temb,
    int L, int post) {
  constexpr int D = VEC * 64;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= R) return;
  const int col0 = lane * VEC;
  float h[VEC];
  RowIO<VEC>::load(y + row * D + col0, h);
  if (pos) {
    float t[VEC];
    RowIO<VEC>::load(pos + (row % L) * D + col0, t);
#pragma unroll
    for (int i = 0; i < VEC; ++i) h[i] += t[i];
  }
  if (temb) {
    float t[VEC];
    RowIO<VEC>::load(temb + (row / L) * D + col0, t);
#pragma unroll
    for (int i = 0; i < VEC; ++i) h[i] += t[i];
  }
  if (p > 0.f && !post) {
    bool keep[VEC];
    dropout_keep<VEC>(seed, offset, row, col0, p, keep);
    const float sc = 1.f / (1.f - p);
#pragma unroll
    for (int i = 0; i < VEC; ++i) h[i] = keep[i] ? h[i] * sc : 0.f;
  }
  if (res) {
    float r[VEC];
    RowIO<VEC>::load(res + row * D + col0, r);
#pragma unroll
    for (int i = 0; i < VEC; ++i) h[i] += r[i];
  }
  // round h to bf16 first so the backward (which reloads the bf16 copy) is consistent
#pragma unroll
  for (int i = 0; i < VEC; ++i) h[i] = bf2f(f2bf(h[i]));
  if (hsave) RowIO<VEC>::store(hsave + row * D + col0, h);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VEC; ++i) s += h[i];
  const float mean = wave_sum(s) * (1.f / D);
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < VEC; ++i) { const float d = h[i] - mean; v += d * d; }
  const float rstd = rsqrtf(wave_sum(v) * (1.f / D) + eps);
  float g[VEC], b[VEC], o[VEC];
  RowIO<VEC>::load(gamma + col0, g);
  RowIO<VEC>::load(beta + col0, b);
#pragma unroll
  for (int i = 0; i < VEC; ++i) o[i] = (h[i] - mean) * rstd * g[i] + b[i];
  if (p > 0.f && post) {
    bool keep[VEC];
    dropout_keep<VEC>(seed, offset, row, col0, p, keep);
    const float sc = 1.f / (1.f - p);
#pragma unroll
    for (int i = 0; i < VEC; ++i) o[i] = keep[i] ? o[i] * sc : 0.f;
  }
  RowIO<VEC>::store(out + row * D + col0, o);
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// grid-stride over rows; block = 4 waves; partial dgamma/dbeta per block.
// POST at compile time (the two dropout placements share no loop body) and <= 128 VGPRs
// (4 waves per SIMD: the LDS reduction buffer allows 4 blocks per CU); D > 768 keeps
// 6 x VEC live accumulator/row floats: 2 waves per SIMD up to D = 1536, 1 for D = 2048
// (512 VGPRs) - no scratch spills at any width
template <int VEC, bool POST>
__global__ void __launch_bounds__(256, VEC <= 12 ? 4 : VEC <= 24 ? 2 : 1) add_ln_bwd_kernel(
    const bf16_t* __restrict__ dout, const bf16_t* __restrict__ hsave,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const bf16_t* __restrict__ gamma, bf16_t* __restrict__ dres, bf16_t* __restrict__ dy,
    float* __restrict__ dyb, float* __restrict__ part_dg, float* __restrict__ part_db, int64_t R,
    float p, uint32_t seed, uint32_t offset, const bf16_t* __restrict__ dh_in, float* __restrict__ part) {
  constexpr int D = VEC * 64;
  __shared__ float red[4][D];  // reused for dgamma, dbeta, dyb in turn (D = 2048: 32 KiB)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col0 = lane * VEC;
  float g[VEC], adg[VEC], adb[VEC], ady[VEC];
  RowIO<VEC>::load(gamma + col0, g);
#pragma unroll
  for (int i = 0; i < VEC; ++i) { adg[i] = 0.f; adb[i] = 0.f; ady[i] = 0.f; }
  const float sc = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (int64_t row = (int64_t)blockIdx.x * 4 + w; row < R; row += (int64_t)gridDim.x * 4) {
    float h[VEC], d[VEC];
    RowIO<VEC>::load(hsave + row * D + col0, h);
    RowIO<VEC>::load(dout + row * D + col0, d);
    if (POST && p > 0.f) {
      bool keep[VEC];
      dropout_keep<VEC>(seed, offset, row, col0, p, keep);
#pragma unroll
      for (int i = 0; i < VEC; ++i) d[i] = keep[i] ? d[i] * sc : 0.f;
    }
    const float mean = mean_in[row], rstd = rstd_in[row];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      const float xh = (h[i] - mean) * rstd;
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
      RowIO<VEC>::load(dh_in + row * D + col0, e);
#pragma unroll
      for (int i = 0; i < VEC; ++i) d[i] += e[i];
    }
    if (dres) RowIO<VEC>::store(dres + row * D + col0, d);
    if (dy) {
      if (!POST && p > 0.f) {
        bool keep[VEC];
        dropout_keep<VEC>(seed, offset, row, col0, p, keep);
#pragma unroll
        for (int i = 0; i < VEC; ++i) d[i] = keep[i] ? d[i] * sc : 0.f;
      }
      RowIO<VEC>::store(dy + row * D + col0, d);
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
    for (int i = 0; i < VEC; ++i) red[w][col0 + i] = a == 0 ? adg[i] : a == 1 ? adb[i] : ady[i];
    __syncthreads();
    if (part) {
      float* pr = part + ((int64_t)blockIdx.x * 3 + a) * D;
      for (int c = threadIdx.x; c < D; c += blockDim.x) pr[c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
    } else {
      for (int c = threadIdx.x; c < D; c += blockDim.x)
        atomicAdd(dst[a] + c, red[0][c] + red[1][c] + red[2][c] + red[3][c]);
    }
  }
}

// Second stage of the small-R column sums: grid (D / 64, #accumulators, NSEG); a block sums
// column chunk x of accumulator y over its segment of the nb block partials (64 columns x 4
// row lanes, 16-byte-free coalesced 256-B rows) and adds one atomic per column.
__global__ void __launch_bounds__(256) ln_colreduce_kernel(const float* __restrict__ part, int nb, int D,
                                                          float* __restrict__ d0, float* __restrict__ d1,
                                                          float* __restrict__ d2, int astride) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), rl = threadIdx.x >> 6, a = blockIdx.y;
  const int per = (nb + gridDim.z - 1) / gridDim.z;
  const int r0 = blockIdx.z * per, r1 = min(nb, r0 + per);
  float t = 0.f;
  for (int r = r0 + rl; r < r1; r += 4) t += part[((int64_t)r * astride + a) * D + c];
  red[rl][threadIdx.x & 63] = t;
  __syncthreads();
  if (rl == 0) {
    float* dst = a == 0 ? d0 : a == 1 ? d1 : d2;
    atomicAdd(dst + c, red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x]);
  }
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
                        int L, bool post, hipStream_t s) {
  const unsigned grid = (unsigned)((R + 3) / 4);
  hipLaunchKernelGGL(add_ln_fwd_kernel<VEC>, dim3(grid), dim3(256), 0, s, (const bf16_t*)y,
                     (const bf16_t*)res, (const bf16_t*)g, (const bf16_t*)b, (bf16_t*)out,
                     (bf16_t*)hsave, mean, rstd, R, p, eps, seed, off, (const bf16_t*)pos,
                     (const bf16_t*)temb, L < 1 ? 1 : L, post ? 1 : 0);
}

bool launch_add_ln_fwd(const uint16_t* y, const uint16_t* res, const uint16_t* g, const uint16_t* b,
                       uint16_t* out, uint16_t* hsave, float* mean, float* rstd, int64_t R, int D,
                       float p, float eps, uint32_t seed, uint32_t off, hipStream_t s, const uint16_t* pos,
                       const uint16_t* temb, int L, bool post) {
  if ((pos || temb) && (L < 1 || R % L)) return false;
  DPA_LN_DISPATCH(D, ln_fwd_impl, y, res, g, b, out, hsave, mean, rstd, R, p, eps, seed, off, pos, temb, L,
                  post, s)
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
int64_t ln_bwd_ws_floats(int64_t R, int D) {
  if (R > LN_SMALL_R) return 0;
  const int64_t nb = (R + 7) / 8;
  return nb * 3 * D;
}

template <int VEC>
static void ln_bwd_impl(const uint16_t* dout, const uint16_t* hsave, const float* mean,
                        const float* rstd, const uint16_t* g, uint16_t* dres, uint16_t* dy,
                        float* dyb, float* dg, float* db, int64_t R, float p, uint32_t seed,
                        uint32_t off, const uint16_t* dh_in, bool post, int zero_mask, hipStream_t s,
                        float* ws) {
  constexpr int D = VEC * 64;
  const bool two_stage = ws != nullptr && R <= LN_SMALL_R;
  const int nb = two_stage ? (int)((R + 7) / 8) : ln_bwd_blocks(R);
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
  if (post)
    hipLaunchKernelGGL((add_ln_bwd_kernel<VEC, true>), dim3(nb), dim3(256), 0, s, (const bf16_t*)dout,
                       (const bf16_t*)hsave, mean, rstd, (const bf16_t*)g, (bf16_t*)dres, (bf16_t*)dy,
                       dy ? dyb : nullptr, dg, db, R, p, seed, off, (const bf16_t*)dh_in, part);
  else
    hipLaunchKernelGGL((add_ln_bwd_kernel<VEC, false>), dim3(nb), dim3(256), 0, s, (const bf16_t*)dout,
                       (const bf16_t*)hsave, mean, rstd, (const bf16_t*)g, (bf16_t*)dres, (bf16_t*)dy,
                       dy ? dyb : nullptr, dg, db, R, p, seed, off, (const bf16_t*)dh_in, part);
  if (two_stage) {
    const int nacc = (dy && dyb) ? 3 : 2;
    const int nseg = nb >= 256 ? 16 : nb >= 32 ? 4 : 1;
    hipLaunchKernelGGL(ln_colreduce_kernel, dim3(D / 64, nacc, nseg), dim3(256), 0, s, part, nb, D, dg, db,
                       dy ? dyb : nullptr, 3);
  }
}

// dst[c] += sum_r part[r][c] (fp32 [rows][cols] partials, cols % 64 == 0): the bias
// gradient of a fused epilogue's per-tile column sums, accumulated straight onto the
// parameter's fp32 .grad (no ATen reduce + autograd add per micro-batch)
bool launch_colsum_acc(const float* part, int rows, int cols, float* dst, hipStream_t s) {
  if (cols % 64 || rows <= 0) return false;
  const int nseg = rows >= 256 ? 16 : rows >= 32 ? 4 : 1;
  hipLaunchKernelGGL(ln_colreduce_kernel, dim3(cols / 64, 1, nseg), dim3(256), 0, s, part, rows, cols, dst,
                     (float*)nullptr, (float*)nullptr, 1);
  return true;
}

bool launch_add_ln_bwd(const uint16_t* dout, const uint16_t* hsave, const float* mean,
                       const float* rstd, const uint16_t* g, uint16_t* dres, uint16_t* dy, float* dyb,
                       float* dg, float* db, int64_t R, int D, float p, uint32_t seed, uint32_t off,
                       hipStream_t s, const uint16_t* dh_in, bool post, int zero_mask, float* ws) {
  DPA_LN_DISPATCH(D, ln_bwd_impl, dout, hsave, mean, rstd, g, dres, dy, dyb, dg, db, R, p, seed,
                  off, dh_in, post, zero_mask, s, ws)
  return true;
}

}  // namespace dpa
