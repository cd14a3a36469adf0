// Fused optimizer-side kernels over the flat parameter/gradient buffers of the
// native DDP engine (SURVEY K-1, K-4..K-7).
//
// The reference trainer (utils/trainer.py:237-271, 360-370) runs, per step:
// per-parameter grad-norm `.item()` host syncs, torch AdamW (foreach kernels
// over 209 tensors) and R x P EMA mul_/add_ pairs.  Here a step is:
//   1. sqnorm_partial  : one grid-stride pass over the flat grad buffer
//   2. sqnorm_finalize : one block -> grad norm + clip coefficient (on device)
//   3. adamw_ema       : ONE pass reading g, m, v, p and every EMA buffer,
//                        writing m, v, p, the bf16 compute copy and the EMAs.
// Nothing syncs with the host; the norm stays on device until the logger dumps.
#include "common.h"
#include "launchers.h"

namespace dpa {

template <typename T>
struct Vec4Load;

template <>
struct Vec4Load<float> {
  __device__ __forceinline__ static f32x4 load(const float* p, int64_t i) {
    return *reinterpret_cast<const f32x4*>(p + i);
  }
};

template <>
struct Vec4Load<bf16_t> {
  __device__ __forceinline__ static f32x4 load(const bf16_t* p, int64_t i) {
    uint2 raw = *reinterpret_cast<const uint2*>(p + i);
    f32x4 r;
    r[0] = __uint_as_float(raw.x << 16);
    r[1] = __uint_as_float(raw.x & 0xffff0000u);
    r[2] = __uint_as_float(raw.y << 16);
    r[3] = __uint_as_float(raw.y & 0xffff0000u);
    return r;
  }
};

// ---------------------------------------------------------------------------
// Sum of squares, stage 1: each block writes one partial.  n % 4 == 0.
// ---------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) sqnorm_partial_kernel(const T* __restrict__ g, int64_t n,
                                                             float* __restrict__ partial) {
  __shared__ float red[4];
  float acc = 0.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
    f32x4 v = Vec4Load<T>::load(g, i);
    acc += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
  }
  acc = block_sum(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

// Stage 2: norm = sqrt(sum)*scale; coef = clamp(max_norm/(norm+1e-6), max=1)
// (torch.nn.utils.clip_grad_norm_ semantics).  out[0] = norm (pre-clip),
// out[1] = coef, out[2] = norm after clipping (what the reference logs).
__global__ void __launch_bounds__(1024) sqnorm_finalize_kernel(const float* __restrict__ partial,
                                                               int nparts, float scale, float max_norm,
                                                               float* __restrict__ out) {
  __shared__ double red[16];
  double acc = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) acc += (double)partial[i];
  acc = wave_sum_d(acc);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
    float norm = (float)sqrt(s) * scale;
    float coef = 1.f;
    if (max_norm > 0.f) coef = fminf(1.f, max_norm / (norm + 1e-6f));
    out[0] = norm;
    out[1] = coef;
    out[2] = norm * coef;
  }
}

// ---------------------------------------------------------------------------
// Fused AdamW (torch semantics, decoupled weight decay) + multi-rate EMA +
// bf16 shadow-weight refresh.  All buffers are flat, 16-byte aligned, n % 4 == 0.
// ---------------------------------------------------------------------------
struct EmaArgs {
  float* buf[4];
  float rate[4];
  int count;
};

template <typename T>
__global__ void __launch_bounds__(256) adamw_ema_kernel(
    float* __restrict__ p, const T* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
    bf16_t* __restrict__ p16, EmaArgs ema, int64_t n, float lr, float beta1, float beta2,
    float eps, float wd, float step_size, float inv_bc2_sqrt, float grad_scale,
    const float* __restrict__ clip, const int* __restrict__ skip) {
  // skip != nullptr: the step is refused while *skip != 0 (a failed gradient
  // all-reduce, csrc/ipc_allreduce.hip) - parameters, moments and EMAs stay as they were
  if (skip && __builtin_nontemporal_load(skip) != 0) return;
  const float gs = grad_scale * (clip ? clip[1] : 1.f);
  const float decay = 1.f - lr * wd;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
    f32x4 gv = Vec4Load<T>::load(g, i);
    f32x4 pv = *reinterpret_cast<f32x4*>(p + i);
    f32x4 mv = *reinterpret_cast<f32x4*>(m + i);
    f32x4 vv = *reinterpret_cast<f32x4*>(v + i);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gk = gv[k] * gs;
      float pk = pv[k] * decay;
      float mk = mv[k] + (1.f - beta1) * (gk - mv[k]);
      float vk = vv[k] * beta2 + (1.f - beta2) * gk * gk;
      float denom = sqrtf(vk) * inv_bc2_sqrt + eps;
      pk = pk - step_size * (mk / denom);
      pv[k] = pk; mv[k] = mk; vv[k] = vk;
    }
    *reinterpret_cast<f32x4*>(p + i) = pv;
    *reinterpret_cast<f32x4*>(m + i) = mv;
    *reinterpret_cast<f32x4*>(v + i) = vv;
    if (p16) {
      uint2 packed;
      packed.x = pack_bf2(pv[0], pv[1]);
      packed.y = pack_bf2(pv[2], pv[3]);
      *reinterpret_cast<uint2*>(p16 + i) = packed;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (e < ema.count) {
        float r = ema.rate[e];
        f32x4 ev = *reinterpret_cast<f32x4*>(ema.buf[e] + i);
#pragma unroll
        for (int k = 0; k < 4; ++k) ev[k] = ev[k] * r + pv[k] * (1.f - r);
        *reinterpret_cast<f32x4*>(ema.buf[e] + i) = ev;
      }
    }
  }
}

// Plain EMA update (used when the optimizer is not the fused one).
__global__ void __launch_bounds__(256) ema_kernel(float* __restrict__ e, const float* __restrict__ p,
                                                 int64_t n, float rate) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
    f32x4 ev = *reinterpret_cast<f32x4*>(e + i);
    f32x4 pv = *reinterpret_cast<const f32x4*>(p + i);
#pragma unroll
    for (int k = 0; k < 4; ++k) ev[k] = ev[k] * rate + pv[k] * (1.f - rate);
    *reinterpret_cast<f32x4*>(e + i) = ev;
  }
}

// fp32 -> bf16 flat copy (shadow-weight refresh outside the optimizer).
__global__ void __launch_bounds__(256) cast_bf16_kernel(const float* __restrict__ src,
                                                       bf16_t* __restrict__ dst, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
    f32x4 v = *reinterpret_cast<const f32x4*>(src + i);
    uint2 packed;
    packed.x = pack_bf2(v[0], v[1]);
    packed.y = pack_bf2(v[2], v[3]);
    *reinterpret_cast<uint2*>(dst + i) = packed;
  }
}

// bf16 -> fp32 flat copy (unpacking a bf16-wire gradient bucket).
__global__ void __launch_bounds__(256) cast_f32_kernel(const bf16_t* __restrict__ src,
                                                      float* __restrict__ dst, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += stride) {
    const uint2 u = *reinterpret_cast<const uint2*>(src + i);
    *reinterpret_cast<f32x4*>(dst + i) = f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                                              __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
  }
}

static inline int grid_for(int64_t n, int per_thread, int block, int cap) {
  int64_t g = (n / per_thread + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

// ---------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------
void launch_sqnorm(const void* g, bool g_bf16, int64_t n, float* partial, int nparts, float scale,
                   float max_norm, float* out, hipStream_t s) {
  int grid = grid_for(n, 4, 256, nparts);
  if (g_bf16)
    hipLaunchKernelGGL(sqnorm_partial_kernel<bf16_t>, dim3(grid), dim3(256), 0, s,
                       (const bf16_t*)g, n, partial);
  else
    hipLaunchKernelGGL(sqnorm_partial_kernel<float>, dim3(grid), dim3(256), 0, s,
                       (const float*)g, n, partial);
  hipLaunchKernelGGL(sqnorm_finalize_kernel, dim3(1), dim3(1024), 0, s, partial, grid, scale,
                     max_norm, out);
}

void launch_adamw_ema(float* p, const void* g, bool g_bf16, float* m, float* v, uint16_t* p16,
                      float* const* ema_bufs, const float* ema_rates, int n_ema, int64_t n, float lr,
                      float beta1, float beta2, float eps, float wd, int64_t step, float grad_scale,
                      const float* clip, hipStream_t s, const int* skip) {
  EmaArgs ea;
  ea.count = n_ema > 4 ? 4 : n_ema;
  for (int e = 0; e < 4; ++e) {
    ea.buf[e] = e < ea.count ? ema_bufs[e] : nullptr;
    ea.rate[e] = e < ea.count ? ema_rates[e] : 0.f;
  }
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  const float step_size = (float)(lr / bc1);
  const float inv_bc2_sqrt = (float)(1.0 / sqrt(bc2));
  // ~1 MiB of work per block keeps ~8 blocks/CU resident on 256 CUs.
  int grid = grid_for(n, 4, 256, 256 * 8);
  if (g_bf16)
    hipLaunchKernelGGL(adamw_ema_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, p, (const bf16_t*)g,
                       m, v, (bf16_t*)p16, ea, n, lr, beta1, beta2, eps, wd, step_size,
                       inv_bc2_sqrt, grad_scale, clip, skip);
  else
    hipLaunchKernelGGL(adamw_ema_kernel<float>, dim3(grid), dim3(256), 0, s, p, (const float*)g, m,
                       v, (bf16_t*)p16, ea, n, lr, beta1, beta2, eps, wd, step_size, inv_bc2_sqrt,
                       grad_scale, clip, skip);
  // More than 4 EMA rates: remaining ones as plain passes (not gated by `skip`: the
  // engine raises on a set flag before the next step anyway).
  for (int e = 4; e < n_ema; ++e)
    hipLaunchKernelGGL(ema_kernel, dim3(grid), dim3(256), 0, s, ema_bufs[e], p, n, ema_rates[e]);
}

void launch_ema(float* e, const float* p, int64_t n, float rate, hipStream_t s) {
  hipLaunchKernelGGL(ema_kernel, dim3(grid_for(n, 4, 256, 2048)), dim3(256), 0, s, e, p, n, rate);
}

void launch_cast_f32(const uint16_t* src, float* dst, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(cast_f32_kernel, dim3(grid_for(n, 4, 256, 2048)), dim3(256), 0, s, (const bf16_t*)src,
                     dst, n);
}

void launch_cast_bf16(const float* src, uint16_t* dst, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(cast_bf16_kernel, dim3(grid_for(n, 4, 256, 2048)), dim3(256), 0, s, src,
                     (bf16_t*)dst, n);
}

// ---- batched bf16 transpose (the transposed weight shadows of ops/nn.py shadow_t) -------------
// One launch for every weight: block b takes the 64 x 64 tile that the prefix sums of the per-weight
// tile counts assign it, reads it with 4-byte row loads into LDS (a 66-element row pitch: the
// column reads hit distinct banks) and writes it transposed with 4-byte row stores.
__global__ void __launch_bounds__(256) transpose_bf16_batch_kernel(TransposeBatch d) {
  __shared__ uint16_t tile[64][66];
  int w = 0;
  while (w + 1 < d.n && (int)blockIdx.x >= d.tile_start[w + 1]) ++w;
  const int rows = d.rows[w], cols = d.cols[w];
  const int lt = (int)blockIdx.x - d.tile_start[w], tc = cols / 64;
  const int r0 = (lt / tc) * 64, c0 = (lt % tc) * 64;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const uint16_t* src = d.src[w];
  uint16_t* dst = d.dst[w];
#pragma unroll
  for (int r = ty; r < 64; r += 8) {
    const uint32_t v = *reinterpret_cast<const uint32_t*>(src + (int64_t)(r0 + r) * cols + c0 + 2 * tx);
    tile[r][2 * tx] = (uint16_t)(v & 0xffffu);
    tile[r][2 * tx + 1] = (uint16_t)(v >> 16);
  }
  __syncthreads();
#pragma unroll
  for (int c = ty; c < 64; c += 8) {
    const uint32_t v = (uint32_t)tile[2 * tx][c] | ((uint32_t)tile[2 * tx + 1][c] << 16);
    *reinterpret_cast<uint32_t*>(dst + (int64_t)(c0 + c) * rows + r0 + 2 * tx) = v;
  }
}

bool launch_transpose_bf16_batch(const TransposeBatch& d, hipStream_t s) {
  if (d.n <= 0 || d.n > TransposeBatch::MAXN) return false;
  for (int i = 0; i < d.n; ++i)
    if (d.rows[i] % 64 || d.cols[i] % 64 || d.rows[i] <= 0 || d.cols[i] <= 0) return false;
  const int tiles = d.tile_start[d.n];
  if (tiles <= 0) return false;
  hipLaunchKernelGGL(transpose_bf16_batch_kernel, dim3(tiles), dim3(256), 0, s, d);
  return true;
}

}  // namespace dpa
