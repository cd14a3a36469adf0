// Row-wise softmax cross-entropy over materialised logits: the chunked
// linear-CE path for WIDE inputs (GPT-2's E = 768 against V = 50257), where the
// register-resident fused kernels of xent.hip (E = 128/256) do not fit.
// ops/nn.py computes one token chunk's logits with hipBLASLt into a
// [chunk][ld] bf16 buffer (ld = V padded to a multiple of 64, so every row is
// 16-byte aligned), then:
//
//   xent_rows_fwd : per row  lse = log sum_v exp(l_v),  loss = lse - l_target
//   xent_rows_bwd : in place l_v <- g * (softmax_v - [v == target]),  padding -> 0
//
// so at most one chunk of logits exists at a time.  One 256-thread workgroup per
// row, 16-byte vector loads, online (max, sum) per thread merged across the wave
// by shuffles and across the 4 waves through LDS.  Targets outside [0, V) are
// ignored (loss 0, no gradient), as in xent.hip.
#include "common.h"
#include "launchers.h"

namespace dpa {

static constexpr float XR_LOG2E = 1.4426950408889634f;

__device__ __forceinline__ void xr_unpack8(const uint4& r, float* v) {
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = __uint_as_float(w[k] << 16);
    v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 xr_pack8(const float* v) {
  uint4 r;
  r.x = pack_bf2(v[0], v[1]);
  r.y = pack_bf2(v[2], v[3]);
  r.z = pack_bf2(v[4], v[5]);
  r.w = pack_bf2(v[6], v[7]);
  return r;
}

// (m, s) <- merge with (m2, s2): running max and sum of exp(x - max)
__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  const float M = fmaxf(m, m2);
  if (M == -INFINITY) return;  // both still empty
  s = s * fexp2((m - M) * XR_LOG2E) + s2 * fexp2((m2 - M) * XR_LOG2E);
  m = M;
}

__global__ void __launch_bounds__(256) xent_rows_fwd_kernel(const bf16_t* __restrict__ lg, int64_t ld,
                                                            int V, const int64_t* __restrict__ tgt,
                                                            float* __restrict__ loss,
                                                            float* __restrict__ lse_out) {
  __shared__ float red_m[4], red_s[4];
  const int64_t r = blockIdx.x;
  const bf16_t* row = lg + r * ld;
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x * 8; c < V; c += 256 * 8) {
    float v[8];
    xr_unpack8(*reinterpret_cast<const uint4*>(row + c), v);
    float tm = -INFINITY;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (c + k >= V) v[k] = -INFINITY;
      tm = fmaxf(tm, v[k]);
    }
    const float mn = fmaxf(m, tm);  // finite: column c < V is valid
    float add = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) add += fexp2((v[k] - mn) * XR_LOG2E);
    s = s * fexp2((m - mn) * XR_LOG2E) + add;
    m = mn;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lse_merge(m, s, __shfl_xor(m, o, 64), __shfl_xor(s, o, 64));
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    red_m[w] = m;
    red_s[w] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = red_m[0], S = red_s[0];
#pragma unroll
    for (int i = 1; i < 4; ++i) lse_merge(M, S, red_m[i], red_s[i]);
    const float l = M + logf(S);
    const int64_t t = tgt[r];
    const bool valid = t >= 0 && t < V;
    loss[r] = valid ? l - bf2f(row[t]) : 0.f;
    lse_out[r] = l;
  }
}

__global__ void __launch_bounds__(256) xent_rows_bwd_kernel(bf16_t* __restrict__ lg, int64_t ld, int V,
                                                            const int64_t* __restrict__ tgt,
                                                            const float* __restrict__ lse,
                                                            const float* __restrict__ dloss) {
  const int64_t r = blockIdx.x;
  bf16_t* row = lg + r * ld;
  const int64_t t = tgt[r];
  const bool valid = t >= 0 && t < V;
  const float g = valid ? dloss[r] : 0.f;
  const float l2 = lse[r] * XR_LOG2E;
  for (int c = threadIdx.x * 8; c < ld; c += 256 * 8) {
    float v[8];
    xr_unpack8(*reinterpret_cast<const uint4*>(row + c), v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int col = c + k;
      float p = col < V ? g * fexp2(fmaf(v[k], XR_LOG2E, -l2)) : 0.f;
      if (col == t) p -= g;
      v[k] = p;
    }
    *reinterpret_cast<uint4*>(row + c) = xr_pack8(v);
  }
}

// Forward that also leaves the UNSCALED gradient in place (training path when the
// logits chunk is kept for the backward):
//   l_v <- softmax_v - [v == target]   (0 for padding and for ignored targets)
// The row (~100 KB for GPT-2) is read from HBM for the statistics and read again right
// away for the gradient - a hit in the XCD's L2 - so HBM sees one read and one write per
// row instead of the fwd + bwd passes' two reads and one write; the backward only scales
// by the per-token upstream gradient (ops/nn.py folds that into the dx rows and the
// wgrad's x rows).  256 threads, low registers: many rows in flight per CU.
__global__ void __launch_bounds__(256) xent_rows_fwd_grad_kernel(bf16_t* __restrict__ lg, int64_t ld, int V,
                                                                const int64_t* __restrict__ tgt,
                                                                float* __restrict__ loss,
                                                                float* __restrict__ lse_out) {
  __shared__ float red_m[4], red_s[4], bcast;
  const int64_t r = blockIdx.x;
  bf16_t* row = lg + r * ld;
  const int64_t t = tgt[r];
  const bool valid = t >= 0 && t < V;
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x * 8; c < V; c += 256 * 8) {
    float v[8];
    xr_unpack8(*reinterpret_cast<const uint4*>(row + c), v);
    float tm = -INFINITY;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (c + k >= V) v[k] = -INFINITY;
      tm = fmaxf(tm, v[k]);
    }
    const float mn = fmaxf(m, tm);
    float add = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) add += fexp2((v[k] - mn) * XR_LOG2E);
    s = s * fexp2((m - mn) * XR_LOG2E) + add;
    m = mn;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lse_merge(m, s, __shfl_xor(m, o, 64), __shfl_xor(s, o, 64));
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    red_m[w] = m;
    red_s[w] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = red_m[0], S = red_s[0];
#pragma unroll
    for (int i = 1; i < 4; ++i) lse_merge(M, S, red_m[i], red_s[i]);
    const float l = M + logf(S);
    loss[r] = valid ? l - bf2f(row[t]) : 0.f;  // read before the block overwrites the row
    lse_out[r] = l;
    bcast = l * XR_LOG2E;
  }
  __syncthreads();
  const float l2 = bcast;
  for (int c = threadIdx.x * 8; c < ld; c += 256 * 8) {
    float v[8];
    xr_unpack8(*reinterpret_cast<const uint4*>(row + c), v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int col = c + k;
      float p = (valid && col < V) ? fexp2(fmaf(v[k], XR_LOG2E, -l2)) : 0.f;
      if (col == t) p -= 1.f;
      v[k] = p;
    }
    *reinterpret_cast<uint4*>(row + c) = xr_pack8(v);
  }
}

bool launch_xent_rows_fwd_grad(uint16_t* lg, int64_t ld, int V, const int64_t* tgt, int64_t R, float* loss,
                               float* lse, hipStream_t s) {
  if (ld % 8 != 0 || V > ld || V <= 0) return false;
  if (R > 0)
    hipLaunchKernelGGL(xent_rows_fwd_grad_kernel, dim3((unsigned)R), dim3(256), 0, s, (bf16_t*)lg, ld, V, tgt,
                       loss, lse);
  return true;
}

bool launch_xent_rows_fwd(const uint16_t* lg, int64_t ld, int V, const int64_t* tgt, int64_t R,
                          float* loss, float* lse, hipStream_t s) {
  if (ld % 8 != 0 || V > ld || V <= 0) return false;
  if (R > 0)
    hipLaunchKernelGGL(xent_rows_fwd_kernel, dim3((unsigned)R), dim3(256), 0, s, (const bf16_t*)lg, ld, V,
                       tgt, loss, lse);
  return true;
}

bool launch_xent_rows_bwd(uint16_t* lg, int64_t ld, int V, const int64_t* tgt, const float* lse,
                          const float* dloss, int64_t R, hipStream_t s) {
  if (ld % 8 != 0 || V > ld || V <= 0) return false;
  if (R > 0)
    hipLaunchKernelGGL(xent_rows_bwd_kernel, dim3((unsigned)R), dim3(256), 0, s, (bf16_t*)lg, ld, V, tgt,
                       lse, dloss);
  return true;
}

}  // namespace dpa
