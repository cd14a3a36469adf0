// Row-wise softmax cross-entropy over materialised logits: the chunked
// linear-CE path for WIDE inputs (GPT-2's E = 768 against V = 50257), where the
// register-resident fused kernels of xent.hip (E = 128/256) do not fit.
// ops/nn.py computes one token chunk's logits with the native GEMM (gemm256.hip) into a
// [chunk][ld] bf16 buffer (ld = V padded to a multiple of 64, so every row is
// 16-byte aligned), then:
//
//   xent_rows_fwd : per row  lse = log sum_v exp(l_v),  loss = lse - l_target
//   xent_rows_bwd : in place l_v <- g * (softmax_v - [v == target]),  padding -> 0
//
// (the training path keeps the chunks and runs xent_rows_fwd_grad instead: the
// register-resident kernel below for rows up to 64K columns).  One 256-thread workgroup per
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

// Register-resident form of xent_rows_fwd_grad_kernel for rows up to NCH * 4096
// columns (GPT-2: ld = 50304 -> NCH = 13).  512 threads; thread i owns the 16-byte
// pieces at columns 8i + 4096j, j < NCH, and issues all NCH loads before touching
// any, so a workgroup has the whole ~100 KB row in flight at once (the looped kernel
// above keeps 4 KB per workgroup in flight and re-reads the row from L2 for the
// gradient).  The row stays in registers as packed bf16: max; exp(l - max) summed in
// fp32 and kept as bf16 in place of the logits; the gradient is that times 1/sum (one
// multiply instead of a second exp, two bf16 roundings instead of one).  Per-element
// masks are confined to the piece holding column V; the target's "- 1" is one extra
// 2-byte store by the thread that owns it, after its own vector store of that piece.
// the register-resident row must stay packed between passes: without this the compiler
// keeps pass 1's unpacked floats alive for pass 2 (220 VGPRs, 2 waves per SIMD)
__device__ __forceinline__ void xr_opaque(uint4& r) {
  asm volatile("" : "+v"(r.x), "+v"(r.y), "+v"(r.z), "+v"(r.w));
}

template <int NCH>
__global__ void __launch_bounds__(512) xent_rows_reg_kernel(bf16_t* __restrict__ lg, int64_t ld, int V,
                                                            const int64_t* __restrict__ tgt,
                                                            float* __restrict__ loss,
                                                            float* __restrict__ lse_out) {
  __shared__ float red[8];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int L = (int)ld;
  bf16_t* row = lg + (int64_t)blockIdx.x * ld;
  bf16_t* p = row + tid * 8;
  // column bounds relative to this thread's first column: piece j holds columns
  // j*4096 + [0, 8) of that frame, so the masks below compare against constants
  const int remV = V - tid * 8, remL = L - tid * 8;
  uint4 d[NCH];
#pragma unroll
  for (int j = 0; j < NCH; ++j)
    // unconditional loads (a guarded load becomes a branch with a wait per piece); a piece
    // past the row re-reads the row's last 8 columns and is masked out below (all >= V)
    d[j] = *reinterpret_cast<const uint4*>(p + min(j * 4096, remL - 8));
  const int64_t t = tgt[blockIdx.x];
  const bool valid = t >= 0 && t < V;
  const int tt = valid ? (int)t : -1;
  const bool owner = valid && ((tt & 4095) >> 3) == tid;  // holds column t (piece tt >> 12)
  const float vt = bf2f(row[valid ? tt : 0]);            // unconditional: no wait until the end
  // all pieces but the last hold real columns only when (NCH-1)*4096 <= V (the
  // exact-width instantiations): the per-element mask is then needed in the last piece alone
  const bool full = (NCH - 1) * 4096 <= V;
  // pass 1: row max over the V real columns
  float m = -INFINITY;
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    float v[8];
    xr_unpack8(d[j], v);
    if ((full && j < NCH - 1) || j * 4096 + 8 <= remV) {
#pragma unroll
      for (int k = 0; k < 8; ++k) m = fmaxf(m, v[k]);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) m = fmaxf(m, j * 4096 + k < remV ? v[k] : -INFINITY);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (lane == 0) red[w] = m;
  __syncthreads();
  float M = red[0];
#pragma unroll
  for (int i = 1; i < 8; ++i) M = fmaxf(M, red[i]);
  __syncthreads();  // red is reused for the sums
#pragma unroll
  for (int j = 0; j < NCH; ++j) xr_opaque(d[j]);
  // pass 2: e = exp(l - M) (0 past V), summed in fp32, kept as bf16
  const float m2 = M * XR_LOG2E;
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    float v[8];
    xr_unpack8(d[j], v);
    if ((full && j < NCH - 1) || j * 4096 + 8 <= remV) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = fexp2(fmaf(v[k], XR_LOG2E, -m2));
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = j * 4096 + k < remV ? fexp2(fmaf(v[k], XR_LOG2E, -m2)) : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[k];
    d[j] = xr_pack8(v);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) red[w] = s;
  __syncthreads();
  float S = red[0];
#pragma unroll
  for (int i = 1; i < 8; ++i) S += red[i];
  const float l = M + logf(S);
#pragma unroll
  for (int j = 0; j < NCH; ++j) xr_opaque(d[j]);
  asm volatile("" : "+v"(p));  // re-derive the store addresses here, not across the passes
  // pass 3: softmax = e / S in place (padding columns and ignored rows -> 0)
  const float inv = valid ? 1.f / S : 0.f;
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    if (j * 4096 < remL) {
      float v[8];
      xr_unpack8(d[j], v);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] *= inv;
      *reinterpret_cast<uint4*>(p + j * 4096) = xr_pack8(v);
    }
  }
  if (owner) {  // same thread, same address, after its vector store of this piece
    row[tt] = f2bf(fexp2(fmaf(vt, XR_LOG2E, -l * XR_LOG2E)) - 1.f);
    loss[blockIdx.x] = l - vt;
  }
  if (tid == 0) {
    lse_out[blockIdx.x] = l;
    if (!valid) loss[blockIdx.x] = 0.f;
  }
}

static int xent_rows_reg_mode() { return 1; }

bool launch_xent_rows_fwd_grad(uint16_t* lg, int64_t ld, int V, const int64_t* tgt, int64_t R, float* loss,
                               float* lse, hipStream_t s) {
  if (ld % 8 != 0 || V > ld || V <= 0) return false;
  if (R <= 0) return true;
  const int nch = (int)((ld + 4095) / 4096);
  if (xent_rows_reg_mode() && nch <= 16) {
    // instantiated widths; a row between two of them takes the wider one (extra pieces masked)
    const int up = nch <= 4 ? nch : nch <= 6 ? 6 : nch <= 8 ? 8 : nch <= 10 ? 10 : nch <= 13 ? 13 : 16;
#define DPA_XROWS_REG(N)                                                                            \
  case N:                                                                                           \
    hipLaunchKernelGGL(xent_rows_reg_kernel<N>, dim3((unsigned)R), dim3(512), 0, s, (bf16_t*)lg, ld, V, \
                       tgt, loss, lse);                                                             \
    return true;
    switch (up) {
      DPA_XROWS_REG(1) DPA_XROWS_REG(2) DPA_XROWS_REG(3) DPA_XROWS_REG(4) DPA_XROWS_REG(6)
      DPA_XROWS_REG(8) DPA_XROWS_REG(10) DPA_XROWS_REG(13) DPA_XROWS_REG(16)
      default: break;
    }
#undef DPA_XROWS_REG
  }
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
