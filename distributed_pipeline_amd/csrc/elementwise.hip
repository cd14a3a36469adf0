// GEMM epilogue kernels for Linear layers (SURVEY K-M4/K-M5/K-M10/K-M11):
//
//   fwd: z += bias (in place, bf16), y = act(z)            act in {none, gelu(erf), tanh, silu}
//   bwd: dz = dy * act'(z or y), db = sum_rows dz (fp32)
//
// Layout: block (64, 4); threadIdx.x owns 8 consecutive columns (one 16-byte
// vector per row), threadIdx.y strides rows; grid.y splits rows.  Column sums
// stay in registers across all of a thread's rows, are reduced over the 4
// row-lanes in LDS and added with one fp32 atomic per column per block.
#include "act.h"
#include "common.h"
#include "launchers.h"

namespace dpa {

enum Act { ACT_NONE = 0, ACT_GELU = 1, ACT_TANH = 2, ACT_SILU = 3 };
constexpr int kUnroll = 4;

__device__ __forceinline__ float act_f(float z, int act) { return act_apply(z, act); }
// derivative given pre-activation z (gelu/silu) or output y (tanh)
__device__ __forceinline__ float act_grad(float zy, int act) { return act_deriv(zy, act); }

__device__ __forceinline__ void unpack8(const uint4& r, float* v) {
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = __uint_as_float(w[k] << 16);
    v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 pack8(const float* v) {
  uint4 r;
  r.x = pack_bf2(v[0], v[1]);
  r.y = pack_bf2(v[2], v[3]);
  r.z = pack_bf2(v[4], v[5]);
  r.w = pack_bf2(v[6], v[7]);
  return r;
}

__global__ void __launch_bounds__(256) bias_act_fwd_kernel(bf16_t* __restrict__ z,
                                                          const bf16_t* __restrict__ bias,
                                                          bf16_t* __restrict__ y, int64_t R, int N,
                                                          int act) {
  const int c8 = (blockIdx.x * 64 + threadIdx.x) * 8;
  if (c8 >= N) return;
  float b[8];
  if (bias) unpack8(*reinterpret_cast<const uint4*>(bias + c8), b);
  else for (int k = 0; k < 8; ++k) b[k] = 0.f;
  const int64_t S = (int64_t)gridDim.y * 4;
  // kUnroll rows per trip, all loads issued before any math: enough 16-byte
  // requests in flight per CU to cover HBM latency at full occupancy.
  for (int64_t r0 = (int64_t)blockIdx.y * 4 + threadIdx.y; r0 < R; r0 += S * kUnroll) {
    uint4 raw[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int64_t r = r0 + u * S;
      if (r < R) raw[u] = *reinterpret_cast<const uint4*>(z + r * N + c8);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int64_t r = r0 + u * S;
      if (r >= R) break;
      const int64_t o = r * N + c8;
      float v[8];
      unpack8(raw[u], v);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = bf2f(f2bf(v[k] + b[k]));  // z is stored rounded
      if (bias) *reinterpret_cast<uint4*>(z + o) = pack8(v);
      if (y) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = act_f(v[k], act);
        *reinterpret_cast<uint4*>(y + o) = pack8(v);
      }
    }
  }
}

__global__ void __launch_bounds__(256) bias_act_bwd_kernel(const bf16_t* __restrict__ dy,
                                                          const bf16_t* __restrict__ zy,
                                                          bf16_t* __restrict__ dz,
                                                          float* __restrict__ part, int64_t R, int N,
                                                          int act) {
  __shared__ float red[4][64 * 8 + 4];
  const int c8 = (blockIdx.x * 64 + threadIdx.x) * 8;
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  if (c8 < N) {
    const int64_t S = (int64_t)gridDim.y * 4;
    const bool has_aux = act != ACT_NONE;
    for (int64_t r0 = (int64_t)blockIdx.y * 4 + threadIdx.y; r0 < R; r0 += S * kUnroll) {
      uint4 rd[kUnroll], rz[kUnroll];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int64_t r = r0 + u * S;
        if (r < R) {
          rd[u] = *reinterpret_cast<const uint4*>(dy + r * N + c8);
          if (has_aux) rz[u] = *reinterpret_cast<const uint4*>(zy + r * N + c8);
        }
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        const int64_t r = r0 + u * S;
        if (r >= R) break;
        float d[8];
        unpack8(rd[u], d);
        if (has_aux) {
          float zz[8];
          unpack8(rz[u], zz);
#pragma unroll
          for (int k = 0; k < 8; ++k) d[k] *= act_grad(zz[k], act);
        }
        if (dz) *reinterpret_cast<uint4*>(dz + r * N + c8) = pack8(d);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += bf2f(f2bf(d[k]));
      }
    }
  }
  if (!part) return;
#pragma unroll
  for (int k = 0; k < 8; ++k) red[threadIdx.y][threadIdx.x * 8 + k] = acc[k];
  __syncthreads();
  // this row block's column sums, a plain store into part[row block][N]; launch_colsum_acc adds the
  // row blocks in order (deterministic, no fp32 atomics)
  if (threadIdx.y == 0 && c8 < N) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int cc = threadIdx.x * 8 + k;
      part[(int64_t)blockIdx.y * N + c8 + k] = (red[0][cc] + red[1][cc]) + (red[2][cc] + red[3][cc]);
    }
  }
}

static unsigned row_blocks(int64_t R, int col_blocks) {
  int64_t target = 2048 / (col_blocks > 0 ? col_blocks : 1);
  if (target < 1) target = 1;
  int64_t need = (R + 3) / 4;
  return (unsigned)(need < target ? need : target);
}

void launch_bias_act_fwd(uint16_t* z, const uint16_t* bias, uint16_t* y, int64_t R, int N, int act,
                         hipStream_t s) {
  const int cb = (N / 8 + 63) / 64;
  hipLaunchKernelGGL(bias_act_fwd_kernel, dim3(cb, row_blocks(R, cb)), dim3(64, 4), 0, s,
                     (bf16_t*)z, (const bf16_t*)bias, (bf16_t*)y, R, N, act);
}

int64_t bias_act_bwd_ws_floats(int64_t R, int N) {
  const int cb = (N / 8 + 63) / 64;
  return (int64_t)row_blocks(R, cb) * N;
}

// db (nullable) += column sums of dz; ws: bias_act_bwd_ws_floats(R, N) floats when db is given
void launch_bias_act_bwd(const uint16_t* dy, const uint16_t* zy, uint16_t* dz, float* db, int64_t R,
                         int N, int act, hipStream_t s, float* ws) {
  const int cb = (N / 8 + 63) / 64;
  const unsigned rb = row_blocks(R, cb);
  float* part = db ? ws : nullptr;
  hipLaunchKernelGGL(bias_act_bwd_kernel, dim3(cb, rb), dim3(64, 4), 0, s,
                     (const bf16_t*)dy, (const bf16_t*)zy, (bf16_t*)dz, part, R, N, act);
  if (part) launch_colsum_acc(part, (int)rb, N, db, s);
}

}  // namespace dpa
