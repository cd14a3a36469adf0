// bf16 MFMA GEMM for the transformer Linear layers (SURVEY K-M5/K-M7/K-M9..K-M11),
// one template for the three products of a Linear layer y = x W^T + b:
//
//   fwd   : y[T][N]  = x[T][K]  . W[N][K]^T   (+ bias, activation)   A "MK",  B "NK"
//   dgrad : dx[T][K] = dy[T][N] . W[N][K]                            A "MK",  B "KN"
//   wgrad : dW[N][K] += dy[T][N]^T . x[T][K]   (+ db = colsum dy)     A "KM",  B "KN"
//
// Tiles: 128 x 128 per workgroup, BK = 64, 4 waves as 2 x 2, each wave a 64 x 64
// block of four v_mfma_f32_32x32x16_bf16 accumulators.  Operands are staged
// global -> registers -> XOR-swizzled LDS (double buffered; the next tile's
// global loads are issued before the current tile's MFMAs, T14).  "MK"/"NK"
// operands are read as rows (ds_read_b128); "KM"/"KN" operands (reduction
// dimension outermost in memory) are read transposed with ds_read_b64_tr_b16,
// so no operand is ever transposed in global memory.
//
// wgrad splits the reduction (tokens) over grid.z and adds fp32 partial tiles
// straight into the fp32 gradient buffer with atomics: gradient accumulation
// across micro-batches is fused into the GEMM (no separate `grad += dW` pass),
// and db (if requested) is reduced from the staged dy tiles.
#include "common.h"
#include "launchers.h"
#include "mfma.h"

namespace dpa {

enum GemmEpi { EPI_BF16 = 0, EPI_BIAS_ACT = 1, EPI_ATOMIC_F32 = 2 };

__device__ __forceinline__ float gemm_act(float z, int act) {
  switch (act) {
    case 1: return 0.5f * z * (1.f + erff(z * 0.70710678118654752f));
    case 2: return tanhf(z);
    case 3: return z / (1.f + __expf(-z));
    default: return z;
  }
}

// One operand tile: either [128 rows][64 k] ("row", 128-B rows) or [64 k][128 cols] ("tr", 256-B rows)
template <bool TR>
struct Operand {
  static constexpr int ROWB = TR ? 256 : 128;
  static constexpr int CHR = TR ? 16 : 8;  // 16-B chunks per LDS row
  uint4 r[4];                              // 1024 chunks / 256 threads

  // global: element (i, k) of the logical [128][64] tile is at base[i*ld_i + k*ld_k]
  // with the contiguous dimension being k (row form) or i (tr form).
  __device__ __forceinline__ void load(const bf16_t* __restrict__ g, int64_t ld, int tid) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = tid + 256 * j;
      const int row = c / CHR, ch = c % CHR;
      r[j] = *reinterpret_cast<const uint4*>(g + (int64_t)row * ld + ch * 8);
    }
  }
  __device__ __forceinline__ void store(char* lds, int tid) const {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = tid + 256 * j;
      const int row = c / CHR, ch = c % CHR;
      *reinterpret_cast<uint4*>(lds + swz<ROWB>(row, ch)) = r[j];
    }
  }
  // fragment for MFMA k-step kk (16 wide) of the 32-row/col block starting at `b0`
  __device__ __forceinline__ static bf16x8 frag(const char* lds, int b0, int kk, int lane) {
    if constexpr (TR) return lds_tr_frag_nat<256>(lds, 16 * kk, b0, lane);
    else return lds_frag<128>(lds, b0 + (lane & 31), 2 * kk + (lane >> 5));
  }
};

template <bool A_TR, bool B_TR, int EPI>
__global__ void __launch_bounds__(256) gemm_kernel(
    const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ B, int64_t ldb,
    int M, int N, int K, int k_per_split, bf16_t* __restrict__ C, int64_t ldc,
    float* __restrict__ Cf, const bf16_t* __restrict__ bias, int act, bf16_t* __restrict__ Zout,
    float* __restrict__ colsum) {
  constexpr int TILE = 16384;  // bytes per operand tile
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.x * 128, n0 = blockIdx.y * 128;
  const int kbeg = blockIdx.z * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  const int nk = (kend - kbeg) / 64;

  // operand base pointers for the tile at k offset `k`
  auto a_ptr = [&](int k) -> const bf16_t* {
    return A_TR ? A + (int64_t)k * lda + m0 : A + (int64_t)m0 * lda + k;
  };
  auto b_ptr = [&](int k) -> const bf16_t* {
    return B_TR ? B + (int64_t)k * ldb + n0 : B + (int64_t)n0 * ldb + k;
  };

  Operand<A_TR> sa;
  Operand<B_TR> sb;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = zero16();

  // db = column sums of A (wgrad: A = dy^T, tr form, columns = m)
  const bool do_colsum = (EPI == EPI_ATOMIC_F32) && colsum != nullptr && blockIdx.y == 0;
  float cs[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) cs[i] = 0.f;

  if (nk > 0) {
    sa.load(a_ptr(kbeg), lda, tid);
    sb.load(b_ptr(kbeg), ldb, tid);
  }
  for (int t = 0; t < nk; ++t) {
    char* la = smem + (t & 1) * 2 * TILE;
    char* lb = la + TILE;
    sa.store(la, tid);
    sb.store(lb, tid);
    if constexpr (A_TR && EPI == EPI_ATOMIC_F32) {
      if (do_colsum) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t wv[4] = {sa.r[j].x, sa.r[j].y, sa.r[j].z, sa.r[j].w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            cs[2 * q] += __uint_as_float(wv[q] << 16);
            cs[2 * q + 1] += __uint_as_float(wv[q] & 0xffff0000u);
          }
        }
      }
    }
    __syncthreads();
    if (t + 1 < nk) {
      sa.load(a_ptr(kbeg + (t + 1) * 64), lda, tid);
      sb.load(b_ptr(kbeg + (t + 1) * 64), ldb, tid);
    }
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = Operand<A_TR>::frag(la, wm * 64 + i * 32, kk, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = Operand<B_TR>::frag(lb, wn * 64 + j * 32, kk, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(af[i], bfr[j], acc[i][j]);
    }
  }

  // ---- epilogue: acc[i][j] reg r -> row m0 + wm*64 + i*32 + acc_row(r, h), col n0 + wn*64 + j*32 + lane&31
  const int h = lane >> 5;
  if constexpr (EPI == EPI_ATOMIC_F32) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm * 64 + i * 32 + acc_row(r, h);
          const int col = n0 + wn * 64 + j * 32 + (lane & 31);
          atomicAdd(Cf + (int64_t)row * ldc + col, acc[i][j][r]);
        }
    if (do_colsum) {
      // this thread's 8 columns: chunk (tid % 16) of every staged row
      const int c0 = m0 + (tid & 15) * 8;
#pragma unroll
      for (int q = 0; q < 8; ++q) atomicAdd(colsum + c0 + q, cs[q]);
    }
  } else {
    float bv[2] = {0.f, 0.f};
    if (EPI == EPI_BIAS_ACT && bias) {
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[j] = bf2f(bias[n0 + wn * 64 + j * 32 + (lane & 31)]);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wm * 64 + i * 32 + acc_row(r, h);
          const int col = n0 + wn * 64 + j * 32 + (lane & 31);
          float v = acc[i][j][r] + bv[j];
          if (EPI == EPI_BIAS_ACT && act != 0) {
            v = bf2f(f2bf(v));
            if (Zout) Zout[(int64_t)row * ldc + col] = f2bf(v);
            v = gemm_act(v, act);
          }
          C[(int64_t)row * ldc + col] = f2bf(v);
        }
  }
}

static bool gemm_shape_ok(int M, int N, int K) { return M % 128 == 0 && N % 128 == 0 && K % 64 == 0; }

bool launch_gemm_nt(const uint16_t* x, const uint16_t* W, const uint16_t* bias, uint16_t* y,
                    uint16_t* z, int T, int N, int K, int act, hipStream_t s) {
  if (!gemm_shape_ok(T, N, K)) return false;
  dim3 grid(T / 128, N / 128, 1);
  hipLaunchKernelGGL((gemm_kernel<false, false, EPI_BIAS_ACT>), grid, dim3(256), 0, s,
                     (const bf16_t*)x, (int64_t)K, (const bf16_t*)W, (int64_t)K, T, N, K, K,
                     (bf16_t*)y, (int64_t)N, nullptr, (const bf16_t*)bias, act, (bf16_t*)z, nullptr);
  return true;
}

bool launch_gemm_nn(const uint16_t* dy, const uint16_t* W, uint16_t* dx, int T, int N, int K,
                    hipStream_t s) {
  // dx[T][K] = dy[T][N] . W[N][K]: M = T, N' = K, reduction = N
  if (!gemm_shape_ok(T, K, N)) return false;
  dim3 grid(T / 128, K / 128, 1);
  hipLaunchKernelGGL((gemm_kernel<false, true, EPI_BF16>), grid, dim3(256), 0, s,
                     (const bf16_t*)dy, (int64_t)N, (const bf16_t*)W, (int64_t)K, T, K, N, N,
                     (bf16_t*)dx, (int64_t)K, nullptr, nullptr, 0, nullptr, nullptr);
  return true;
}

bool launch_gemm_wgrad(const uint16_t* dy, const uint16_t* x, float* dW, float* db, int T, int N,
                       int K, hipStream_t s) {
  // dW[N][K] += dy[T][N]^T . x[T][K]: M = N, N' = K, reduction = T (split over grid.z)
  if (!gemm_shape_ok(N, K, T)) return false;
  const int tiles = (N / 128) * (K / 128);
  int splits = (1024 + tiles - 1) / tiles;
  const int ksteps = T / 64;
  if (splits > ksteps) splits = ksteps;
  if (splits < 1) splits = 1;
  const int kps = ((ksteps + splits - 1) / splits) * 64;
  splits = (T + kps - 1) / kps;
  dim3 grid(N / 128, K / 128, splits);
  hipLaunchKernelGGL((gemm_kernel<true, true, EPI_ATOMIC_F32>), grid, dim3(256), 0, s,
                     (const bf16_t*)dy, (int64_t)N, (const bf16_t*)x, (int64_t)K, N, K, T, kps,
                     nullptr, (int64_t)K, dW, nullptr, 0, nullptr, db);
  return true;
}

}  // namespace dpa
