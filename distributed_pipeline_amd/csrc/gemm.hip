// bf16 MFMA GEMM for the transformer Linear layers (SURVEY K-M5/K-M7/K-M9..K-M11),
// one template for the three products of a Linear layer y = x W^T + b:
//
//   fwd   : y[T][N]  = x[T][K]  . W[N][K]^T   (+ bias, activation)   A "MK",  B "NK"
//   dgrad : dx[T][K] = dy[T][N] . W[N][K]                            A "MK",  B "KN"
//   wgrad : dW[N][K] += dy[T][N]^T . x[T][K]   (+ db = colsum dy)     A "KM",  B "KN"
//
// Structure (CDNA4): 128 x 128 output tile per workgroup, BK = 64, 4 waves as
// 2 x 2 each owning a 64 x 64 block of four v_mfma_f32_32x32x16_bf16
// accumulators.  Operands go global -> LDS with global_load_lds_dwordx4 (no
// VGPR round trip, no ds_write), double buffered with the next tile in flight
// across the compute of the current one (counted vmcnt + raw s_barrier, never
// a vmcnt(0)-draining __syncthreads in the loop).  LDS images are XOR-swizzled
// through the per-lane *source* address (the DMA writes lane-linearly):
// "MK"/"NK" tiles are read as rows (ds_read_b128), "KM"/"KN" tiles - whose
// reduction dimension is outermost in memory - are read transposed with
// ds_read_b64_tr_b16, so no operand is ever transposed in global memory.
// Workgroup ids are remapped so tiles sharing an operand panel run on one XCD.
//
// wgrad splits the reduction (tokens) over workgroups and adds fp32 partial
// tiles straight into the fp32 gradient buffer with atomics (two 128-B row
// segments per wave instruction): gradient accumulation across micro-batches
// is fused into the GEMM, and db is reduced from the staged dy tiles.
#include "act.h"
#include "common.h"
#include "launchers.h"
#include "mfma.h"

namespace dpa {

enum GemmEpi { EPI_BF16 = 0, EPI_BIAS_ACT = 1, EPI_ATOMIC_F32 = 2 };

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void glob_void;

__device__ __forceinline__ float gemm_act(float z, int act) { return act_apply(z, act); }

// Operand tile: row form [128][64] (128-B rows) or transposed form [64][128] (256-B rows).
template <bool TR>
struct Op {
  static constexpr int ROWB = TR ? 256 : 128;
  static constexpr int CHR = TR ? 16 : 8;      // 16-B chunks per row
  static constexpr int RPP = 1024 / ROWB;      // rows per 1-KiB DMA piece

  // this wave issues 4 of the tile's 16 pieces; g points at element (row 0, chunk 0)
  __device__ __forceinline__ static void issue(char* lds, const bf16_t* __restrict__ g, int64_t ld,
                                               int w, int lane) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int pc = w * 4 + i;
      const int row = pc * RPP + lane / CHR;
      const int phys = lane % CHR;
      int logical;
      if constexpr (TR) logical = phys ^ swz_x256<>(row);  // inverse of swz<256>
      else logical = phys ^ ((row >> 1) & 7);
      const bf16_t* src = g + (int64_t)row * ld + logical * 8;
      __builtin_amdgcn_global_load_lds((glob_void*)src, (lds_void*)(lds + pc * 1024), 16, 0, 0);
    }
  }
  // Row form: an ordinary (compiler-counted) ds_read_b128.  Transposed form:
  // ds_read_b64_tr_b16 issued from inline asm - hipcc treats the builtin as
  // possibly aliasing the in-flight LDS-DMA and would drain vmcnt(0) before it,
  // serialising the prefetch; the caller waits lgkmcnt(0) on the results itself.
  __device__ __forceinline__ static bf16x8 frag(const char* lds, int b0, int kk, int lane) {
    if constexpr (TR) {
      const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3, h = lane >> 5;
      const int col = b0 + 16 * (g & 1) + 4 * p;
      const int ra = 16 * kk + 8 * h + q;
      const uint32_t base = lds_addr(lds);
      const uint32_t pa = base + swz<256>(ra, col >> 3) + (col & 7) * 2;
      const uint32_t pb = base + swz<256>(ra + 4, col >> 3) + (col & 7) * 2;
      bf16x4 a, b;
      asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(a) : "v"(pa));
      asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(b) : "v"(pb));
      return cat44(a, b);
    } else {
      return lds_frag<128>(lds, b0 + (lane & 31), 2 * kk + (lane >> 5));
    }
  }
  __device__ __forceinline__ static uint32_t lds_addr(const char* p) {
    return (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) char*)p);
  }
};

__device__ __forceinline__ void wait_lds_and_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ void wait_vm8_barrier() {
  asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ void wait_vm0_barrier() {
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
}

template <bool A_TR, bool B_TR, int EPI>
__global__ void __launch_bounds__(256) gemm_kernel(
    const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ B, int64_t ldb,
    int M, int N, int K, int k_per_split, int splits, bf16_t* __restrict__ C, int64_t ldc,
    float* __restrict__ Cf, const bf16_t* __restrict__ bias, int act, bf16_t* __restrict__ Zout,
    float* __restrict__ colsum) {
  constexpr int TILE = 16384;
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int MT = M / 128, NT = N / 128;
  const int tile = xcd_remap(blockIdx.x, MT * NT * splits);
  const int nt = tile % NT, mt = (tile / NT) % MT, z = tile / (NT * MT);
  const int m0 = mt * 128, n0 = nt * 128;
  const int kbeg = z * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  const int nk = (kend - kbeg) / 64;

  auto a_ptr = [&](int k) -> const bf16_t* {
    return A_TR ? A + (int64_t)k * lda + m0 : A + (int64_t)m0 * lda + k;
  };
  auto b_ptr = [&](int k) -> const bf16_t* {
    return B_TR ? B + (int64_t)k * ldb + n0 : B + (int64_t)n0 * ldb + k;
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = zero16();

  const bool do_colsum = (EPI == EPI_ATOMIC_F32) && colsum != nullptr && nt == 0;
  float cs[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) cs[i] = 0.f;

  if (nk > 0) {
    Op<A_TR>::issue(smem, a_ptr(kbeg), lda, w, lane);
    Op<B_TR>::issue(smem + TILE, b_ptr(kbeg), ldb, w, lane);
    if (nk > 1) {
      Op<A_TR>::issue(smem + 2 * TILE, a_ptr(kbeg + 64), lda, w, lane);
      Op<B_TR>::issue(smem + 3 * TILE, b_ptr(kbeg + 64), ldb, w, lane);
      wait_vm8_barrier();
    } else {
      wait_vm0_barrier();
    }
  }
  for (int t = 0; t < nk; ++t) {
    const char* la = smem + (t & 1) * 2 * TILE;
    const char* lb = la + TILE;
    if constexpr (A_TR && EPI == EPI_ATOMIC_F32) {
      if (do_colsum) {
        // 16 chunk-columns x 16 row groups of 4 rows of the [64 k][128 m] A image
        const int ch = tid & 15, rg = tid >> 4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rg * 4 + r;
          const uint4 v = *reinterpret_cast<const uint4*>(la + swz<256>(row, ch));
          const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            cs[2 * q] += __uint_as_float(wv[q] << 16);
            cs[2 * q + 1] += __uint_as_float(wv[q] & 0xffff0000u);
          }
        }
      }
    }
    // k-steps pipelined through two fragment register sets: the LDS reads of
    // step kk+1 are in flight while the 4 MFMAs of step kk issue.
    bf16x8 af[2][2], bfr[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) af[0][i] = Op<A_TR>::frag(la, wm * 64 + i * 32, 0, lane);
#pragma unroll
    for (int j = 0; j < 2; ++j) bfr[0][j] = Op<B_TR>::frag(lb, wn * 64 + j * 32, 0, lane);
    if constexpr (A_TR || B_TR)
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(af[0][0]), "+v"(af[0][1]), "+v"(bfr[0][0]), "+v"(bfr[0][1]));
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int cur = kk & 1, nxt = cur ^ 1;
      if (kk < 3) {
#pragma unroll
        for (int i = 0; i < 2; ++i) af[nxt][i] = Op<A_TR>::frag(la, wm * 64 + i * 32, kk + 1, lane);
#pragma unroll
        for (int j = 0; j < 2; ++j) bfr[nxt][j] = Op<B_TR>::frag(lb, wn * 64 + j * 32, kk + 1, lane);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma32(af[cur][i], bfr[cur][j], acc[i][j]);
      if constexpr (A_TR || B_TR) {
        if (kk < 3)  // retire the asm transposed reads (results named as operands)
          asm volatile("s_waitcnt lgkmcnt(0)"
                       : "+v"(af[nxt][0]), "+v"(af[nxt][1]), "+v"(bfr[nxt][0]), "+v"(bfr[nxt][1]));
      }
    }
    if (t + 1 < nk) {
      wait_lds_and_barrier();  // every wave is done reading this buffer
      if (t + 2 < nk) {
        char* da = smem + (t & 1) * 2 * TILE;
        Op<A_TR>::issue(da, a_ptr(kbeg + (t + 2) * 64), lda, w, lane);
        Op<B_TR>::issue(da + TILE, b_ptr(kbeg + (t + 2) * 64), ldb, w, lane);
        wait_vm8_barrier();    // tile t+1 landed (this wave's pieces), then everyone's
      } else {
        wait_vm0_barrier();
      }
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
      const int c0 = m0 + (tid & 15) * 8;
#pragma unroll
      for (int q = 0; q < 8; ++q) atomicAdd(colsum + c0 + q, cs[q]);
    }
  } else {
    // Stage the bf16 tile through LDS and write whole 256-B rows with 16-B stores
    // (instead of 64 scattered 2-B stores per lane).  Z (pre-activation) second.
    constexpr int LDC = 136;  // padded row (elements)
    bf16_t* ct = reinterpret_cast<bf16_t*>(smem);
    float bv[2] = {0.f, 0.f};
    if (EPI == EPI_BIAS_ACT && bias) {
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[j] = bf2f(bias[n0 + wn * 64 + j * 32 + (lane & 31)]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // operand LDS no longer read
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = wm * 64 + i * 32 + acc_row(r, h);
          const int col = wn * 64 + j * 32 + (lane & 31);
          ct[row * LDC + col] = f2bf(acc[i][j][r] + bv[j]);
        }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // 128 rows x 16 chunks of 8: pre-activation to Zout, act(z) to C
#pragma unroll 2
    for (int c = 0; c < 8; ++c) {
      const int idx = tid + c * 256;
      const int row = idx >> 4, ch = idx & 15;
      uint4 v = *reinterpret_cast<const uint4*>(ct + row * LDC + ch * 8);
      const int64_t o = (int64_t)(m0 + row) * ldc + n0 + ch * 8;
      if (EPI == EPI_BIAS_ACT && act != 0) {
        if (Zout) *reinterpret_cast<uint4*>(Zout + o) = v;
        uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float lo = gemm_act(__uint_as_float(wv[q] << 16), act);
          const float hi = gemm_act(__uint_as_float(wv[q] & 0xffff0000u), act);
          wv[q] = pack_bf2(lo, hi);
        }
        v = make_uint4(wv[0], wv[1], wv[2], wv[3]);
      }
      *reinterpret_cast<uint4*>(C + o) = v;
    }
  }
}

static bool gemm_shape_ok(int M, int N, int K) { return M % 128 == 0 && N % 128 == 0 && K % 64 == 0; }

// Compute units of the current device (cached per device id): the persistent GEMMs
// launch one workgroup per CU.
int device_cu_count() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cache[dev] <= 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

// zderiv (in/out, nullable): requests act'(pre-activation) in z instead of the
// pre-activation; reset to false when the kernel that ran stored the pre-activation.
bool launch_gemm_nt(const uint16_t* x, const uint16_t* W, const uint16_t* bias, uint16_t* y,
                    uint16_t* z, int T, int N, int K, int act, hipStream_t s, bool* zderiv, int hm) {
  const bool want_d = zderiv && *zderiv;
  if (launch_gemmp_nt(x, W, bias, y, z, T, N, K, act, device_cu_count(), s, want_d, hm)) return true;
  if (hm) return false;  // the head-major store exists on the persistent kernel only
  if (zderiv) *zderiv = false;
  if (launch_gemm256_nt(x, W, bias, y, z, T, N, K, act, s)) return true;
  if (!gemm_shape_ok(T, N, K)) return false;
  const int blocks = (T / 128) * (N / 128);
  hipLaunchKernelGGL((gemm_kernel<false, false, EPI_BIAS_ACT>), dim3(blocks), dim3(256), 0, s,
                     (const bf16_t*)x, (int64_t)K, (const bf16_t*)W, (int64_t)K, T, N, K, K, 1,
                     (bf16_t*)y, (int64_t)N, nullptr, (const bf16_t*)bias, act, (bf16_t*)z, nullptr);
  return true;
}

bool launch_gemm_nn(const uint16_t* dy, const uint16_t* W, uint16_t* dx, int T, int N, int K,
                    hipStream_t s, const uint16_t* WT) {
  // dx[T][K] = dy[T][N] . W[N][K]: M = T, N' = K, reduction = N
  if (launch_gemmp_nn(dy, W, dx, nullptr, 0, T, N, K, device_cu_count(), s, nullptr, WT)) return true;
  if (launch_gemm256_nn(dy, W, dx, T, N, K, s)) return true;
  if (!gemm_shape_ok(T, K, N)) return false;
  const int blocks = (T / 128) * (K / 128);
  hipLaunchKernelGGL((gemm_kernel<false, true, EPI_BF16>), dim3(blocks), dim3(256), 0, s,
                     (const bf16_t*)dy, (int64_t)N, (const bf16_t*)W, (int64_t)K, T, K, N, N, 1,
                     (bf16_t*)dx, (int64_t)K, nullptr, nullptr, 0, nullptr, nullptr);
  return true;
}

bool launch_gemm_wgrad(const uint16_t* dy, const uint16_t* x, float* dW, float* db, int T, int N,
                       int K, hipStream_t s, float* ws) {
  // dW[N][K] += dy[T][N]^T . x[T][K]: M = N, N' = K, reduction = T (split over workgroups)
  if (launch_gemm256_wgrad(dy, x, dW, db, T, N, K, s, ws)) return true;
  if (!gemm_shape_ok(N, K, T)) return false;
  const int tiles = (N / 128) * (K / 128);
  int splits = (1024 + tiles - 1) / tiles;
  const int ksteps = T / 64;
  // at least 16 K-steps (1024 tokens) per split: an 8192-token micro-batch of the 128-wide
  // up/down projections otherwise split 128 ways, 128 x the gradient in fp32 atomics
  if (splits > ksteps / 16) splits = ksteps / 16;
  if (splits > ksteps) splits = ksteps;
  if (splits < 1) splits = 1;
  const int kps = ((ksteps + splits - 1) / splits) * 64;
  splits = (T + kps - 1) / kps;
  hipLaunchKernelGGL((gemm_kernel<true, true, EPI_ATOMIC_F32>), dim3(tiles * splits), dim3(256), 0,
                     s, (const bf16_t*)dy, (int64_t)N, (const bf16_t*)x, (int64_t)K, N, K, T, kps,
                     splits, nullptr, (int64_t)K, dW, nullptr, 0, nullptr, db);
  return true;
}

}  // namespace dpa
