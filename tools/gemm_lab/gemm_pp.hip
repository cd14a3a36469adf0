// Ping-pong persistent bf16 GEMM for gfx950: two wave groups on two different output
// tiles, so one group's epilogue (bias / activation math, LDS transpose, stores) runs
// under the other group's MFMAs instead of stalling the matrix cores.
//
// Why (profiles/gemm_lab_r2*.txt): the 256 x 256 persistent kernel (gemm256.hip) runs
// its main loop at ~1.35 PFLOP/s, but every workgroup's 8 waves reach the epilogue
// together, so the epilogue is fully exposed - 18 % of a K = 768 GEMM with a plain
// bias epilogue, ~40 % with GELU + GELU' (0.28 ms of erf/exp VALU per call, no MFMA in
// flight).  Keeping the next tile's accumulators live while draining the previous
// tile would need 64 more VGPRs than the 256 a 2-waves/SIMD kernel has.
//
// Structure (512 threads, one workgroup per CU):
// * group g = waves 4g..4g+3 owns a 256 x 128 output tile (2 x 2 waves, 128 x 64 each,
//   16x16x32 MFMAs, C^T in the accumulators = the register-direct epilogue layout of
//   gemm256's persistent kernel).  Waves w and w+4 share a SIMD.
// * BK = 32, a 3-deep LDS ring per group (3 x 24 KiB x 2 groups = 144 KiB) filled by
//   buffer_load ... lds (6 x 1 KiB per wave per step); the prefetch runs 2 steps ahead
//   and continues across tiles (the next tile's first 2 steps are staged during the
//   current tile's last 2 steps, so they land under the epilogue).
// * Lock-step slots: every slot is [A] barrier [B] barrier for all 8 waves, group 1 one
//   barrier behind group 0, so group 0's [B] (its 32 MFMAs) coincides with group 1's [A]
//   and vice versa.  A main-loop slot is [A] = DMA issue + fragment reads + counted
//   vmcnt, [B] = MFMAs.  An epilogue slot puts one epilogue unit in [A] (under the other
//   group's MFMAs) and nothing in [B].
// * Group 1 starts half a period (main + epilogue slots of one tile) late, so the two
//   groups' epilogues alternate instead of coinciding; both groups execute the same
//   number of slots (idle slots at the start / end), so the barriers always pair up.
// * LDS images: A [256 rows][32 k] and row-form B [128 n][32 k] have 64-byte rows, the
//   16-byte chunk index XOR-ed with f(row) = {0,2,3,1}[(row >> 2) & 3] (conflict-free for
//   the ds_read_b128 lane groups of a 16 x 32 fragment); transposed B [32 k][128 n]
//   (data-gradient GEMMs) uses gemm256's 256-byte-row XOR and ds_read_b64_tr_b16.
//
// Epilogues (EPI): 0 bf16 (+bias); 6 y = act(x + bias) and d = act'(x + bias), both
// stored (GELU forward that hands its derivative to the backward); -1 none (timing
// probe of the main loop).
#include <type_traits>

#include "act.h"
#include "common.h"
#include "launchers.h"
#include "mfma.h"

namespace dpa {
namespace pp {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_v;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4_v;

constexpr int BK = 32;
constexpr int A_IMG = 256 * BK * 2;          // 16 KiB
constexpr int B_IMG = 128 * BK * 2;          // 8 KiB
constexpr int STAGE = A_IMG + B_IMG;         // 24 KiB
constexpr int RING = 3;
constexpr int GROUP_LDS = RING * STAGE;      // 72 KiB
constexpr int STG_OFF = 2 * GROUP_LDS;       // 8 waves x 2 KiB epilogue transpose slots
constexpr int LDS_BYTES = STG_OFF + 8 * 2048;  // 160 KiB

// compile-time loop: f(std::integral_constant<int, U>) for U = I .. E-1
template <int I, int E>
struct Unroll {
  template <class F>
  __device__ __forceinline__ static void run(F&& f) {
    f(std::integral_constant<int, I>{});
    Unroll<I + 1, E>::run(f);
  }
};
template <int E>
struct Unroll<E, E> {
  template <class F>
  __device__ __forceinline__ static void run(F&&) {}
};

template <int EPI>
struct Epi {
  // epilogue units (one per slot) and the VMEM ops they issue after the next tile's
  // prefetched steps (bias loads + stores)
  static constexpr int E = EPI == 6 ? 16 : EPI == 0 ? 8 : 1;
  static constexpr int XS = EPI == 6 ? 36 : EPI == 0 ? 20 : 0;
};

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_v, a),
                                                 __builtin_bit_cast(bf16x8_v, b), c, 0, 0, 0);
}
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) char*)p);
}
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }
template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory"); }
__device__ __forceinline__ int lane_id() {
  return (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ int opaque(int x) {
  int y;
  asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
  return y;
}
// 64-byte-row image: chunk XOR of row r
__device__ __forceinline__ int f64(int r) { return (0x1320 >> (((r >> 2) & 3) * 4)) & 3; }
// 256-byte-row transposed image: chunk XOR of k-row r (gemm256 tr_x)
__device__ __forceinline__ int tr_x(int r) { return ((r & 3) << 1) | (((r >> 3) & 1) << 3); }

__device__ __forceinline__ void lds_write_b128(uint32_t addr, const uint4& v) {
  const u32x4_v x = {v.x, v.y, v.z, v.w};
  asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(x) : "memory");
}
__device__ __forceinline__ uint4 lds_read_b128_sync(uint32_t addr) {
  u32x4_v v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  return make_uint4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

template <int ACT>
__device__ __forceinline__ uint4 act_dact8(const uint4& u, uint4& dv) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
  uint32_t o[4], g[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f32x2 d;
    const f32x2 y = act_dact2<ACT>(f32x2{bf_lo(w[q]), bf_hi(w[q])}, d);
    o[q] = pack_bf2(y.x, y.y);
    g[q] = pack_bf2(d.x, d.y);
  }
  dv = make_uint4(g[0], g[1], g[2], g[3]);
  return make_uint4(o[0], o[1], o[2], o[3]);
}

template <bool B_TR, int EPI, int ACT>
__global__ void __launch_bounds__(512) gemm_pp_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                      const bf16_t* __restrict__ B, int64_t ldb, int M, int N,
                                                      int K, bf16_t* __restrict__ C, int64_t ldc,
                                                      const bf16_t* __restrict__ bias, bf16_t* __restrict__ Z) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  constexpr int E = Epi<EPI>::E, XS = Epi<EPI>::XS;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = w >> 2, q = w & 3;
  const int wm = q >> 1, wn = q & 1;
  const int NT = N / 128, ntiles = (M / 256) * NT;
  const int G = gridDim.x;
  const int KS = K / BK;
  const int P = KS + E;
  const uint32_t sbase = lds_u32(smem);
  char* const ring = smem + grp * GROUP_LDS;
  const uint32_t ring_u = sbase + grp * GROUP_LDS;

  // tiles of this workgroup: first + G i; group g takes i = g, g + 2, ...
  const int first = xcd_remap(blockIdx.x, G);
  const int ntot = first < ntiles ? (ntiles - first + G - 1) / G : 0;
  const int n_mine = (ntot + 1 - grp) / 2;
  const int off = P / 2;
  const int total = max(((ntot + 1) / 2) * P, off + (ntot / 2) * P);
  const int my_start = grp ? off : 0;

  // ---- per-lane DMA offsets (bytes from the tile / k-step origin) and read bases ----
  uint32_t offA[4], offB[2];
  {
    const int lane = lane_id();
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int r = (q * 4 + t) * 16 + (lane >> 2);
      offA[t] = (uint32_t)(r * (int)lda + (((lane & 3) ^ f64(r)) << 3)) * 2u;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if constexpr (B_TR) {
        const int kr = (q * 2 + t) * 4 + (lane >> 4);
        offB[t] = (uint32_t)(kr * (int)ldb + (((lane & 15) ^ tr_x(kr)) << 3)) * 2u;
      } else {
        const int r = (q * 2 + t) * 16 + (lane >> 2);
        offB[t] = (uint32_t)(r * (int)ldb + (((lane & 3) ^ f64(r)) << 3)) * 2u;
      }
    }
  }

  auto stage = [&](int t, int ks, int slot) {
    const int mt = t / NT, nt = t % NT;
    char* img = ring + slot * STAGE;
    const bf16_t* a0 = A + (int64_t)mt * 256 * lda + ks * BK;
    const auto ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(a0), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int t4 = 0; t4 < 4; ++t4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(img + (q * 4 + t4) * 1024), 16, offA[t4], 0, 0, 0);
    const bf16_t* b0 = B_TR ? B + (int64_t)ks * BK * ldb + nt * 128 : B + (int64_t)nt * 128 * ldb + ks * BK;
    const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(b0), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int t2 = 0; t2 < 2; ++t2)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(img + A_IMG + (q * 2 + t2) * 1024), 16, offB[t2], 0,
                                               0, 0);
  };

  f32x4 acc[8][4];
  bf16x8 fa[8], fb[4];

  // prologue: both groups stage steps 0 and 1 of their first tile
  if (n_mine > 0) {
    const int t0 = first + G * grp;
    stage(t0, 0, 0);
    stage(t0, 1, 1);
    wait_vm<6>();
  }
  barrier();
  if (grp == 1) barrier();  // group 1 runs one barrier behind group 0
  for (int s = 0; s < my_start; ++s) {
    barrier();
    barrier();
  }

  int slot = 0;  // ring slot of the current step
  for (int it = 0; it < n_mine; ++it) {
    const int t = first + G * (2 * it + grp);
    const int tn = first + G * (2 * it + 2 + grp);
    const bool has_next = it + 1 < n_mine;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int j = 0; j < KS; ++j) {
      // [A] prefetch step +2 (this tile or the next), fragment reads, counted wait
      const int ps = slot == 0 ? 2 : slot - 1;  // (slot + 2) % 3
      bool pf = true;
      if (j + 2 < KS) stage(t, j + 2, ps);
      else if (has_next) stage(tn, j + 2 - KS, ps);
      else pf = false;
      {
        const int lane = lane_id();
        const int li = lane & 15, g4 = lane >> 4;
        const uint32_t sl = ring_u + slot * STAGE;
        const uint32_t ra = sl + (uint32_t)((wm * 128 + li) * 64 + ((g4 ^ f64(li)) << 4));
#pragma unroll
        for (int i = 0; i < 8; ++i)
          asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fa[i]) : "v"(ra), "i"(i * 1024));
        if constexpr (B_TR) {
          const int qq = li >> 2, pp = li & 3;
          const int x = (qq << 1) | ((g4 & 1) << 3);
#pragma unroll
          for (int jb = 0; jb < 4; ++jb) {
            const int cb = wn * 64 + jb * 16;
            const int ch = ((cb >> 3) + (pp >> 1)) ^ x;
            const uint32_t rb = sl + A_IMG + (uint32_t)((8 * g4 + qq) * 256 + ch * 16 + (pp & 1) * 8);
            bf16x4 lo, hi;
            asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(rb));
            asm volatile("ds_read_b64_tr_b16 %0, %1 offset:1024" : "=v"(hi) : "v"(rb));
            fb[jb] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          }
        } else {
          const uint32_t rb = sl + A_IMG + (uint32_t)((wn * 64 + li) * 64 + ((g4 ^ f64(li)) << 4));
#pragma unroll
          for (int jb = 0; jb < 4; ++jb)
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(fb[jb]) : "v"(rb), "i"(jb * 1024));
        }
      }
      // retire the DMA of step +1 (read next slot); at the first step of a later tile the
      // previous epilogue's XS ops were issued after it as well
      if (j == 0 && it > 0) wait_vm<6 + XS>();
      else if (pf) wait_vm<6>();
      else wait_vm<0>();
      barrier();
      // [B] 32 MFMAs
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) acc[i][jb] = mfma16(fb[jb], fa[i], acc[i][jb]);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      barrier();
      slot = slot == 2 ? 0 : slot + 1;
    }

    // ---- epilogue: E units, one per slot, in [A] (under the other group's MFMAs) ----
    const int mt = t / NT, nt = t % NT;
    const int64_t row0 = (int64_t)mt * 256 + wm * 128;
    const int col0 = nt * 128 + wn * 64;
    float bv[4][4];
    uint4 val1 = make_uint4(0, 0, 0, 0);
    Unroll<0, E>::run([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      if constexpr (EPI < 0) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int jb = 0; jb < 4; ++jb) asm volatile("" ::"v"(acc[i][jb]));
      } else {
        const int ln = opaque(lane_id());
        const int R = ln >> 4, li = ln & 15;
        const int cofs = ((R & 1) << 4) | ((R >> 1) << 3);
        const uint32_t stg = sbase + STG_OFF + w * 2048;
        const int rr = ln >> 3, ch = ln & 7;
        if constexpr (u == 0) {
#pragma unroll
          for (int jb = 0; jb < 4; ++jb) {
            if (bias) {
              const uint2 b2 = *reinterpret_cast<const uint2*>(bias + col0 + jb * 16 + 4 * R);
              bv[jb][0] = bf_lo(b2.x); bv[jb][1] = bf_hi(b2.x);
              bv[jb][2] = bf_lo(b2.y); bv[jb][3] = bf_hi(b2.y);
            } else {
              bv[jb][0] = bv[jb][1] = bv[jb][2] = bv[jb][3] = 0.f;
            }
          }
          wait_vm<0>();
        }
        constexpr int ro = EPI == 6 ? u / 2 : u;
        constexpr bool first_part = EPI == 6 ? (u % 2) == 0 : true;
        auto store_off = [&](int k) -> int64_t {
          return (row0 + ro * 16 + k * 8 + rr) * ldc + col0 + ch * 8;
        };
        if constexpr (first_part) {
          // stage the round's 16 rows x 64 columns (+bias) through the wave's LDS slot
#pragma unroll
          for (int qb = 0; qb < 2; ++qb) {
            float v[2][4];
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
              for (int r = 0; r < 4; ++r) v[j][r] = acc[ro][qb * 2 + j][r] + bv[qb * 2 + j][r];
            const uint32_t x0 = pack_bf2(v[0][0], v[0][1]), x1 = pack_bf2(v[0][2], v[0][3]);
            const uint32_t y0 = pack_bf2(v[1][0], v[1][1]), y1 = pack_bf2(v[1][2], v[1][3]);
            const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
            const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
            const int lchunk = qb * 4 + (cofs >> 3);
            lds_write_b128(stg + li * 128 + ((lchunk ^ (li & 7)) << 4), make_uint4(s0[0], s1[0], s0[1], s1[1]));
          }
          uint4 val[2];
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const int row = k * 8 + rr;
            val[k] = lds_read_b128_sync(stg + row * 128 + ((ch ^ (row & 7)) << 4));
          }
          if constexpr (EPI == 0) {
#pragma unroll
            for (int k = 0; k < 2; ++k) *reinterpret_cast<uint4*>(C + store_off(k)) = val[k];
          } else {
            uint4 dv;
            const uint4 y = act_dact8<ACT>(val[0], dv);
            *reinterpret_cast<uint4*>(Z + store_off(0)) = dv;
            *reinterpret_cast<uint4*>(C + store_off(0)) = y;
            val1 = val[1];
          }
        } else {
          uint4 dv;
          const uint4 y = act_dact8<ACT>(val1, dv);
          *reinterpret_cast<uint4*>(Z + store_off(1)) = dv;
          *reinterpret_cast<uint4*>(C + store_off(1)) = y;
        }
      }
      barrier();
      barrier();
    });
  }
  // idle slots until the later group is done, then re-align the two groups
  for (int s = my_start + n_mine * P; s < total; ++s) {
    barrier();
    barrier();
  }
  if (grp == 0) barrier();
  wait_vm<0>();
}

}  // namespace pp

// y[T][N] = x[T][K] . W[N][K]^T (+bias) on the ping-pong kernel; act != 0 (with z): y =
// act(x W^T + b), z = act'(x W^T + b).  False when the shape is not covered.
bool launch_gemm_pp_nt(const uint16_t* x, const uint16_t* W, const uint16_t* bias, uint16_t* y, uint16_t* z,
                       int T, int N, int K, int act, int ncu, hipStream_t s, int epi_override) {
  if (T % 256 || N % 128 || K % (2 * pp::BK) || K < 4 * pp::BK) return false;
  const int tiles = (T / 256) * (N / 128);
  int grid = (tiles + 1) / 2;
  if (grid > ncu) grid = ncu;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, s, (const bf16_t*)x, (int64_t)K, (const bf16_t*)W,
                       (int64_t)K, T, N, K, (bf16_t*)y, (int64_t)N, (const bf16_t*)bias, (bf16_t*)z);
  };
  if (epi_override < 0) go(pp::gemm_pp_kernel<false, -1, 0>);
  else if (act == 0) go(pp::gemm_pp_kernel<false, 0, 0>);
  else if (act == 1 && z) go(pp::gemm_pp_kernel<false, 6, 1>);
  else return false;
  return true;
}

// dx[T][K] = dy[T][N] . W[N][K] on the ping-pong kernel (B transposed images).
bool launch_gemm_pp_nn(const uint16_t* dy, const uint16_t* W, uint16_t* dx, int T, int N, int K, int ncu,
                       hipStream_t s, int epi_override) {
  if (T % 256 || K % 128 || N % (2 * pp::BK) || N < 4 * pp::BK) return false;
  const int tiles = (T / 256) * (K / 128);
  int grid = (tiles + 1) / 2;
  if (grid > ncu) grid = ncu;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(512), 0, s, (const bf16_t*)dy, (int64_t)N, (const bf16_t*)W,
                       (int64_t)K, T, K, N, (bf16_t*)dx, (int64_t)K, (const bf16_t*)nullptr, (bf16_t*)nullptr);
  };
  if (epi_override < 0) go(pp::gemm_pp_kernel<true, -1, 0>);
  else go(pp::gemm_pp_kernel<true, 0, 0>);
  return true;
}

}  // namespace dpa
