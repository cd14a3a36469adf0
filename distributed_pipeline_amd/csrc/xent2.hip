// Fused linear + cross-entropy, E = 128 (the DiffuSeq rounding head: x[N,128]
// against the tied [V,128] word embedding), second generation:
//
// * W tiles (64 vocabulary rows x 256 B) and their bias stream global -> LDS
//   with global_load_lds (LDS-DMA) into a 2-stage ring: the DMA of tile t+1
//   overlaps the matrix-core / softmax work of tile t; every LDS access is
//   inline asm, so hipcc never drains the in-flight DMA with vmcnt(0).
// * Accumulators start at the bias of their rows (-inf past the vocabulary /
//   split), so the per-logit work is one FMA + exp2 (+ max / add): the
//   softmax of 8e9 logits per call is what bounds this kernel, not the MFMAs.
// * 128 tokens per workgroup (4 waves x 32, token on the MFMA lane: S = W x^T),
//   ~4 workgroups per CU (32.5 KiB LDS, < 128 VGPRs) for latency hiding.
// * The W image uses a 256-B-row XOR swizzle that is conflict-free for both the
//   row reads (A operand of S) and the transposed reads (B operand of dx = dS W),
//   with per-lane base addresses + immediate tile offsets.
//
// fwd : online log-sum-exp over the vocabulary (split over workgroups when the
//       token count alone cannot fill the chip; partial (max, sum) merged by
//       lxent_combine_kernel in xent.hip), target logit picked from registers.
// dx  : dS = g (softmax - onehot) rebuilt per tile, fed from the accumulators as
//       the A operand of dx += dS^T W with W read transposed.
#include <cstdlib>

#include "common.h"
#include "launchers.h"
#include "mfma.h"

namespace dpa {
namespace x2 {

constexpr int E = 128, ROWB = 256, TILE = 64;
constexpr int WIMG = TILE * ROWB;      // 16 KiB
constexpr int STAGE = WIMG + 256;      // + 64 bias dwords (bf16 in the low half)
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void glob_void;

__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) char*)p);
}
template <int IMM>
__device__ __forceinline__ bf16x8 rd128o(uint32_t a) {
  bf16x8 f;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f) : "v"(a), "i"(IMM));
  return f;
}
template <int IMM>
__device__ __forceinline__ bf16x4 rd64o(uint32_t a) {
  bf16x4 f;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(f) : "v"(a), "i"(IMM));
  return f;
}
template <int IMM>
__device__ __forceinline__ bf16x4 rdtro(uint32_t a) {
  bf16x4 f;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(f) : "v"(a), "i"(IMM));
  return f;
}
__device__ __forceinline__ void lgkm0() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// 256-B row image: chunk XOR ((row & 3) << 2) | ((row >> 2) & 3)
__device__ __forceinline__ int fsw(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

// DMA W rows [v0, v0 + 64) (clamped to V - 1) and their bias into a stage.
// Wave w issues pieces 4w..4w+3 (4 rows each); wave 0 also the 64 bias values.
__device__ __forceinline__ void issue_tile(char* st, const bf16_t* __restrict__ W,
                                           const bf16_t* __restrict__ bias, int v0, int V, int w,
                                           int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int pc = w * 4 + i;
    const int r = pc * 4 + (lane >> 4), phys = lane & 15;
    const int v = min(v0 + r, V - 1);
    const bf16_t* src = W + (int64_t)v * E + ((phys ^ fsw(r)) << 3);
    __builtin_amdgcn_global_load_lds((glob_void*)src, (lds_void*)(st + pc * 1024), 16, 0, 0);
  }
  if (w == 0 && bias != nullptr) {
    const bf16_t* src = bias + min(v0 + lane, V - 1);
    __builtin_amdgcn_global_load_lds((glob_void*)src, (lds_void*)(st + WIMG), 2, 0, 0);
  }
}

// Per-lane read bases (relative to a stage), all tile offsets are immediates.
struct Bases {
  uint32_t rowr[8];       // A-operand row read: W row (lane & 31), chunk 2s + h, s = 0..7
  uint32_t tr1[4], tr2[4];  // transposed (permuted k) read of W for dx column tile kt
  uint32_t bias;          // bias of rows 8g + 4h .. (+ 32 vt + 8 g)
};

__device__ __forceinline__ Bases make_bases(int lane) {
  Bases B;
  const int h = lane >> 5, r = lane & 31;
  // rows (lane & 31) + 32 vt: fsw depends on row bits 0..3 only -> vt is an immediate
#pragma unroll
  for (int s = 0; s < 8; ++s) B.rowr[s] = (uint32_t)(r * ROWB + (((2 * s + h) ^ fsw(r)) << 4));
  // transposed: rows r0 + 4h + q (+8), r0 = 32 vt + 16 s (multiple of 16):
  // fsw(row) = (q << 2) | h, fsw(row + 8) = (q << 2) | (h + 2); column chunk 4 kt + c'
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int cp = 2 * (g & 1) + (p >> 1), e = (p & 1) * 8;
#pragma unroll
  for (int kt = 0; kt < 4; ++kt) {
    B.tr1[kt] = (uint32_t)((4 * h + q) * ROWB + (((4 * kt + cp) ^ ((q << 2) | h)) << 4) + e);
    B.tr2[kt] = (uint32_t)((4 * h + q + 8) * ROWB + (((4 * kt + cp) ^ ((q << 2) | (h + 2))) << 4) + e);
  }
  B.bias = (uint32_t)(WIMG + (4 * h) * 4);
  return B;
}

// acc = bias of rows vt*32 + acc_row(i, h).  Sub-dword LDS-DMA writes one dword
// per lane (zero-extended, probed on gfx950: tools/probes/glds_width.hip), so
// row r's bf16 bias sits in the low half of dword r; -inf patched past the split.
template <int IMM>
__device__ __forceinline__ uint4 rd128u(uint32_t a) {
  uint4 f;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f) : "v"(a), "i"(IMM));
  return f;
}
template <int VT>
__device__ __forceinline__ void init_bias(f32x16& acc, uint32_t st, const Bases& B, bool has_bias) {
  if (!has_bias) {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    return;
  }
  uint4 b4[4];
  b4[0] = rd128u<VT * 128 + 0>(st + B.bias);
  b4[1] = rd128u<VT * 128 + 32>(st + B.bias);
  b4[2] = rd128u<VT * 128 + 64>(st + B.bias);
  b4[3] = rd128u<VT * 128 + 96>(st + B.bias);
  lgkm0();
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    acc[4 * g + 0] = __uint_as_float(b4[g].x << 16);
    acc[4 * g + 1] = __uint_as_float(b4[g].y << 16);
    acc[4 * g + 2] = __uint_as_float(b4[g].z << 16);
    acc[4 * g + 3] = __uint_as_float(b4[g].w << 16);
  }
}

// S^T tile: acc[i] (+)= sum_k W[vt*32 + row(i)][k] x[token][k]
template <int VT>
__device__ __forceinline__ void logits(f32x16& acc, uint32_t st, const Bases& B,
                                       const bf16x8 (&xf)[8]) {
  bf16x8 a[8];
  a[0] = rd128o<VT * 32 * ROWB>(st + B.rowr[0]);
  a[1] = rd128o<VT * 32 * ROWB>(st + B.rowr[1]);
  a[2] = rd128o<VT * 32 * ROWB>(st + B.rowr[2]);
  a[3] = rd128o<VT * 32 * ROWB>(st + B.rowr[3]);
  a[4] = rd128o<VT * 32 * ROWB>(st + B.rowr[4]);
  a[5] = rd128o<VT * 32 * ROWB>(st + B.rowr[5]);
  a[6] = rd128o<VT * 32 * ROWB>(st + B.rowr[6]);
  a[7] = rd128o<VT * 32 * ROWB>(st + B.rowr[7]);
  lgkm0();
#pragma unroll
  for (int s = 0; s < 8; ++s) acc = mfma32(a[s], xf[s], acc);
}

// Past-the-split rows of the last tile: bias -> -inf (their softmax is 0).
// (Without a bias the in-range rows get 0: nothing was DMA'd for them.)
__device__ __forceinline__ void patch_tail(char* st, int v0, int vend, int tid, bool has_bias) {
  if (tid < TILE && (v0 + tid >= vend || !has_bias)) {
    const uint32_t a = lds_u32(st + WIMG + tid * 4);
    const uint32_t val = (v0 + tid >= vend) ? 0xff80u : 0u;  // bf16 -inf / 0 (low half)
    asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(val) : "memory");
  }
}

// Make values loaded before the DMA loop opaque to hipcc's wait-count pass, so
// it does not re-drain the in-flight LDS-DMA (vmcnt(0)) before their uses.
template <typename T>
__device__ __forceinline__ void launder(T& v) {
  asm volatile("" : "+v"(v));
}

__device__ __forceinline__ float sel16(const f32x16& a, int i) {
  float v = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) v = (k == i) ? a[k] : v;
  return v;
}

// ============================================================================
__global__ void __launch_bounds__(256) lxent2_fwd_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ W, const bf16_t* __restrict__ bias,
    const int64_t* __restrict__ target, int N, int V, int v_per_split, float* __restrict__ loss,
    float* __restrict__ lse_out, float* __restrict__ part_m, float* __restrict__ part_s,
    float* __restrict__ tgt_logit) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
  const int t = blockIdx.x * 128 + w * 32 + (lane & 31);
  const bool tok_ok = t < N;
  bf16x8 xf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    if (tok_ok) xf[s] = ld_frag(x + (int64_t)t * E + 16 * s + 8 * h);
    else for (int j = 0; j < 8; ++j) xf[s][j] = 0;
  }
  int64_t tg = tok_ok ? target[t] : -1;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int s = 0; s < 8; ++s) launder(xf[s]);
  launder(tg);
  const int vbeg = blockIdx.y * v_per_split;
  const int vend = min(V, vbeg + v_per_split);
  const int ntiles = (vend - vbeg + TILE - 1) / TILE;
  const bool has_bias = bias != nullptr;
  const Bases B = make_bases(lane);
  const uint32_t sb = lds_u32(smem);
  float m = -1e30f, ssum = 0.f, tl = -INFINITY;

  if (ntiles > 0) issue_tile(smem, W, bias, vbeg, V, w, lane);
  for (int it = 0; it < ntiles; ++it) {
    const int v0 = vbeg + it * TILE;
    char* stp = smem + (it & 1) * STAGE;
    const uint32_t st = sb + (it & 1) * STAGE;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();
    if (it + 1 < ntiles) issue_tile(smem + ((it + 1) & 1) * STAGE, W, bias, v0 + TILE, V, w, lane);
    if (v0 + TILE > vend) {  // last, partial tile (uniform)
      patch_tail(stp, v0, vend, tid, has_bias);
      barrier();
    }
    f32x16 acc[2];
    init_bias<0>(acc[0], st, B, has_bias || v0 + TILE > vend);
    init_bias<1>(acc[1], st, B, has_bias || v0 + TILE > vend);
    logits<0>(acc[0], st, B, xf);
    logits<1>(acc[1], st, B, xf);
    float tmax = fmaxf(acc[0][0], acc[1][0]);
#pragma unroll
    for (int i = 1; i < 16; ++i) tmax = fmaxf(tmax, fmaxf(acc[0][i], acc[1][i]));
    const float mn = fmaxf(m, tmax * LOG2E);
    float add = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      add += fexp2(fmaf(acc[0][i], LOG2E, -mn)) + fexp2(fmaf(acc[1][i], LOG2E, -mn));
    ssum = ssum * fexp2(m - mn) + add;
    m = mn;
    const int64_t r = tg - v0;
    if (r >= 0 && r < TILE && tg < vend) {
      const int rr = (int)r & 31;
      if (((rr >> 2) & 1) == h) {
        const int i = (rr & 3) + 4 * (rr >> 3);
        tl = (r >> 5) ? sel16(acc[1], i) : sel16(acc[0], i);
      }
    }
  }
  const float m2 = __shfl_xor(m, 32, 64), s2 = __shfl_xor(ssum, 32, 64);
  const float tl2 = __shfl_xor(tl, 32, 64);
  const float M = fmaxf(m, m2);
  const float S = ssum * fexp2(m - M) + s2 * fexp2(m2 - M);
  tl = fmaxf(tl, tl2);
  if (h == 0 && tok_ok) {
    if (gridDim.y == 1) {
      const bool valid = tg >= 0 && tg < V;
      const float lse = (M + log2f(S)) * LN2;
      loss[t] = valid ? lse - tl : 0.f;
      lse_out[t] = lse;
    } else {
      part_m[(int64_t)blockIdx.y * N + t] = M;
      part_s[(int64_t)blockIdx.y * N + t] = S;
      if (tl > -INFINITY) tgt_logit[t] = tl;
    }
  }
}

// dx[t][k] += sum_v dS[v][t] W[v][k] for one 32-row vocabulary tile
template <int VT>
__device__ __forceinline__ void dx_accum(f32x16 (&dacc)[4], const f32x16& ds, uint32_t st,
                                         const Bases& B) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const bf16x8 af = acc_to_frag(ds, s);
    bf16x8 bw[4];
    // rows VT*32 + 16 s + 4h + q (+8), columns 32 kt + 16 (g&1) + 4p: immediates
    switch (s) {
      case 0:
        bw[0] = cat44(rdtro<(VT * 32) * ROWB>(st + B.tr1[0]), rdtro<(VT * 32) * ROWB>(st + B.tr2[0]));
        bw[1] = cat44(rdtro<(VT * 32) * ROWB>(st + B.tr1[1]), rdtro<(VT * 32) * ROWB>(st + B.tr2[1]));
        bw[2] = cat44(rdtro<(VT * 32) * ROWB>(st + B.tr1[2]), rdtro<(VT * 32) * ROWB>(st + B.tr2[2]));
        bw[3] = cat44(rdtro<(VT * 32) * ROWB>(st + B.tr1[3]), rdtro<(VT * 32) * ROWB>(st + B.tr2[3]));
        break;
      default:
        bw[0] = cat44(rdtro<(VT * 32 + 16) * ROWB>(st + B.tr1[0]), rdtro<(VT * 32 + 16) * ROWB>(st + B.tr2[0]));
        bw[1] = cat44(rdtro<(VT * 32 + 16) * ROWB>(st + B.tr1[1]), rdtro<(VT * 32 + 16) * ROWB>(st + B.tr2[1]));
        bw[2] = cat44(rdtro<(VT * 32 + 16) * ROWB>(st + B.tr1[2]), rdtro<(VT * 32 + 16) * ROWB>(st + B.tr2[2]));
        bw[3] = cat44(rdtro<(VT * 32 + 16) * ROWB>(st + B.tr1[3]), rdtro<(VT * 32 + 16) * ROWB>(st + B.tr2[3]));
        break;
    }
    lgkm0();
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) dacc[kt] = mfma32(af, bw[kt], dacc[kt]);
  }
}

template <int VT>
__device__ __forceinline__ void dx_tile(f32x16 (&dacc)[4], uint32_t st, const Bases& B,
                                        const bf16x8 (&xf)[8], bool bias_init, float g, float lse2,
                                        int64_t tg, int v0, int vend, int h) {
  f32x16 acc;
  init_bias<VT>(acc, st, B, bias_init);
  logits<VT>(acc, st, B, xf);
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = g * fexp2(fmaf(acc[i], LOG2E, -lse2));
  const int64_t rt = tg - (v0 + VT * 32);
  if (rt >= 0 && rt < 32 && tg < vend && ((rt >> 2) & 1) == h) {
    const int itg = ((int)rt & 3) + 4 * ((int)rt >> 3);
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] -= (i == itg) ? g : 0.f;
  }
  dx_accum<VT>(dacc, acc, st, B);
}

__global__ void __launch_bounds__(256) lxent2_dx_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ W, const bf16_t* __restrict__ bias,
    const int64_t* __restrict__ target, const float* __restrict__ lse, const float* __restrict__ dloss,
    int N, int V, int v_per_split, bf16_t* __restrict__ dx, float* __restrict__ dx_acc) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
  const int t = blockIdx.x * 128 + w * 32 + (lane & 31);
  const bool tok_ok = t < N;
  bf16x8 xf[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    if (tok_ok) xf[s] = ld_frag(x + (int64_t)t * E + 16 * s + 8 * h);
    else for (int j = 0; j < 8; ++j) xf[s][j] = 0;
  }
  int64_t tg = tok_ok ? target[t] : -1;
  const bool valid = tok_ok && tg >= 0 && tg < V;
  float g = valid ? dloss[t] : 0.f;
  float lse2 = tok_ok ? lse[t] * LOG2E : 0.f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int s = 0; s < 8; ++s) launder(xf[s]);
  launder(tg);
  launder(g);
  launder(lse2);
  const int vbeg = blockIdx.y * v_per_split;
  const int vend = min(V, vbeg + v_per_split);
  const int ntiles = (vend - vbeg + TILE - 1) / TILE;
  const bool has_bias = bias != nullptr;
  const Bases B = make_bases(lane);
  const uint32_t sb = lds_u32(smem);
  f32x16 dacc[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) dacc[k] = zero16();

  if (ntiles > 0) issue_tile(smem, W, bias, vbeg, V, w, lane);
  for (int it = 0; it < ntiles; ++it) {
    const int v0 = vbeg + it * TILE;
    char* stp = smem + (it & 1) * STAGE;
    const uint32_t st = sb + (it & 1) * STAGE;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();
    if (it + 1 < ntiles) issue_tile(smem + ((it + 1) & 1) * STAGE, W, bias, v0 + TILE, V, w, lane);
    const bool tail = v0 + TILE > vend;
    if (tail) {
      patch_tail(stp, v0, vend, tid, has_bias);
      barrier();
    }
    dx_tile<0>(dacc, st, B, xf, has_bias || tail, g, lse2, tg, v0, vend, h);
    dx_tile<1>(dacc, st, B, xf, has_bias || tail, g, lse2, tg, v0, vend, h);
  }
  // dacc[kt] reg i: row = token (w*32 + acc_row(i,h)), col = k (kt*32 + lane&31)
  const int tb = blockIdx.x * 128 + w * 32;
#pragma unroll
  for (int kt = 0; kt < 4; ++kt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int tt = tb + acc_row(i, h);
      if (tt < N) {
        const int64_t o = (int64_t)tt * E + kt * 32 + (lane & 31);
        if (dx_acc) atomicAdd(dx_acc + o, dacc[kt][i]);
        else dx[o] = f2bf(dacc[kt][i]);
      }
    }
}

}  // namespace x2

// Used by xent.hip for E == 128; returns false when not applicable.
static bool xent2_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("DPA_XENT2");
    return e && e[0] == '1';  // opt-in: v1 (xent.hip) measured faster on fwd
  }();
  return on;
}

bool launch_lxent2_fwd(const uint16_t* x, const uint16_t* W, const uint16_t* b, const int64_t* tgt,
                       int N, int V, int E, int splits, int vps, float* loss, float* lse,
                       float* part_m, float* part_s, float* tgt_logit, hipStream_t s) {
  if (E != x2::E || !xent2_enabled()) return false;
  hipLaunchKernelGGL(x2::lxent2_fwd_kernel, dim3((N + 127) / 128, splits), dim3(256), 0, s,
                     (const bf16_t*)x, (const bf16_t*)W, (const bf16_t*)b, tgt, N, V, vps, loss,
                     lse, part_m, part_s, tgt_logit);
  return true;
}

bool launch_lxent2_dx(const uint16_t* x, const uint16_t* W, const uint16_t* b, const int64_t* tgt,
                      const float* lse, const float* dloss, int N, int V, int E, int splits, int vps,
                      uint16_t* dx, float* dx_acc, hipStream_t s) {
  if (E != x2::E || !xent2_enabled()) return false;
  hipLaunchKernelGGL(x2::lxent2_dx_kernel, dim3((N + 127) / 128, splits), dim3(256), 0, s,
                     (const bf16_t*)x, (const bf16_t*)W, (const bf16_t*)b, tgt, lse, dloss, N, V,
                     vps, (bf16_t*)dx, dx_acc);
  return true;
}

}  // namespace dpa
