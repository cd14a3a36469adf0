// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels.
//
// All kernels in this directory are written for wave64 CDNA4 only: block
// sizes are multiples of 64, cross-lane reductions go across 64 lanes, bf16 is
// moved in 8/16-byte vectors (hipcc does not vectorise scalar bf16 loads).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DPA_WAVE 64

namespace dpa {

typedef uint16_t bf16_t;  // raw bf16 bits in memory
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) short bf16x8;   // MFMA A/B fragment
typedef __attribute__((ext_vector_type(4))) short bf16x4;

__device__ __forceinline__ float bf2f(bf16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}

// Round-to-nearest-even f32 -> bf16 (NaN-preserving) on CDNA4's hardware
// converter: v_cvt_pk_bf16_f32 rounds two floats into one packed dword in a
// single VALU op (the bit-twiddled RNE costs ~6 ops per element, which made the
// activation / LayerNorm epilogues VALU-bound rather than HBM-bound).
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_hw;

__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  const f32x2 v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_hw));
}

__device__ __forceinline__ bf16_t f2bf(float f) {
  return __builtin_bit_cast(bf16_t, (__bf16)f);
}

// ---- device-side base of the in-kernel Philox offsets -----------------------
// Every kernel that draws noise or dropout adds g_rng_base to the offset its launch passes; it
// is 0 in eager runs.  A replayed HIP graph bakes its launches' offsets, so the trainer bumps
// the base once per replay (rng_base_add, a one-thread kernel) and every replay draws fresh
// numbers.  Internal linkage: one copy per translation unit, so each TU that draws numbers
// exports its own rng_base_add_<tu> (DPA_RNG_BASE_EXPORT) and bindings.cpp bumps them all.
static __device__ uint32_t g_rng_base;
static __global__ void rng_base_add_kernel(uint32_t d) {
  if (threadIdx.x == 0) g_rng_base += d;
}
__device__ __forceinline__ uint32_t rng_base() { return g_rng_base; }
#define DPA_RNG_BASE_EXPORT(NAME)                                          \
  void rng_base_add_##NAME(uint32_t d, hipStream_t s) {                    \
    hipLaunchKernelGGL(rng_base_add_kernel, dim3(1), dim3(64), 0, s, d);   \
  }

// ---- wave64 reductions ----------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum for blockDim.x <= 1024; `red` needs blockDim.x/64 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = (threadIdx.x < (unsigned)nw) ? red[threadIdx.x] : 0.f;
  if (wid == 0) r = wave_sum(r);
  if (threadIdx.x == 0) red[0] = r;
  __syncthreads();
  r = red[0];
  __syncthreads();
  return r;
}

// ---- counter-based RNG (Philox-4x32-7-ish) for dropout / noise -------------
// Stateless: (seed, offset, subsequence) -> 4 uniform u32.  Replays inside a
// HIP graph read seed/offset from device memory so every replay advances.
__device__ __forceinline__ void philox4(uint32_t k0, uint32_t k1, uint32_t c0, uint32_t c1,
                                        uint32_t c2, uint32_t c3, uint32_t out[4]) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
    uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += W0; k1 += W1;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

// ---- cheap hashes for dropout bits inside matrix-core and memory-bound loops ---------
// lowbias32: 32-bit avalanche hash (two multiplies).
__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

// One-multiply finaliser for the per-element attention dropout bits (v_mul_lo_u32 is
// quarter rate, so each multiply dropped saves 12 issue cycles per key pair); keep
// rate, neighbour correlations and per-row variance match lowbias32 within noise over
// 1024 x 1024 masks (measured host-side).
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  return x;
}

// Dropout bits of the post-LN sublayers whose residual + dropout run in the producing GEMM's
// epilogue (gemm256.hip EPI 7) and whose LayerNorm backward regenerates them (norm.hip
// drop_hash mode): element (row, col) of the [T, D] branch output keeps iff the 16-bit half
// (col & 1) of pair_hash(row, col) is >= thr16 = round(p * 2^16) - one one-multiply hash per
// column pair instead of a Philox-7 block per 4 columns (the GEMM epilogue cannot afford
// Philox: ~38 VALU cycles per element against a ~170-cycle-per-element tile budget).
__device__ __forceinline__ uint32_t pair_seedmix(uint32_t seed, uint32_t offset) {
  return lowbias32(seed ^ lowbias32(offset * 0xC2B2AE3Du ^ 0x68E31DA4u));
}
__device__ __forceinline__ uint32_t pair_hash(uint32_t seedmix, uint32_t row, uint32_t col) {
  return mix32(seedmix ^ (row * 0x9E3779B1u) ^ ((col >> 1) * 0x85EBCA77u));
}
__device__ __forceinline__ bool pair_keep(uint32_t h, uint32_t col, uint32_t thr16) {
  return ((col & 1u) ? (h >> 16) : (h & 0xffffu)) >= thr16;
}
__host__ __device__ __forceinline__ uint32_t pair_thr16(float p) { return (uint32_t)(p * 65536.f + 0.5f); }

// Attention dropout on a packed bf16 key pair (keys 2k, 2k + 1 of one query = the low and high
// halves of the pair's hash; a half is kept when half >= thr16, unsigned).  With both sides
// offset by 0x8000 the keep test is a signed 16-bit compare, done for both halves at once by a
// saturating packed subtract whose sign, spread by a packed shift, masks the dropped half
// (exact for every thr16).  Three VALU ops per PAIR (the 0x8000 offset rides the hash's last
// xor) replace a compare, a select and a scale multiply per element, and the caller moves the
// 1 / (1 - p) scale to its output normalisation.  The equivalent vector C compiles to per-half
// compares and selects, hence the asm.
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
// drop_hash_t(dc, qt, kt) ^ 0x80008000 from sq = seedmix ^ qt: mix32 with its last two xors
// as one three-input xor
__device__ __forceinline__ uint32_t drop_hash_s(uint32_t sq, uint32_t kt, uint32_t c8000) {
  uint32_t x = sq ^ kt;
  x ^= x >> 16;
  x *= 0x7feb352du;
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(x), "v"(x >> 15), "v"(c8000));
  return r;
}
__device__ __forceinline__ uint32_t drop_pair(uint32_t pk, uint32_t hs, uint32_t ts2, uint32_t c15) {
  // hs = hash ^ 0x80008000, ts2 = (thr16 ^ 0x8000) in both halves, c15 = 15 in both halves
  uint32_t d, msk;
  asm("v_pk_sub_i16 %0, %1, %2 clamp" : "=v"(d) : "v"(hs), "v"(ts2));
  asm("v_pk_ashrrev_i16 %0, %1, %2" : "=v"(msk) : "v"(c15), "v"(d));
  return pk & ~msk;
}

__device__ __forceinline__ float u32_to_unit(uint32_t x) {  // [0,1)
  return (float)(x >> 8) * (1.0f / 16777216.0f);
}

// Raw v_exp_f32 (2^x): no denormal range reduction (the libm exp2f adds a
// compare / select / ldexp around every call); results below 2^-126 flush to 0,
// which is exact enough for softmax / activation math.
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float fexp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }

}  // namespace dpa
