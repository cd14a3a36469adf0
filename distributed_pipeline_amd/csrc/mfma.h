// CDNA4 (gfx950) matrix-core helpers: bf16 MFMA 32x32x16 with fp32 accumulate,
// fragment loaders and the LDS transposed read.
//
// v_mfma_f32_32x32x16_bf16 lane maps (lane l, r = l & 31, h = l >> 5):
//   A (32 x 16):  lane l holds A[row r][k = 8h + j], j = 0..7   (8 bf16, 4 VGPRs)
//   B (16 x 32):  lane l holds B[k = 8h + j][col r]
//   C/D (32x32):  reg i (0..15) of lane l is C[row (i&3) + 8*(i>>2) + 4h][col r]
//
// "Accumulator as the next operand": a C tile X (rows in registers, column on
// the lane) converted pairwise to bf16 is directly the A operand of Z = X^T*B
// (k-step s uses registers 8s..8s+7), with the k order permuted: element j of
// lane half h is row 16s + 8(j>>2) + 4h + (j&3) of X - the B operand must be
// loaded in that same k order (see tr_rows_for_acc_operand below).
#pragma once
#include "common.h"

namespace dpa {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a),
                                                 __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// Row index (within the 32x32 tile) of accumulator register i for lane half h.
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// Pack accumulator registers 8s..8s+7 (scaled) to a bf16x8 A/B fragment.
__device__ __forceinline__ bf16x8 acc_to_frag(const f32x16& c, int s) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (short)f2bf(c[8 * s + j]);
  return f;
}

// 16-byte global load as a fragment (8 bf16).
__device__ __forceinline__ bf16x8 ld_frag(const bf16_t* p) {
  return *reinterpret_cast<const bf16x8*>(p);
}

// XOR applied to the 16-byte chunk index of row `row` in rows of >= 256 bytes (a bank
// period).  Both read shapes on these tiles are conflict-free with it
// (MI355X_MICROARCH LDS banking table):
//  * ds_read_b128 of 32 consecutive rows at one chunk - lane groups {0-3,12-15,20-27}
//    and {4-11,16-19,28-31} each get 16 distinct chunk positions;
//  * ds_read_b64_tr_b16 (lds_tr_frag*): a 32-lane group reads rows 4m..4m+3 at 4 chunk
//    offsets x 2 halves: (row & 3) in the high two bits keeps the 32 8-byte slots apart.
// The previous XOR (row & 15) left the transposed reads 4-way conflicted
// (PMC r2: 3.0 conflict cycles per LDS instruction in lxent_fwd_dx).
// LEG selects the previous XOR (row & 15): same-box A/B (round 2) had the fused CE
// forward+dx and dx kernels 6-8% faster with the new XOR but lxent_dw 8% slower, so the dW
// kernel's x tile keeps it.
template <bool LEG = false>
__host__ __device__ __forceinline__ constexpr int swz_x256(int row) {
  return LEG ? (row & 15) : (((row & 3) << 2) | ((row >> 2) & 3));
}

// LDS byte offset of 16-byte chunk `ch` of row `row` for a [rows][ROWBYTES]
// bf16 tile with XOR swizzle (conflict-free ds_read_b128 row reads and 8-byte
// transposed reads).  ROWBYTES is 64, 128 or a multiple of 256.
template <int ROWBYTES, bool LEG = false>
__device__ __forceinline__ int swz(int row, int ch) {
  if constexpr (ROWBYTES == 64) {
    return row * 64 + ((ch ^ ((row >> 2) & 3)) << 4);
  } else if constexpr (ROWBYTES == 128) {
    return row * 128 + ((ch ^ ((row >> 1) & 7)) << 4);
  } else {
    static_assert(ROWBYTES % 256 == 0, "row must be 64, 128 or a multiple of 256 bytes");
    return row * ROWBYTES + ((ch ^ swz_x256<LEG>(row)) << 4);
  }
}

// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p supplies the address of
// row q (cols 4p..4p+3) of a 4x16 block; lane i of the group receives column
// i of the 4 rows (row q in element q).
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
__device__ __forceinline__ bf16x4 ds_read_tr16(const void* lds_ptr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(lds_ptr));
}

// A/B fragment (8 bf16 of row `row`, 16-byte chunk `ch`) from a swizzled tile.
template <int ROWB, bool LEG = false>
__device__ __forceinline__ bf16x8 lds_frag(const char* lds, int row, int ch) {
  return *reinterpret_cast<const bf16x8*>(lds + swz<ROWB, LEG>(row, ch));
}

__device__ __forceinline__ bf16x8 cat44(const bf16x4& a, const bf16x4& b) {
  bf16x8 f;
  f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3];
  f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
  return f;
}

// B fragment for "accumulator as A operand" products (k order permuted as in
// the header comment): rows r0 + 4h + q and r0 + 8 + 4h + q (q = 0..3) of the
// column block col0..col0+31 (this lane receives column col0 + (lane & 31)),
// read transposed from a swizzled LDS tile.  EXEC must be all ones.
template <int ROWB, bool LEG = false>
__device__ __forceinline__ bf16x8 lds_tr_frag(const char* lds, int r0, int col0, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3, h = lane >> 5;
  const int col = col0 + 16 * (g & 1) + 4 * p;
  const int ra = r0 + 4 * h + q;
  const char* pa = lds + swz<ROWB, LEG>(ra, col >> 3) + (col & 7) * 2;
  const char* pb = lds + swz<ROWB, LEG>(ra + 8, col >> 3) + (col & 7) * 2;
  return cat44(ds_read_tr16(pa), ds_read_tr16(pb));
}

// Same, natural k order (B[k = 8h + j][col]): rows r0 + 8h + q and r0 + 8h + 4 + q.
template <int ROWB>
__device__ __forceinline__ bf16x8 lds_tr_frag_nat(const char* lds, int r0, int col0, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3, h = lane >> 5;
  const int col = col0 + 16 * (g & 1) + 4 * p;
  const int ra = r0 + 8 * h + q;
  const char* pa = lds + swz<ROWB>(ra, col >> 3) + (col & 7) * 2;
  const char* pb = lds + swz<ROWB>(ra + 4, col >> 3) + (col & 7) * 2;
  return cat44(ds_read_tr16(pa), ds_read_tr16(pb));
}

// Bijective XCD remap: workgroup ids with equal (id % 8) run on one XCD; give
// each XCD a contiguous range of logical tile ids (neighbouring tiles share
// operand panels in that XCD's L2).
__device__ __forceinline__ int xcd_remap(int id, int total) {
  const int q = total >> 3, r = total & 7, xcd = id & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (id >> 3);
}

}  // namespace dpa
