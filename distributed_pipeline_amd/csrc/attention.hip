// Fused multi-head attention for head_dim 64 on CDNA4 matrix cores
// (SURVEY K-M8): softmax(Q K^T / 8) with attention dropout, bidirectional
// (DiffuSeq/BERT) or causal (GPT-2).  Inputs are the packed QKV projection
// [B, L, 3, H, 64] so no head split/transposes are materialised.
//
// Forward: one workgroup = 128 queries of one (batch, head), 4 waves x 32.
//   S^T = K Q^T is computed key-major (keys in the accumulator registers, the
//   query on the MFMA lane) so softmax statistics are lane-local.  Pass 1
//   streams K tiles and builds (max, sum) per query -> LSE; pass 2 recomputes
//   S^T, forms the exact probabilities (no online rescale of O needed),
//   applies dropout and feeds them - still in registers - as the A operand of
//   O = P^T V, with V read transposed from LDS (ds_read_b64_tr_b16).
//   For L <= 128 a single pass holds the whole S^T column in registers.
// Backward: two lean kernels, neither with atomics (the q-kernel runs first and also
//   forms delta = rowsum(dO * O) for its queries).  kv-kernel: 128 keys per
//   workgroup (keys on the lane, K/V in registers), sweeps query tiles:
//   dV += dropout(P)^T dO and dK += dS^T Q straight from the accumulators.
//   q-kernel: 128 queries per workgroup (like the forward), sweeps key tiles:
//   dQ += dS K with dS^T as the A operand.  P and dP are recomputed in each.
// Dropout: keep/drop bits come from a per-(query, key-pair) hash of
//   (seed, offset, batch*head), so forward and backward agree without storing
//   a mask.
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "launchers.h"
#include "mfma.h"

namespace dpa {

static constexpr int HD = 64;                        // head dim
static constexpr float ATT_C = 1.4426950408889634f / 8.0f;  // log2(e) / sqrt(64)
static constexpr float LN2f = 0.6931471805599453f;

struct DropCfg {
  uint32_t seedmix;
  uint32_t thr16;  // drop if (16 random bits) < thr16
  float scale;     // 1 / (1 - p)
  bool on;
};

__device__ __forceinline__ DropCfg make_drop(float p, uint32_t seed, uint32_t offset, uint32_t bh) {
  DropCfg d;
  d.on = p > 0.f;
  d.thr16 = (uint32_t)(p * 65536.f + 0.5f);
  d.scale = d.on ? 1.f / (1.f - p) : 1.f;
  d.seedmix = lowbias32(seed ^ lowbias32((offset + rng_base()) * 0xC2B2AE3Du ^ (bh * 0x27D4EB2Fu)));
  return d;
}

__device__ __forceinline__ uint32_t drop_hash(const DropCfg& d, int q, int key) {
  return mix32(d.seedmix ^ ((uint32_t)q * 0x9E3779B1u) ^ ((uint32_t)(key >> 1) * 0x85EBCA77u));
}
__device__ __forceinline__ bool keep_from(const DropCfg& d, uint32_t h, int key) {
  const uint32_t r = (key & 1) ? (h >> 16) : (h & 0xffffu);
  return r >= d.thr16;
}
// keep_from for a per-lane key parity (sh = 16 for an even key, 0 for odd): one shift and one
// compare instead of extracting and selecting a 16-bit half
__device__ __forceinline__ bool keep_sh(const DropCfg& d, uint32_t h, uint32_t sh) {
  return (h << sh) >= (d.thr16 << 16);
}
__device__ __forceinline__ bool keep_bit(const DropCfg& d, int q, int key) {
  return keep_from(d, drop_hash(d, q, key), key);
}
// The same hash from precomputed terms: qt = q * 0x9E3779B1, kt = (key >> 1) * 0x85EBCA77.
// Inside a tile the per-register rows differ by compile-time constants, so the caller
// forms both terms with adds instead of quarter-rate multiplies.
__device__ __forceinline__ uint32_t drop_hash_t(const DropCfg& d, uint32_t qt, uint32_t kt) {
  return mix32(d.seedmix ^ qt ^ kt);
}
constexpr uint32_t DROP_CQ = 0x9E3779B1u, DROP_CK = 0x85EBCA77u;
// accumulator row offset of register i relative to acc_row(0, h) (even for even i)
__host__ __device__ constexpr int acc_off(int i) { return (i & 3) + 8 * (i >> 2); }

// softmax scale in the exp2 domain and the 1/sqrt(D) gradient scale
template <int D>
__device__ __forceinline__ constexpr float att_c() { return D == 64 ? ATT_C : 1.4426950408889634f * 0.08838834764831845f; }
template <int D>
__device__ __forceinline__ constexpr float rsqrt_d() { return D == 64 ? 0.125f : 0.08838834764831845f; }

// stage a [64 rows][D] bf16 tile (rows r0.., stride `ld` elements) -> swizzled LDS
// rows of 2*D bytes; 64*D/8 16-byte chunks over 256 threads
template <int D>
__device__ __forceinline__ void stage_tile(char* lds, const bf16_t* __restrict__ src, int64_t ld,
                                           int r0, int nrows, int tid) {
  constexpr int CPR = D / 8;  // chunks per row
#pragma unroll
  for (int i = 0; i < 64 * CPR / 256; ++i) {
    const int c = tid + i * 256;
    const int row = c / CPR, ch = c % CPR;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r0 + row < nrows) v = *reinterpret_cast<const uint4*>(src + (int64_t)(r0 + row) * ld + ch * 8);
    *reinterpret_cast<uint4*>(lds + swz<2 * D>(row, ch)) = v;
  }
}

// register-staged variant of stage_tile: global -> registers (issued early, so the
// loads of tile t+1 are in flight while tile t is computed), registers -> LDS later
template <int D>
struct TileRegs {
  static constexpr int N = 64 * (D / 8) / 256;
  uint4 v[N];
};

template <int D>
__device__ __forceinline__ void tile_load(TileRegs<D>& r, const bf16_t* __restrict__ src, int64_t ld,
                                          int r0, int nrows, int tid) {
  constexpr int CPR = D / 8;
#pragma unroll
  for (int i = 0; i < TileRegs<D>::N; ++i) {
    const int c = tid + i * 256;
    const int row = c / CPR, ch = c % CPR;
    r.v[i] = make_uint4(0, 0, 0, 0);
    if (r0 + row < nrows) r.v[i] = *reinterpret_cast<const uint4*>(src + (int64_t)(r0 + row) * ld + ch * 8);
  }
}

template <int D>
__device__ __forceinline__ void tile_store(char* lds, const TileRegs<D>& r, int tid) {
  constexpr int CPR = D / 8;
#pragma unroll
  for (int i = 0; i < TileRegs<D>::N; ++i) {
    const int c = tid + i * 256;
    *reinterpret_cast<uint4*>(lds + swz<2 * D>(c / CPR, c % CPR)) = r.v[i];
  }
}

// stage a [64 rows][64 d] bf16 tile (rows r0.., stride `ld` elements) -> swizzled LDS
__device__ __forceinline__ void stage64(char* lds, const bf16_t* __restrict__ src, int64_t ld,
                                        int r0, int nrows, int tid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + i * 256;  // 512 chunks of 16 B
    const int row = c >> 3, ch = c & 7;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r0 + row < nrows) v = *reinterpret_cast<const uint4*>(src + (int64_t)(r0 + row) * ld + ch * 8);
    *reinterpret_cast<uint4*>(lds + swz<128>(row, ch)) = v;
  }
}

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
// Work item (row tile, head, batch) of a 1-D grid of NT x H x B blocks (NT = L/128 row
// tiles).  Blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH "Workgroup
// dispatch"), so the plain 3-D grid (tile fastest, NT = 8 at L = 1024) put every block
// of row tile k on one XCD: causal work per tile is 1..NT units, and the XCD holding the
// heaviest tile finished last (~NT / ((NT + 1) / 2) = 1.8x the balanced time).  Here the
// 8 consecutive blocks dealt to the 8 XCDs share a tile index and take 8 different
// (b, h); the tile index advances every 8 blocks, so each XCD sees every tile of its
// (b, h) items back to back (K/V panel reuse in that XCD's L2) and the same work mix as
// the others.  Causal: row tiles are paired (see below).
struct AttnItem { int t, hd, b, npass; };
__device__ __forceinline__ AttnItem attn_item(int L, int H, bool causal) {
  const int NT = (L + 127) / 128;
  // causal: one block runs row tiles r and NT - 1 - r of its (b, h) one after the other,
  // (r + 1) + (NT - r) = NT + 1 work units for every block - the per-block imbalance of
  // 1..NT units left ~25% of the wave slots empty (PMC: 7.6% more wave-cycles than the
  // non-causal kernel for the same work, 44% more wall time)
  const int NI = causal ? (NT + 1) / 2 : NT;
  const int i = blockIdx.x, BH = gridDim.x / NI;
  int r, bh;
  if ((BH & 7) == 0) {
    const int j = i >> 3;
    r = j % NI;
    bh = (j / NI) * 8 + (i & 7);
  } else {
    r = i % NI;
    bh = i / NI;
  }
  AttnItem it;
  it.t = r;
  it.npass = causal && NT - 1 - r != r ? 2 : 1;
  it.hd = bh % H;
  it.b = bh / H;
  return it;
}
__device__ __forceinline__ AttnItem attn_pass(const AttnItem& it0, int pass, int L) {
  AttnItem it = it0;
  if (pass) it.t = (L + 127) / 128 - 1 - it0.t;
  return it;
}

// blocks of the attn_item() grid
static unsigned attn_grid(int B, int L, int H, bool causal) {
  const int NT = (L + 127) / 128;
  return (unsigned)((causal ? (NT + 1) / 2 : NT) * H * B);
}

template <int D, bool CAUSAL>
__global__ void __launch_bounds__(256) attn_fwd_kernel(const bf16_t* __restrict__ qkv,
                                                      bf16_t* __restrict__ out, float* __restrict__ lse,
                                                      int L, int H, float p, uint32_t seed,
                                                      uint32_t offset) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 64 * 2 * D];
  char* kt_lds = smem;
  char* vt_lds = smem + 64 * 2 * D;
  const AttnItem it0 = attn_item(L, H, CAUSAL);
  for (int pass = 0; pass < it0.npass; ++pass) {  // 2 row tiles per block when causal
  const AttnItem it = attn_pass(it0, pass, L);
  const int b = it.b, hd = it.hd;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hf = lane >> 5;
  const int64_t ld = 3LL * H * D;  // token stride
  const bf16_t* qb = qkv + (int64_t)b * L * ld + (int64_t)hd * D;
  const bf16_t* kb = qb + (int64_t)H * D;
  const bf16_t* vb = qb + 2LL * H * D;
  const int qbase = it.t * 128 + w * 32;
  const int q = qbase + (lane & 31);
  const bool q_ok = q < L;
  bf16x8 qf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    if (q_ok) qf[s] = ld_frag(qb + (int64_t)q * ld + 16 * s + 8 * hf);
    else for (int j = 0; j < 8; ++j) qf[s][j] = 0;
  }
  const DropCfg dc = make_drop(p, seed, offset, (uint32_t)(b * H + hd));
  const int kv_end = CAUSAL ? min(L, it.t * 128 + 128) : L;

  // ---- pass 1: row statistics -------------------------------------------------
  float m = -1e30f, l = 0.f;
  for (int kv0 = 0; kv0 < kv_end; kv0 += 64) {
    stage_tile<D>(kt_lds, kb, ld, kv0, L, tid);
    __syncthreads();
    f32x16 acc[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      acc[t] = zero16();
#pragma unroll
      for (int s = 0; s < D / 16; ++s) acc[t] = mfma32(lds_frag<2 * D>(kt_lds, t * 32 + (lane & 31), 2 * s + hf), qf[s], acc[t]);
    }
    float tmax = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = kv0 + t * 32 + acc_row(i, hf);
        float y = acc[t][i] * att_c<D>();
        if (CAUSAL && key > q) y = -INFINITY;
        acc[t][i] = y;
        tmax = fmaxf(tmax, y);
      }
    const float mn = fmaxf(m, tmax);
    float add = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) add += fexp2(acc[t][i] - mn);
    l = l * fexp2(m - mn) + add;
    m = mn;
    __syncthreads();
  }
  {
    const float m2 = __shfl_xor(m, 32, 64), l2 = __shfl_xor(l, 32, 64);
    const float M = fmaxf(m, m2);
    l = l * fexp2(m - M) + l2 * fexp2(m2 - M);
    m = M;
  }
  const float lse2 = m + log2f(l);
  if (hf == 0 && q_ok) lse[((int64_t)b * H + hd) * L + q] = lse2 * LN2f;

  // ---- pass 2: O = dropout(P) V --------------------------------------------------
  f32x16 o[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) o[dt] = zero16();
  for (int kv0 = 0; kv0 < kv_end; kv0 += 64) {
    stage_tile<D>(kt_lds, kb, ld, kv0, L, tid);
    stage_tile<D>(vt_lds, vb, ld, kv0, L, tid);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      f32x16 acc = zero16();
#pragma unroll
      for (int s = 0; s < D / 16; ++s) acc = mfma32(lds_frag<2 * D>(kt_lds, t * 32 + (lane & 31), 2 * s + hf), qf[s], acc);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = kv0 + t * 32 + acc_row(i, hf);
        float pr = fexp2(acc[i] * att_c<D>() - lse2);
        if (CAUSAL && key > q) pr = 0.f;
        if (dc.on) pr = keep_bit(dc, q, key) ? pr * dc.scale : 0.f;
        acc[i] = pr;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 af = acc_to_frag(acc, s);
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt)
          o[dt] = mfma32(af, lds_tr_frag<2 * D>(vt_lds, t * 32 + 16 * s, dt * 32, lane), o[dt]);
      }
    }
    __syncthreads();
  }
  // o[dt] reg i: row = query qbase + acc_row(i,hf), col = d (dt*32 + lane&31)
  bf16_t* ob = out + (int64_t)b * L * H * D + (int64_t)hd * D;
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int qq = qbase + acc_row(i, hf);
      if (qq < L) ob[(int64_t)qq * H * D + dt * 32 + (lane & 31)] = f2bf(o[dt][i]);
    }
  __syncthreads();  // LDS reuse by the next pass
  }
}


// Single-pass variant (online softmax): per 64-key tile, S^T = K Q^T, the
// per-query running max is combined across the two lane halves (both halves
// feed the same O rows through the MFMA k dimension, so they must share it),
// P = exp2(S - m) goes straight into O += P^T V, and O is rescaled by
// exp2(m_old - m_new).  O's rows live on accumulator registers, not lanes, so a
// register's factor is fetched from the lane that owns that query (one
// ds_bpermute per register per tile).  K is read once instead of twice.
// DROP (attention dropout on, p > 0) is a template parameter in the single-pass forward and
// both backward kernels: the per-score dropout work then carries no wave-uniform branch.
template <int D, bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(256, D == 64 ? 2 : 1) attn_fwd_online_kernel(const bf16_t* __restrict__ qkv,
                                                             bf16_t* __restrict__ out,
                                                             float* __restrict__ lse, int L, int H,
                                                             float p, uint32_t seed, uint32_t offset) {
  // two K/V stages: tile i+1 is stored into the other stage while tile i is read, so one
  // barrier per tile (it both publishes stage i+1 and retires stage i)
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * 64 * 2 * D];
  const AttnItem it0 = attn_item(L, H, CAUSAL);
  for (int pass = 0; pass < it0.npass; ++pass) {  // 2 row tiles per block when causal
  const AttnItem it = attn_pass(it0, pass, L);
  const int b = it.b, hd = it.hd;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hf = lane >> 5;
  const int64_t ld = 3LL * H * D;
  const bf16_t* qb = qkv + (int64_t)b * L * ld + (int64_t)hd * D;
  const bf16_t* kb = qb + (int64_t)H * D;
  const bf16_t* vb = qb + 2LL * H * D;
  const int qbase = it.t * 128 + w * 32;
  const int q = qbase + (lane & 31);
  const bool q_ok = q < L;
  bf16x8 qf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    if (q_ok) qf[s] = ld_frag(qb + (int64_t)q * ld + 16 * s + 8 * hf);
    else for (int j = 0; j < 8; ++j) qf[s][j] = 0;
  }
  const DropCfg dc = make_drop(p, seed, offset, (uint32_t)(b * H + hd));
  const uint32_t qterm = (uint32_t)q * DROP_CQ;
  const uint32_t thr_h = min(dc.thr16, 65535u) ^ 0x8000u;  // p < 1 - 2^-17
  const uint32_t ts2 = thr_h | (thr_h << 16), c15 = 0x000F000Fu, c8000 = 0x80008000u;
  const uint32_t sq = dc.seedmix ^ qterm;
  const int kv_end = CAUSAL ? min(L, it.t * 128 + 128) : L;
  // source lane (in this half's numbering) of the query that register i of O belongs to
  int src[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) src[i] = acc_row(i, hf);
  float m = -1e30f, l = 0.f;
  f32x16 o[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) o[dt] = zero16();
  TileRegs<D> kr, vr;
  tile_load<D>(kr, kb, ld, 0, L, tid);
  tile_load<D>(vr, vb, ld, 0, L, tid);
  tile_store<D>(smem, kr, tid);
  tile_store<D>(smem + 64 * 2 * D, vr, tid);
  __syncthreads();
  for (int kv0 = 0, stg = 0; kv0 < kv_end; kv0 += 64, stg ^= 1) {
    char* kt_lds = smem + stg * (2 * 64 * 2 * D);
    char* vt_lds = kt_lds + 64 * 2 * D;
    const bool more = kv0 + 64 < kv_end;
    if (more) {  // next tile's loads overlap this tile's matrix-core work
      tile_load<D>(kr, kb, ld, kv0 + 64, L, tid);
      tile_load<D>(vr, vb, ld, kv0 + 64, L, tid);
    }
    // wave-uniform: 32-key subtiles past this wave's last query are skipped outright
    // (causal), and the element mask runs only on tiles that cross the diagonal or L.
    // Tiles wholly below the diagonal and inside L (all but <= 2 per row block) run a
    // specialisation with no mask and both subtiles: no per-element compares/selects
    // and static MFMA/accumulator control flow on the hot path.
    const bool tile_masked = (CAUSAL && kv0 + 63 > qbase) || kv0 + 64 > L;
    auto tile = [&](auto mtag) {
      constexpr bool MASKED = decltype(mtag)::value;
      const int nsub = MASKED && CAUSAL ? min(2, max(0, (qbase + 31 - kv0) / 32 + 1)) : 2;
      f32x16 acc[2];
      float tm[2] = {-1e30f, -1e30f};  // two independent max chains, one per subtile
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        acc[t] = zero16();
        if (t >= nsub) continue;
#pragma unroll
        for (int s = 0; s < D / 16; ++s)
          acc[t] = mfma32(lds_frag<2 * D>(kt_lds, t * 32 + (lane & 31), 2 * s + hf), qf[s], acc[t]);
        if constexpr (MASKED) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int key = kv0 + t * 32 + acc_row(i, hf);
            if ((CAUSAL && key > q) || key >= L) acc[t][i] = -INFINITY;
          }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) tm[t] = fmaxf(tm[t], acc[t][i]);
      }
      if (nsub > 0) {
        // running max in the scaled (exp2) domain; O and l are rescaled only when some
        // query's max grew by more than 2^8 (lazy rescale: p <= 256 otherwise, exact
        // in fp32 and bf16), which after the first tiles is almost never
        float tmax = fmaxf(tm[0], tm[1]);
        tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64)) * att_c<D>();
        if (__any(tmax > m + 8.f)) {
          const float mn = fmaxf(m, tmax);
          const float alpha = fexp2(m - mn);
          m = mn;
          l *= alpha;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float f = __shfl(alpha, src[i] + 32 * hf, 64);
#pragma unroll
            for (int dt = 0; dt < D / 32; ++dt) o[dt][i] *= f;
          }
        }
        float add = 0.f;
        bf16x8 pf[2][2];  // P (dropped) as the A fragments of O += P^T V
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          if (t >= nsub) continue;
          // key pair of register i: (kv0 + 32 t + 4 hf + acc_off(i)) / 2, all terms even
          const uint32_t kt0 = (uint32_t)((kv0 + t * 32 + 4 * hf) >> 1) * DROP_CK;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const float pr = fexp2(fmaf(acc[t][i], att_c<D>(), -m));
            add += pr;
            acc[t][i] = pr;
          }
          // registers 2j, 2j + 1 are keys 2k, 2k + 1 of one query: one packed dword per pair,
          // dropped as a pair from its hash (drop_pair)
          uint32_t pk[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) pk[j] = pack_bf2(acc[t][2 * j], acc[t][2 * j + 1]);
          if constexpr (DROP) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
              pk[j] = drop_pair(pk[j], drop_hash_s(sq, kt0 + (uint32_t)(acc_off(2 * j) >> 1) * DROP_CK, c8000), ts2, c15);
          }
#pragma unroll
          for (int s = 0; s < 2; ++s)
            pf[t][s] = __builtin_bit_cast(bf16x8, (u32x4){pk[4 * s], pk[4 * s + 1], pk[4 * s + 2], pk[4 * s + 3]});
        }
        l += add;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          if (t >= nsub) continue;
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const bf16x8 af = pf[t][s];
#pragma unroll
            for (int dt = 0; dt < D / 32; ++dt)
              o[dt] = mfma32(af, lds_tr_frag<2 * D>(vt_lds, t * 32 + 16 * s, dt * 32, lane), o[dt]);
          }
        }
      }
    };
    if (tile_masked) tile(std::true_type{});
    else tile(std::false_type{});
    if (more) {  // the other stage: every wave left it at the previous barrier
      char* nk = smem + (stg ^ 1) * (2 * 64 * 2 * D);
      tile_store<D>(nk, kr, tid);
      tile_store<D>(nk + 64 * 2 * D, vr, tid);
    }
    __syncthreads();
  }
  l += __shfl_xor(l, 32, 64);
  if (hf == 0 && q_ok) lse[((int64_t)b * H + hd) * L + q] = (m + log2f(l)) * LN2f;
  const float inv_l = (DROP ? dc.scale : 1.f) / l;  // the kept probabilities' 1 / (1 - p)
  bf16_t* ob = out + (int64_t)b * L * H * D + (int64_t)hd * D;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float f = __shfl(inv_l, src[i] + 32 * hf, 64);
    const int qq = qbase + acc_row(i, hf);
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
      if (qq < L) ob[(int64_t)qq * H * D + dt * 32 + (lane & 31)] = f2bf(o[dt][i] * f);
  }
  __syncthreads();  // LDS reuse by the next pass
  }
}

// L <= 128: every key of the (batch, head) fits one LDS image and the whole
// S^T column of a query fits in registers -> exact softmax in one pass.
template <bool CAUSAL>
__global__ void __launch_bounds__(256) attn_fwd_small_kernel(const bf16_t* __restrict__ qkv,
                                                            bf16_t* __restrict__ out,
                                                            float* __restrict__ lse, int L, int H,
                                                            float p, uint32_t seed, uint32_t offset) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 128 * 128];
  char* kt_lds = smem;
  char* vt_lds = smem + 128 * 128;
  const int b = blockIdx.z, hd = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hf = lane >> 5;
  const int64_t ld = 3LL * H * HD;
  const bf16_t* qb = qkv + (int64_t)b * L * ld + (int64_t)hd * HD;
  const bf16_t* kb = qb + (int64_t)H * HD;
  const bf16_t* vb = qb + 2LL * H * HD;
  const int nt = L >> 5;  // 32-key tiles (<= 4)
  for (int r0 = 0; r0 < L; r0 += 64) {
    stage64(kt_lds + r0 * 128, kb, ld, r0, L, tid);
    stage64(vt_lds + r0 * 128, vb, ld, r0, L, tid);
  }
  const int qbase = w * 32;
  const int q = qbase + (lane & 31);
  const bool q_ok = q < L;
  bf16x8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (q_ok) qf[s] = ld_frag(qb + (int64_t)q * ld + 16 * s + 8 * hf);
    else for (int j = 0; j < 8; ++j) qf[s][j] = 0;
  }
  const DropCfg dc = make_drop(p, seed, offset, (uint32_t)(b * H + hd));
  __syncthreads();
  if (qbase >= L) return;  // whole wave idle (L < 128); no barrier follows
  f32x16 acc[4];
  float m = -INFINITY;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    acc[t] = zero16();
    if (t < nt) {
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[t] = mfma32(lds_frag<128>(kt_lds, t * 32 + (lane & 31), 2 * s + hf), qf[s], acc[t]);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = t * 32 + acc_row(i, hf);
        float y = acc[t][i] * ATT_C;
        if (CAUSAL && key > q) y = -INFINITY;
        acc[t][i] = y;
        m = fmaxf(m, y);
      }
    }
  }
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  float l = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t)
    if (t < nt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float e = fexp2(acc[t][i] - m);
        acc[t][i] = e;
        l += e;
      }
  l += __shfl_xor(l, 32, 64);
  const float inv_l = 1.f / l;
  if (hf == 0 && q_ok) lse[((int64_t)b * H + hd) * L + q] = (m + log2f(l)) * LN2f;
  f32x16 o[2];
  o[0] = zero16();
  o[1] = zero16();
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (t < nt) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float pr = acc[t][i] * inv_l;
        if (dc.on) pr = keep_bit(dc, q, t * 32 + acc_row(i, hf)) ? pr * dc.scale : 0.f;
        acc[t][i] = pr;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 af = acc_to_frag(acc[t], s);
#pragma unroll
        for (int dt = 0; dt < 2; ++dt)
          o[dt] = mfma32(af, lds_tr_frag<128>(vt_lds, t * 32 + 16 * s, dt * 32, lane), o[dt]);
      }
    }
  }
  bf16_t* ob = out + (int64_t)b * L * H * HD + (int64_t)hd * HD;
#pragma unroll
  for (int dt = 0; dt < 2; ++dt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int qq = qbase + acc_row(i, hf);
      if (qq < L) ob[(int64_t)qq * H * HD + dt * 32 + (lane & 31)] = f2bf(o[dt][i]);
    }
}


// ---------------------------------------------------------------------------
// backward, part 1: dK, dV.  Workgroup = 128 keys (4 waves x 32, keys on the
// MFMA lane, K/V fragments in registers); sweeps query tiles of 64 staged in LDS.
//   S = Q K^T, dP = dO V^T (queries in registers);  P from the saved LSE;
//   dV += dropout(P)^T dO,  dK += dS^T Q   with dS = P (dropout'(dP) - delta),
// both straight from the accumulators (dO / Q read transposed from LDS).
// ---------------------------------------------------------------------------
// Column-sum partials of one 128-row block of a backward output (the qkv bias gradient):
// lane-local sums of the bf16-rounded values over the wave's 16 rows per register column,
// the two lane halves, then the 4 waves through LDS -> dst[D] (= on pass 0, += after).
// rows_ok(i) tells whether register i's row exists (the tail past L).
template <int D, class RowOk>
__device__ __forceinline__ void block_colsum(const f32x16 (&v)[D / 32], float scale, RowOk rows_ok, float* red,
                                             float* dst, bool accumulate, int w, int lane, int tid) {
  const int hf = lane >> 5;
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) {
    float cs = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (rows_ok(i)) cs += bf2f(f2bf(v[dt][i] * scale));
    cs += __shfl_xor(cs, 32, 64);
    if (hf == 0) red[w * D + dt * 32 + (lane & 31)] = cs;
  }
  __syncthreads();
  if (tid < D) {
    const float t = red[tid] + red[D + tid] + red[2 * D + tid] + red[3 * D + tid];
    dst[tid] = accumulate ? dst[tid] + t : t;
  }
  __syncthreads();
}

// colpart slot of the block: [(b * NI + r) * H + h][3 * D] with r the block's (first) row tile
__device__ __forceinline__ int64_t colpart_slot(const AttnItem& it0, int L, int H, bool causal) {
  const int NT = (L + 127) / 128, NI = causal ? (NT + 1) / 2 : NT;
  return ((int64_t)it0.b * NI + it0.t) * H + it0.hd;
}

template <int D, bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(256, D == 64 ? 2 : 1) attn_bwd_kv_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, bf16_t* __restrict__ dqkv, int L, int H, float p,
    uint32_t seed, uint32_t offset, float* __restrict__ colpart) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 64 * 2 * D + 2 * 64 * 4];
  __shared__ float cred[4 * D];
  char* qt_lds = smem;
  char* dot_lds = smem + 64 * 2 * D;
  float* s_lse = reinterpret_cast<float*>(smem + 2 * 64 * 2 * D);
  float* s_del = s_lse + 64;
  const AttnItem it0 = attn_item(L, H, CAUSAL);
  for (int pass = 0; pass < it0.npass; ++pass) {  // 2 row tiles per block when causal
  const AttnItem it = attn_pass(it0, pass, L);
  const int b = it.b, hd = it.hd;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hf = lane >> 5;
  const int64_t ld = 3LL * H * D, ldo = (int64_t)H * D;
  const bf16_t* qb = qkv + (int64_t)b * L * ld + (int64_t)hd * D;
  const bf16_t* kb = qb + (int64_t)H * D;
  const bf16_t* vb = qb + 2LL * H * D;
  const bf16_t* dob = dout + (int64_t)b * L * ldo + (int64_t)hd * D;
  const int kbase = it.t * 128 + w * 32;
  const int key = kbase + (lane & 31);
  const bool k_ok = key < L;
  bf16x8 kf[D / 16], vf[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    if (k_ok) {
      kf[s] = ld_frag(kb + (int64_t)key * ld + 16 * s + 8 * hf);
      vf[s] = ld_frag(vb + (int64_t)key * ld + 16 * s + 8 * hf);
    } else {
      for (int j = 0; j < 8; ++j) { kf[s][j] = 0; vf[s][j] = 0; }
    }
  }
  const DropCfg dc = make_drop(p, seed, offset, (uint32_t)(b * H + hd));
  const int64_t lrow = ((int64_t)b * H + hd) * L;
  f32x16 dk[D / 32], dv[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) { dk[dt] = zero16(); dv[dt] = zero16(); }
  const int qbeg = CAUSAL ? it.t * 128 : 0;
  TileRegs<D> qr, dr;  // register prefetch of the next query tile (Q, dO)
  tile_load<D>(qr, qb, ld, qbeg, L, tid);
  tile_load<D>(dr, dob, ldo, qbeg, L, tid);
  for (int q0 = qbeg; q0 < L; q0 += 64) {
    tile_store<D>(qt_lds, qr, tid);
    tile_store<D>(dot_lds, dr, tid);
    if (tid < 64) {
      const bool ok = q0 + tid < L;
      s_lse[tid] = ok ? lse[lrow + q0 + tid] * 1.4426950408889634f : 0.f;
      s_del[tid] = ok ? delta[lrow + q0 + tid] : 0.f;
    }
    __syncthreads();
    if (q0 + 64 < L) {
      tile_load<D>(qr, qb, ld, q0 + 64, L, tid);
      tile_load<D>(dr, dob, ldo, q0 + 64, L, tid);
    }
#pragma unroll 1
    for (int qt = 0; qt < 2; ++qt) {
      const int qs = q0 + qt * 32;
      // wave-uniform: causal subtiles whose queries all precede this wave's keys are
      // skipped; the element mask runs only across the diagonal / past L
      if (CAUSAL && qs + 31 < kbase) continue;
      const bool sub_masked = (CAUSAL && qs < kbase + 31) || qs + 32 > L || kbase + 32 > L;
      auto sub = [&](auto mtag) {
        constexpr bool MASKED = decltype(mtag)::value;
        f32x16 sacc = zero16(), dpacc = zero16();
#pragma unroll
        for (int s = 0; s < D / 16; ++s) {
          sacc = mfma32(lds_frag<2 * D>(qt_lds, qt * 32 + (lane & 31), 2 * s + hf), kf[s], sacc);
          dpacc = mfma32(lds_frag<2 * D>(dot_lds, qt * 32 + (lane & 31), 2 * s + hf), vf[s], dpacc);
        }
        // dropout hashes: lanes key and key^1 need the same (query, key pair) hashes, so
        // each lane of an adjacent pair computes every other one and takes the rest from
        // its neighbour (DPP quad_perm [1,0,3,2]) - half the quarter-rate multiplies
        uint32_t hh[16];
        if constexpr (DROP) {
          const int par = lane & 1;
          const uint32_t kt = (uint32_t)(key >> 1) * DROP_CK;
          const uint32_t qt0 = (uint32_t)(q0 + qt * 32 + 4 * hf + par) * DROP_CQ;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            // query of register 2j + par: q0 + 32 qt + 4 hf + acc_off(2j) + par
            const uint32_t mine = drop_hash_t(dc, qt0 + (uint32_t)acc_off(2 * j) * DROP_CQ, kt);
            const uint32_t other = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)mine, 0xB1, 0xF, 0xF, true);
            hh[2 * j] = par ? other : mine;
            hh[2 * j + 1] = par ? mine : other;
          }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[i] = fexp2(fmaf(sacc[i], att_c<D>(), -s_lse[qt * 32 + acc_row(i, hf)]));
        // the causal instance serves every subtile: its element mask runs behind a wave-uniform
        // branch, only on subtiles that cross the diagonal or L (not a per-element select on all)
        if (MASKED && (!CAUSAL || sub_masked)) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int qq = q0 + qt * 32 + acc_row(i, hf);
            if ((CAUSAL && key > qq) || !k_ok || qq >= L) sacc[i] = 0.f;
          }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int r = qt * 32 + acc_row(i, hf);
          const float pr = sacc[i];
          if constexpr (DROP) {  // one select per score: the kept-and-scaled multiplier serves P and dP
            const float m = keep_sh(dc, hh[i], (key & 1) ? 0u : 16u) ? dc.scale : 0.f;
            sacc[i] = pr * m;
            dpacc[i] = pr * fmaf(dpacc[i], m, -s_del[r]);
          } else {
            dpacc[i] = pr * (dpacc[i] - s_del[r]);
          }
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 pf = acc_to_frag(sacc, s);
          const bf16x8 sf = acc_to_frag(dpacc, s);
#pragma unroll
          for (int dt = 0; dt < D / 32; ++dt) {
            dv[dt] = mfma32(pf, lds_tr_frag<2 * D>(dot_lds, qt * 32 + 16 * s, dt * 32, lane), dv[dt]);
            dk[dt] = mfma32(sf, lds_tr_frag<2 * D>(qt_lds, qt * 32 + 16 * s, dt * 32, lane), dk[dt]);
          }
        }
      };
      // causal: one instance only (a second copy of these large loop bodies measured
      // slower, 1.76 -> 1.90 ms at L = 1024); non-causal: the mask-free body
      if (CAUSAL || sub_masked) sub(std::true_type{});
      else sub(std::false_type{});
    }
    __syncthreads();
  }
  {
    // per-lane 32-bit offset once (rows 4 hf + c of the wave's 32 keys); the per-register
    // row steps are wave-uniform, and full 32-key blocks need no row guard
    bf16_t* const kvb = dqkv + ((int64_t)b * L + kbase) * ld + (int64_t)hd * D + (int64_t)H * D;
    const uint32_t lo = __umul24((uint32_t)(4 * hf), (uint32_t)ld) + (uint32_t)(lane & 31);
    const bool full = kbase + 32 <= L;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (full || kbase + acc_row(i, hf) < L) {
          bf16_t* base = (kvb + ((int64_t)((i & 3) + 8 * (i >> 2)) * ld + dt * 32)) + lo;
          base[0] = f2bf(dk[dt][i] * rsqrt_d<D>());
          base[(int64_t)H * D] = f2bf(dv[dt][i]);
        }
      }
  }
  if (colpart) {  // k and v bias-gradient partials of this block's keys
    float* cp = colpart + colpart_slot(it0, L, H, CAUSAL) * (3 * D);
    auto ok = [&](int i) { return kbase + acc_row(i, hf) < L; };
    block_colsum<D>(dk, rsqrt_d<D>(), ok, cred, cp + D, pass > 0, w, lane, tid);
    block_colsum<D>(dv, 1.f, ok, cred, cp + 2 * D, pass > 0, w, lane, tid);
  }
  __syncthreads();  // LDS reuse by the next pass
  }
}

// ---------------------------------------------------------------------------
// backward, part 2: dQ.  Workgroup = 128 queries (queries on the lane, Q and dO
// fragments in registers, like the forward); sweeps key tiles of 64 in LDS:
//   S^T = K Q^T, dP^T = V dO^T (keys in registers), dS^T rebuilt, and
//   dQ += dS K with dS^T fed as the A operand and K read transposed.
// No atomics: each workgroup owns its queries' dQ rows completely.
// ---------------------------------------------------------------------------
template <int D, bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(256, D == 64 ? 2 : 1) attn_bwd_q_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout, const float* __restrict__ lse,
    float* __restrict__ delta, bf16_t* __restrict__ dqkv, int L, int H, float p,
    uint32_t seed, uint32_t offset, const bf16_t* __restrict__ out, float* __restrict__ colpart) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 64 * 2 * D];
  __shared__ float cred[4 * D];
  char* kt_lds = smem;
  char* vt_lds = smem + 64 * 2 * D;
  const AttnItem it0 = attn_item(L, H, CAUSAL);
  for (int pass = 0; pass < it0.npass; ++pass) {  // 2 row tiles per block when causal
  const AttnItem it = attn_pass(it0, pass, L);
  const int b = it.b, hd = it.hd;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hf = lane >> 5;
  const int64_t ld = 3LL * H * D, ldo = (int64_t)H * D;
  const bf16_t* qb = qkv + (int64_t)b * L * ld + (int64_t)hd * D;
  const bf16_t* kb = qb + (int64_t)H * D;
  const bf16_t* vb = qb + 2LL * H * D;
  const bf16_t* dob = dout + (int64_t)b * L * ldo + (int64_t)hd * D;
  const int qbase = it.t * 128 + w * 32;
  const int q = qbase + (lane & 31);
  const bool q_ok = q < L;
  bf16x8 qf[D / 16], df[D / 16];
#pragma unroll
  for (int s = 0; s < D / 16; ++s) {
    if (q_ok) {
      qf[s] = ld_frag(qb + (int64_t)q * ld + 16 * s + 8 * hf);
      df[s] = ld_frag(dob + (int64_t)q * ldo + 16 * s + 8 * hf);
    } else {
      for (int j = 0; j < 8; ++j) { qf[s][j] = 0; df[s][j] = 0; }
    }
  }
  const int64_t lrow = ((int64_t)b * H + hd) * L;
  const float lse2 = q_ok ? lse[lrow + q] * 1.4426950408889634f : 0.f;
  // delta = rowsum(dO * O) of this lane's query, from the dO fragments already in
  // registers and the matching O chunks (the two lane halves hold complementary
  // columns); published for the dK/dV kernel, which runs after this one
  float dlt = 0.f;
  if (q_ok) {
    const bf16_t* obq = out + ((int64_t)b * L + q) * ldo + (int64_t)hd * D;
#pragma unroll
    for (int s = 0; s < D / 16; ++s) {
      const bf16x8 of = ld_frag(obq + 16 * s + 8 * hf);
#pragma unroll
      for (int j = 0; j < 8; ++j) dlt += bf2f(df[s][j]) * bf2f(of[j]);
    }
  }
  dlt += __shfl_xor(dlt, 32, 64);
  if (q_ok && hf == 0) delta[lrow + q] = dlt;
  const DropCfg dc = make_drop(p, seed, offset, (uint32_t)(b * H + hd));
  const uint32_t qterm = (uint32_t)q * DROP_CQ;
  f32x16 dq[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) dq[dt] = zero16();
  const int kv_end = CAUSAL ? min(L, it.t * 128 + 128) : L;
  TileRegs<D> kr, vr;  // register prefetch of the next key tile (K, V)
  tile_load<D>(kr, kb, ld, 0, L, tid);
  tile_load<D>(vr, vb, ld, 0, L, tid);
  for (int kv0 = 0; kv0 < kv_end; kv0 += 64) {
    tile_store<D>(kt_lds, kr, tid);
    tile_store<D>(vt_lds, vr, tid);
    __syncthreads();
    if (kv0 + 64 < kv_end) {
      tile_load<D>(kr, kb, ld, kv0 + 64, L, tid);
      tile_load<D>(vr, vb, ld, kv0 + 64, L, tid);
    }
#pragma unroll 1
    for (int t = 0; t < 2; ++t) {
      const int ks = kv0 + t * 32;
      // wave-uniform subtile skip (all keys after this wave's queries) and diagonal-only mask
      if (CAUSAL && ks > qbase + 31) continue;
      const bool sub_masked = (CAUSAL && ks + 31 > qbase) || ks + 32 > L || qbase + 32 > L;
      auto sub = [&](auto mtag) {
        constexpr bool MASKED = decltype(mtag)::value;
        f32x16 sacc = zero16(), dpacc = zero16();
#pragma unroll
        for (int s = 0; s < D / 16; ++s) {
          sacc = mfma32(lds_frag<2 * D>(kt_lds, t * 32 + (lane & 31), 2 * s + hf), qf[s], sacc);
          dpacc = mfma32(lds_frag<2 * D>(vt_lds, t * 32 + (lane & 31), 2 * s + hf), df[s], dpacc);
        }
        const uint32_t kt0 = (uint32_t)((kv0 + t * 32 + 4 * hf) >> 1) * DROP_CK;
        // dropout hashes first, one per key pair, as an independent batch (ILP)
        uint32_t hh[8];
        if constexpr (DROP) {
#pragma unroll
          for (int j = 0; j < 8; ++j) hh[j] = drop_hash_t(dc, qterm, kt0 + (uint32_t)(acc_off(2 * j) >> 1) * DROP_CK);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[i] = fexp2(fmaf(sacc[i], att_c<D>(), -lse2));
        // element mask behind a wave-uniform branch (see the dK/dV kernel)
        if (MASKED && (!CAUSAL || sub_masked)) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int kk = kv0 + t * 32 + acc_row(i, hf);
            if ((CAUSAL && kk > q) || !q_ok || kk >= L) sacc[i] = 0.f;
          }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float pr = sacc[i];
          float dpd = dpacc[i];
          if constexpr (DROP) dpd = keep_from(dc, hh[i >> 1], i & 1) ? dpd * dc.scale : 0.f;
          sacc[i] = pr * (dpd - dlt);
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 sf = acc_to_frag(sacc, s);
#pragma unroll
          for (int dt = 0; dt < D / 32; ++dt)
            dq[dt] = mfma32(sf, lds_tr_frag<2 * D>(kt_lds, t * 32 + 16 * s, dt * 32, lane), dq[dt]);
        }
      };
      // causal: one instance only (a second copy of these large loop bodies measured
      // slower, 1.76 -> 1.90 ms at L = 1024); non-causal: the mask-free body
      if (CAUSAL || sub_masked) sub(std::true_type{});
      else sub(std::false_type{});
    }
    __syncthreads();
  }
  {
    bf16_t* const qob = dqkv + ((int64_t)b * L + qbase) * ld + (int64_t)hd * D;
    const uint32_t lo = __umul24((uint32_t)(4 * hf), (uint32_t)ld) + (uint32_t)(lane & 31);
    const bool full = qbase + 32 <= L;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (full || qbase + acc_row(i, hf) < L)
          ((qob + ((int64_t)((i & 3) + 8 * (i >> 2)) * ld + dt * 32)) + lo)[0] = f2bf(dq[dt][i] * rsqrt_d<D>());
  }
  if (colpart) {  // q bias-gradient partials of this block's queries
    float* cp = colpart + colpart_slot(it0, L, H, CAUSAL) * (3 * D);
    block_colsum<D>(dq, rsqrt_d<D>(), [&](int i) { return qbase + acc_row(i, hf) < L; }, cred, cp, pass > 0, w,
                    lane, tid);
  }
  __syncthreads();  // LDS reuse by the next pass
  }
}

template <int D>
static void attn_fwd_general(const uint16_t* qkv, uint16_t* out, float* lse, int B, int L, int H,
                             float p, bool causal, uint32_t seed, uint32_t offset, hipStream_t s) {
  dim3 grid(attn_grid(B, L, H, causal));  // attn_item() layout
#define DPA_FWD_ONLINE(C, DR)                                                                      \
  hipLaunchKernelGGL((attn_fwd_online_kernel<D, C, DR>), grid, dim3(256), 0, s, (const bf16_t*)qkv, \
                     (bf16_t*)out, lse, L, H, p, seed, offset)
  const bool drop = p > 0.f;
  if (causal) {
    if (drop) DPA_FWD_ONLINE(true, true); else DPA_FWD_ONLINE(true, false);
  } else {
    if (drop) DPA_FWD_ONLINE(false, true); else DPA_FWD_ONLINE(false, false);
  }
#undef DPA_FWD_ONLINE
}

bool launch_attn_fwd(const uint16_t* qkv, uint16_t* out, float* lse, int B, int L, int H, int D,
                     float p, bool causal, uint32_t seed, uint32_t offset, hipStream_t s, bool head_major) {
  if (head_major)  // only the persistent L = 128 kernels read the head-major layout
    return attn128_supports(L, D, causal) &&
           launch_attn128_fwd(qkv, out, lse, B, L, H, p, causal, seed, offset, s, true);
  if (D == 128) {
    if (launch_attn128_fwd_d128(qkv, out, lse, B, L, H, p, causal, seed, offset, s)) return true;
    attn_fwd_general<128>(qkv, out, lse, B, L, H, p, causal, seed, offset, s);
    return true;
  }
  if (launch_attn128_fwd(qkv, out, lse, B, L, H, p, causal, seed, offset, s)) return true;
  if (L <= 128) {
    dim3 grid((L + 127) / 128, H, B);
    if (causal)
      hipLaunchKernelGGL(attn_fwd_small_kernel<true>, grid, dim3(256), 0, s, (const bf16_t*)qkv,
                         (bf16_t*)out, lse, L, H, p, seed, offset);
    else
      hipLaunchKernelGGL(attn_fwd_small_kernel<false>, grid, dim3(256), 0, s, (const bf16_t*)qkv,
                         (bf16_t*)out, lse, L, H, p, seed, offset);
    return true;
  }
  attn_fwd_general<64>(qkv, out, lse, B, L, H, p, causal, seed, offset, s);
  return true;
}

bool attn_bwd_needs_dq_acc(int L) { (void)L; return false; }

template <int D>
static void attn_bwd_general(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout,
                             const float* lse, float* delta, uint16_t* dqkv, int B, int L, int H,
                             float p, bool causal, uint32_t seed, uint32_t offset, hipStream_t s,
                             float* colpart = nullptr) {
  // dQ kernel first: it forms delta = rowsum(dO * O) in-kernel and publishes it for the
  // dK/dV kernel (no separate delta pass over O and dO)
  dim3 grid(attn_grid(B, L, H, causal));  // attn_item() layout
#define DPA_BWD(C, DR)                                                                            \
  do {                                                                                            \
    hipLaunchKernelGGL((attn_bwd_q_kernel<D, C, DR>), grid, dim3(256), 0, s, (const bf16_t*)qkv,  \
                       (const bf16_t*)dout, lse, delta, (bf16_t*)dqkv, L, H, p, seed, offset,     \
                       (const bf16_t*)out, colpart);                                              \
    hipLaunchKernelGGL((attn_bwd_kv_kernel<D, C, DR>), grid, dim3(256), 0, s, (const bf16_t*)qkv, \
                       (const bf16_t*)dout, lse, delta, (bf16_t*)dqkv, L, H, p, seed, offset,     \
                       colpart);                                                                  \
  } while (0)
  const bool drop = p > 0.f;
  if (causal) {
    if (drop) DPA_BWD(true, true); else DPA_BWD(true, false);
  } else {
    if (drop) DPA_BWD(false, true); else DPA_BWD(false, false);
  }
#undef DPA_BWD
}

bool launch_attn_bwd(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout, const float* lse,
                     float* delta, uint16_t* dqkv, float* dq_acc, float* colpart, float* dbias, int B,
                     int L, int H, int D, float p, bool causal, uint32_t seed, uint32_t offset,
                     hipStream_t s, bool head_major, bool db_accumulate, bool defer_reduce) {
  (void)dq_acc;
  if (head_major)  // caller checked attn128_supports
    return launch_attn128_bwd(qkv, out, dout, lse, dqkv, colpart, dbias, B, L, H, p, causal, seed, offset, s,
                              true, db_accumulate, defer_reduce) && dbias != nullptr;
  // dbias != nullptr: the kernels also write per-block column-sum partials of dq / dk / dv
  // into colpart ([attn_colpart_rows][3 D], attn_colpart_floats) and one reduce pass adds
  // them into dbias (zeroed first unless db_accumulate)
  float* cp = dbias ? colpart : nullptr;
  if (D == 128) {
    if (!launch_attn128_bwd_d128(qkv, out, dout, lse, delta, dqkv, B, L, H, p, causal, seed, offset, s, cp))
      attn_bwd_general<128>(qkv, out, dout, lse, delta, dqkv, B, L, H, p, causal, seed, offset, s, cp);
  } else {
    if (launch_attn128_bwd(qkv, out, dout, lse, dqkv, colpart, dbias, B, L, H, p, causal, seed, offset,
                           s, false, db_accumulate, defer_reduce))
      return dbias != nullptr;
    attn_bwd_general<64>(qkv, out, dout, lse, delta, dqkv, B, L, H, p, causal, seed, offset, s, cp);
  }
  if (!dbias) return false;
  if (defer_reduce) return true;  // partials left in colpart for the caller's launch_colpart_reduce
  if (!db_accumulate) (void)hipMemsetAsync(dbias, 0, sizeof(float) * 3 * H * D, s);
  launch_colpart_reduce(colpart, dbias, (int)(attn_colpart_rows(B, L, H, D, causal) / H), H, D, s);
  return true;
}

// rows of the colpart scratch: one per (b, row-tile block, h) of the general kernels (the
// persistent L = 128 kernels: NI = 1, one per (b, h) item)
int64_t attn_colpart_rows(int B, int L, int H, int D, bool causal) {
  (void)D;
  const int NT = (L + 127) / 128, NI = causal ? (NT + 1) / 2 : NT;
  return (int64_t)B * NI * H;
}

// db[part * H * D + h * D + d] += sum_r colpart[(r * H + h) * 3 D + part * D + d] over the R row
// groups in two fixed-order passes (no fp32 atomics: deterministic).  Pass 1, grid
// (3 * H * D / 64, chunks of R), 4 row lanes x 64 columns per block: the chunk's sum is stored in
// place over the chunk's first row (read by no other block); pass 2 adds the chunk sums in order.
__global__ void __launch_bounds__(256) colpart_reduce_d_kernel(float* __restrict__ colpart, int R, int H, int D,
                                                               int rchunk) {
  __shared__ float red[4][64];
  const int c64 = D / 64, x = blockIdx.x;
  const int part = x / (H * c64), h = (x / c64) % H, cc = x % c64;
  const int d = cc * 64 + (threadIdx.x & 63), rl = threadIdx.x >> 6;
  const int r0 = blockIdx.y * rchunk, r1 = min(R, r0 + rchunk);
  float t = 0.f;
  for (int r = r0 + rl; r < r1; r += 4) t += colpart[((int64_t)r * H + h) * 3 * D + part * D + d];
  red[rl][threadIdx.x & 63] = t;
  __syncthreads();
  if (rl == 0 && r0 < r1) {
    const int i = threadIdx.x;
    colpart[((int64_t)r0 * H + h) * 3 * D + part * D + d] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
  }
}

// grid (3 * H * D / 64), 64 threads
__global__ void __launch_bounds__(64) colpart_final_d_kernel(const float* __restrict__ colpart, float* __restrict__ db,
                                                             int R, int H, int D, int rchunk) {
  const int c64 = D / 64, x = blockIdx.x;
  const int part = x / (H * c64), h = (x / c64) % H, cc = x % c64;
  const int d = cc * 64 + threadIdx.x;
  float t = 0.f;
  for (int r0 = 0; r0 < R; r0 += rchunk) t += colpart[((int64_t)r0 * H + h) * 3 * D + part * D + d];
  db[part * H * D + h * D + d] += t;
}

void launch_colpart_reduce(float* colpart, float* db, int R, int H, int D, hipStream_t s) {
  const int rchunk = 64, nch = (R + rchunk - 1) / rchunk;
  hipLaunchKernelGGL(colpart_reduce_d_kernel, dim3(3 * H * (D / 64), nch), dim3(256), 0, s, colpart, R, H, D,
                     rchunk);
  hipLaunchKernelGGL(colpart_final_d_kernel, dim3(3 * H * (D / 64)), dim3(64), 0, s, (const float*)colpart, db, R, H,
                     D, rchunk);
}

DPA_RNG_BASE_EXPORT(attention)

}  // namespace dpa
