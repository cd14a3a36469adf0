// DiffuSeq diffusion-side kernels (SURVEY K-M1..K-M4, K-M13; the workload the
// reference trainer was adapted for, reference utils/trainer.py:1-4, Appendix B):
//
//   emb_qsample_fwd : x0_mean = W[ids] (fp32 word embedding: the diffusion space)
//                     x_start = x0_mean + std0 * eps0
//                     x_t     = mask ? sqrt(abar_t) x_start + sqrt(1-abar_t) eps : x_start
//                     -> x_start fp32, x_start bf16 (rounding-head input), x_t bf16 (model input).
//                     eps0 / eps are generated in-kernel (counter-based Philox + Box-Muller), so
//                     the noise tensors never exist in memory.
//   emb_qsample_bwd : dW[ids] += d_xstart + d_xstart16 + (mask ? sqrt(abar_t) : 1) d_x_t
//                     (a deterministic segment sum over the stably sorted ids straight into the
//                     tied embedding's gradient; the tied rounding head's dW comes from the fused
//                     linear-CE kernel, also without atomics)
//   diff_loss_fwd   : per sample  mse = mean((target - out)^2), target = t==0 ? x0_mean : x_start
//                                 tT  = mean((sqrt(abar_{T-1}) x_start)^2)
//   diff_loss_bwd   : d_out, d_xstart (fp32) and, for t==0 samples, d x0_mean: folded into
//                     d_xstart (fold_t0: x_start = x0_mean + noise, so it reaches dW through
//                     emb_qsample_bwd) or added into dW[ids] with fp32 atomics
//   timestep_emb    : [cos(t f_j) | sin(t f_j)], f_j = 10000^(-j/half) -> bf16
//
// Forward layout: a token row of E fp32 values is owned by E/4 consecutive lanes
// (16-byte vectors), so every load/store is part of a full 128-byte line.  The
// scatter-add backward is element-per-lane instead: one wave-instruction's 64
// atomics then cover 256 contiguous bytes, the shape the memory-side atomic
// units serve at full rate (MI355X_MICROARCH, Global float atomics).
//
// Timestep indices are trusted to lie in [0, T) (they come from the schedule
// sampler); token ids outside [0, V) contribute nothing.
#include "common.h"
#include "launchers.h"

namespace dpa {

// Four standard normals for (seed, stream, element-group) via one Philox call.
__device__ __forceinline__ void normal4(uint32_t seed, uint32_t stream, uint32_t offset,
                                        uint64_t grp, float out[4]) {
  uint32_t r[4];
  philox4(seed, 0x2545F491u ^ stream, (uint32_t)grp, (uint32_t)(grp >> 32), offset + rng_base(), stream, r);
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    // u1 in (0, 1]: never log(0)
    const float u1 = ((float)(r[2 * k] >> 8) + 1.0f) * (1.0f / 16777216.0f);
    const float u2 = (float)(r[2 * k + 1] >> 8) * (1.0f / 16777216.0f);
    const float rad = sqrtf(-2.0f * __logf(u1));
    float s, c;
    __sincosf(6.283185307179586f * u2, &s, &c);
    out[2 * k] = rad * c;
    out[2 * k + 1] = rad * s;
  }
}

__device__ __forceinline__ f32x4 load4_bf(const bf16_t* p) {
  const uint2 raw = *reinterpret_cast<const uint2*>(p);
  f32x4 r;
  r[0] = __uint_as_float(raw.x << 16);
  r[1] = __uint_as_float(raw.x & 0xffff0000u);
  r[2] = __uint_as_float(raw.y << 16);
  r[3] = __uint_as_float(raw.y & 0xffff0000u);
  return r;
}

__device__ __forceinline__ void store4_bf(bf16_t* p, const f32x4& v) {
  uint2 raw;
  raw.x = pack_bf2(v[0], v[1]);
  raw.y = pack_bf2(v[2], v[3]);
  *reinterpret_cast<uint2*>(p) = raw;
}

__global__ void __launch_bounds__(256) emb_qsample_fwd_kernel(
    const int64_t* __restrict__ ids, const int64_t* __restrict__ mask, const int64_t* __restrict__ t,
    const float* __restrict__ W, const float* __restrict__ sa, const float* __restrict__ s1a,
    int64_t NT, int L, int E, int V, float std0, uint32_t seed, uint32_t offset,
    float* __restrict__ x_start, bf16_t* __restrict__ x_start16, bf16_t* __restrict__ x_t) {
  const int vpr = E >> 2;  // 16-byte vectors per row
  const int64_t n = NT * vpr;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t tok = q / vpr;
    const int c = (int)(q - tok * vpr) * 4;
    const int64_t id = ids[tok];
    f32x4 x0 = {0.f, 0.f, 0.f, 0.f};
    if (id >= 0 && id < V) x0 = *reinterpret_cast<const f32x4*>(W + id * E + c);
    float e0[4], e1[4];
    normal4(seed, 0u, offset, (uint64_t)q, e0);
    normal4(seed, 1u, offset, (uint64_t)q, e1);
    const bool noised = mask[tok] != 0;
    const int64_t ts = t[tok / L];
    const float a = noised ? sa[ts] : 1.f, b = noised ? s1a[ts] : 0.f;
    f32x4 xs, xt;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      xs[k] = x0[k] + std0 * e0[k];
      xt[k] = a * xs[k] + b * e1[k];
    }
    const int64_t o = tok * E + c;
    *reinterpret_cast<f32x4*>(x_start + o) = xs;
    if (x_start16) store4_bf(x_start16 + o, xs);
    store4_bf(x_t + o, xt);
  }
}

// Gradients are bf16 (d_xs16, d_xt16) or fp32 (d_xs, d_xt32); any may be null.
__global__ void __launch_bounds__(256) emb_qsample_bwd_kernel(
    const int64_t* __restrict__ ids, const int64_t* __restrict__ mask, const int64_t* __restrict__ t,
    const float* __restrict__ sa, const float* __restrict__ d_xs, const bf16_t* __restrict__ d_xs16,
    const bf16_t* __restrict__ d_xt16, const float* __restrict__ d_xt32, int64_t NT, int L, int E,
    int V, float* __restrict__ dW) {
  const int64_t n = NT * E;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t tok = q / E;
    const int c = (int)(q - tok * E);
    const int64_t id = ids[tok];
    if (id < 0 || id >= V) continue;
    float g = 0.f;
    if (d_xs) g = d_xs[q];
    if (d_xs16) g += bf2f(d_xs16[q]);
    if (d_xt16 || d_xt32) {
      const float a = mask[tok] != 0 ? sa[t[tok / L]] : 1.f;
      g += a * (d_xt16 ? bf2f(d_xt16[q]) : d_xt32[q]);
    }
    atomicAdd(dW + id * E + c, g);
  }
}

// Sorted variant (ids STABLY sorted on the device beforehand, csrc/sort.hip; perm = the sort
// permutation): one wave walks `chunk` consecutive sorted tokens with its lanes over the E
// columns and sums the gradients of equal ids in registers - ~8 tokens share an id at
// DiffuSeq-base shapes, and the gradient rows are read as coalesced lines.  Deterministic: every
// row of dW has exactly one writer, in a fixed order.
//  * a run of equal ids that lies inside the wave's chunk is added to dW by the wave (plain
//    read-modify-write: no other wave touches that row in this kernel);
//  * a run crossing a chunk boundary leaves per-chunk partials in part[chunk][2][E]: slot 0 = the
//    piece that continues a run from the previous chunk, slot 1 = the piece of a run that starts
//    in this chunk and continues past it; emb_grad_fixup_kernel adds them in chunk order.
//
// The chunk's per-token metadata (sorted id, token, q_sample coefficient) is loaded lane-parallel
// once - lane l holds token l of the chunk - and broadcast with readlane, so the token loop has
// no dependent global loads; the gradient rows of a batch of TB tokens are all in flight before
// the in-order run accumulation consumes them.
__device__ __forceinline__ int64_t readlane64(int64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), l);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ float readlanef(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

template <int CPL>
__global__ void __launch_bounds__(256) emb_grad_sorted_kernel(
    const int64_t* __restrict__ sid, const int64_t* __restrict__ perm, const int64_t* __restrict__ mask,
    const int64_t* __restrict__ t, const float* __restrict__ sa, const float* __restrict__ d_xs,
    const bf16_t* __restrict__ d_xs16, const bf16_t* __restrict__ d_xt16, const float* __restrict__ d_xt32,
    int64_t NT, int L, int V, float* __restrict__ dW, int chunk, float* __restrict__ part) {
  constexpr int E = 64 * CPL;
  constexpr int TB = 64 / CPL > 16 ? 16 : 64 / CPL;  // tokens whose rows are loaded together
  const int lane = threadIdx.x & 63;
  const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t j0 = c * chunk;
  if (j0 >= NT) return;
  const int64_t j1 = j0 + chunk < NT ? j0 + chunk : NT;
  const int n = (int)(j1 - j0);  // <= 64 (emb_chunk)
  int64_t my_id = 0, my_tok = 0;
  float my_a = 0.f;
  if (lane < n) {
    my_id = sid[j0 + lane];
    my_tok = perm[j0 + lane];
    if (d_xt16 || d_xt32) my_a = mask[my_tok] != 0 ? sa[t[my_tok / L]] : 1.f;
  }
  float acc[CPL];
#pragma unroll
  for (int k = 0; k < CPL; ++k) acc[k] = 0.f;
  int64_t cur = readlane64(my_id, 0);
  bool first = true;
  const bool head = j0 > 0 && sid[j0 - 1] == cur;  // the first run continues one from the left
  const int64_t next = j1 < NT ? sid[j1] : -1;
  auto flush = [&](bool at_end) {
    const bool cont = at_end && j1 < NT && next == cur;  // the run goes on past the chunk
    float* dst = nullptr;
    bool add = false;
    if (first && head) dst = part + (c * 2) * E;               // continuation piece
    else if (cont) dst = part + (c * 2 + 1) * E;               // head piece of a crossing run
    else if (cur >= 0 && cur < V) { dst = dW + cur * E; add = true; }  // a whole run
    if (dst) {
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        float* q = dst + lane + 64 * k;
        *q = add ? *q + acc[k] : acc[k];
      }
    }
#pragma unroll
    for (int k = 0; k < CPL; ++k) acc[k] = 0.f;
    first = false;
  };
  for (int b = 0; b < n; b += TB) {
    float g[TB][CPL];
#pragma unroll
    for (int u = 0; u < TB; ++u) {  // every row of the batch in flight (clamped index past n)
      const int jj = b + u < n ? b + u : n - 1;
      const int64_t base = readlane64(my_tok, jj) * E;
      const float a = readlanef(my_a, jj);
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        const int64_t o = base + lane + 64 * k;
        float v = 0.f;
        if (d_xs) v = d_xs[o];
        if (d_xs16) v += bf2f(d_xs16[o]);
        if (d_xt16) v += a * bf2f(d_xt16[o]);
        else if (d_xt32) v += a * d_xt32[o];
        g[u][k] = v;
      }
    }
#pragma unroll
    for (int u = 0; u < TB; ++u) {
      if (b + u < n) {
        const int64_t id = readlane64(my_id, b + u);
        if (id != cur) {  // wave-uniform
          flush(false);
          cur = id;
        }
#pragma unroll
        for (int k = 0; k < CPL; ++k) acc[k] += g[u][k];
      }
    }
  }
  flush(true);
}

// Runs crossing chunk boundaries are combined in two fixed-order levels so a run of tens of
// thousands of tokens (the padding id) is not one wave's serial walk: chunks are grouped by
// EMB_G; emb_grad_group_kernel sums, per group that starts inside a run, the continuation pieces
// (slot 0) of the group's chunks that belong to that run; emb_grad_fixup_kernel then has the
// run's starting chunk add its head piece, the continuation pieces up to its group's end, and
// the group sums of the groups the run covers, in order, and write dW once.
constexpr int EMB_G = 64;

// sum_{k < n} src[k * stride + lane + 64 kk] in k order, U rows in flight
template <int CPL>
__device__ __forceinline__ void emb_sum_rows(float (&acc)[CPL], const float* __restrict__ src, int64_t stride,
                                             int n, int lane) {
  constexpr int U = CPL <= 4 ? 8 : CPL <= 16 ? 2 : 1;
  for (int k0 = 0; k0 < n; k0 += U) {
    float v[U][CPL];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u < n ? k0 + u : n - 1;
#pragma unroll
      for (int kk = 0; kk < CPL; ++kk) v[u][kk] = src[k * stride + lane + 64 * kk];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (k0 + u < n) {
#pragma unroll
        for (int kk = 0; kk < CPL; ++kk) acc[kk] += v[u][kk];
      }
  }
}

template <int CPL>
__global__ void __launch_bounds__(256) emb_grad_group_kernel(const int64_t* __restrict__ sid, int64_t NT,
                                                             int chunk, const float* __restrict__ part,
                                                             float* __restrict__ gsum) {
  constexpr int E = 64 * CPL;
  const int lane = threadIdx.x & 63;
  const int64_t nch = (NT + chunk - 1) / chunk, ng = (nch + EMB_G - 1) / EMB_G;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g == 0 || g >= ng) return;
  const int64_t c0 = g * EMB_G, r = sid[c0 * chunk];
  if (sid[c0 * chunk - 1] != r) return;  // the group does not start inside a run
  const int64_t cl = c0 + lane;
  const bool in = cl < nch && sid[cl * chunk] == r;
  const uint64_t out = __ballot(!in);
  const int n = out ? __builtin_ctzll(out) : 64;  // chunks c0 .. c0+n-1 continue the run
  float acc[CPL];
#pragma unroll
  for (int k = 0; k < CPL; ++k) acc[k] = 0.f;
  emb_sum_rows<CPL>(acc, part + (c0 * 2) * E, 2 * E, n, lane);
#pragma unroll
  for (int k = 0; k < CPL; ++k) gsum[g * E + lane + 64 * k] = acc[k];
}

template <int CPL>
__global__ void __launch_bounds__(256) emb_grad_fixup_kernel(const int64_t* __restrict__ sid, int64_t NT, int V,
                                                             int chunk, const float* __restrict__ part,
                                                             const float* __restrict__ gsum,
                                                             float* __restrict__ dW) {
  constexpr int E = 64 * CPL;
  const int lane = threadIdx.x & 63;
  const int64_t nch = (NT + chunk - 1) / chunk, ng = (nch + EMB_G - 1) / EMB_G;
  const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= nch) return;
  const int64_t j0 = c * chunk, j1 = j0 + chunk < NT ? j0 + chunk : NT;
  if (j1 >= NT) return;
  const int64_t r = sid[j1 - 1];
  if (sid[j1] != r) return;                                    // the last run ends in the chunk
  if (sid[j0] == r && j0 > 0 && sid[j0 - 1] == r) return;      // ... or is a continuation piece
  float acc[CPL];
#pragma unroll
  for (int k = 0; k < CPL; ++k) acc[k] = part[(c * 2 + 1) * E + lane + 64 * k];
  // continuation pieces up to the end of this chunk's group (< EMB_G <= 64 chunks)
  const int64_t gend = (c / EMB_G + 1) * EMB_G < nch ? (c / EMB_G + 1) * EMB_G : nch;
  const int64_t cl = c + 1 + lane;
  const bool in = cl < gend && sid[cl * chunk] == r;
  const uint64_t out = __ballot(!in);
  const int n = out ? __builtin_ctzll(out) : 64;
  emb_sum_rows<CPL>(acc, part + ((c + 1) * 2) * E, 2 * E, n, lane);
  if (c + 1 + n == gend && gend < nch) {  // the run reached the group's end: group sums, 64 at a time
    for (int64_t g2 = gend / EMB_G; g2 < ng;) {
      const int64_t gl = g2 + lane;
      const bool gin = gl < ng && sid[gl * EMB_G * chunk] == r;
      const uint64_t gout = __ballot(!gin);
      const int m = gout ? __builtin_ctzll(gout) : 64;
      emb_sum_rows<CPL>(acc, gsum + g2 * E, E, m, lane);
      if (m < 64) break;
      g2 += 64;
    }
  }
  if (r < 0 || r >= V) return;
#pragma unroll
  for (int k = 0; k < CPL; ++k) dW[r * E + lane + 64 * k] += acc[k];
}

// sorted tokens per wave: 16 for large NT (runs of equal ids summed in registers), down to 1 for
// a few hundred rows (e.g. a position-embedding gradient of 128 distinct ids), so the launch
// still spans the chip instead of a handful of latency-bound waves; the q_sample backward: 16
static int emb_chunk(int64_t NT, bool qsample) {
  if (qsample) return 16;
  const int64_t chunk = NT / 8192;
  return (int)(chunk < 1 ? 1 : chunk > 16 ? 16 : chunk);
}
static int64_t emb_groups(int64_t NT, bool qsample) {
  const int64_t nch = (NT + emb_chunk(NT, qsample) - 1) / emb_chunk(NT, qsample);
  return (nch + EMB_G - 1) / EMB_G;
}
// part = [nch][2][E] chunk pieces, then [ngroups][E] group sums
int64_t emb_grad_part_floats(int64_t NT, int E, bool qsample) {
  const int64_t nch = (NT + emb_chunk(NT, qsample) - 1) / emb_chunk(NT, qsample);
  return (nch * 2 + emb_groups(NT, qsample)) * (int64_t)E;
}

template <int CPL>
static void launch_emb_sorted(const int64_t* sid, const int64_t* perm, const int64_t* mask, const int64_t* t,
                              const float* sa, const float* d_xs, const bf16_t* d_xs16, const bf16_t* d_xt16,
                              const float* d_xt32, int64_t NT, int L, int V, float* dW, int chunk, float* part,
                              int64_t ng, hipStream_t s) {
  constexpr int E = 64 * CPL;
  const int64_t nch = (NT + chunk - 1) / chunk;
  float* gsum = part + nch * 2 * E;
  const unsigned grid = (unsigned)((nch + 3) / 4);
  hipLaunchKernelGGL(emb_grad_sorted_kernel<CPL>, dim3(grid), dim3(256), 0, s, sid, perm, mask, t, sa, d_xs,
                     d_xs16, d_xt16, d_xt32, NT, L, V, dW, chunk, part);
  if (ng > 1)
    hipLaunchKernelGGL(emb_grad_group_kernel<CPL>, dim3((unsigned)((ng + 3) / 4)), dim3(256), 0, s, sid, NT, chunk,
                       (const float*)part, gsum);
  hipLaunchKernelGGL(emb_grad_fixup_kernel<CPL>, dim3(grid), dim3(256), 0, s, sid, NT, V, chunk,
                     (const float*)part, (const float*)gsum, dW);
}

// One workgroup per sample: reductions over the sample's L*E elements.
template <bool OUT_BF16>
__global__ void __launch_bounds__(256) diff_loss_fwd_kernel(
    const float* __restrict__ x_start, const void* __restrict__ out_, const int64_t* __restrict__ ids,
    const int64_t* __restrict__ t, const float* __restrict__ W, int L, int E, int V, float sa_last,
    float* __restrict__ mse, float* __restrict__ tT) {
  __shared__ float red[2][4];
  const int b = blockIdx.x;
  const bool t0 = t[b] == 0;
  const int vpr = E >> 2;
  const int64_t base = (int64_t)b * L * E;
  float s_mse = 0.f, s_tt = 0.f;
  for (int q = threadIdx.x; q < L * vpr; q += blockDim.x) {
    const int tok = q / vpr, c = (q - tok * vpr) * 4;
    const int64_t o = base + (int64_t)tok * E + c;
    const f32x4 xs = *reinterpret_cast<const f32x4*>(x_start + o);
    f32x4 y;
    if (OUT_BF16) y = load4_bf(reinterpret_cast<const bf16_t*>(out_) + o);
    else y = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(out_) + o);
    f32x4 tg = xs;
    if (t0) {
      const int64_t id = ids[(int64_t)b * L + tok];
      tg = (id >= 0 && id < V) ? *reinterpret_cast<const f32x4*>(W + id * E + c)
                               : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float d = tg[k] - y[k];
      s_mse += d * d;
      s_tt += xs[k] * xs[k];
    }
  }
  s_mse = wave_sum(s_mse);
  s_tt = wave_sum(s_tt);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][w] = s_mse;
    red[1][w] = s_tt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float inv = 1.f / (float)(L * E);
    float a = 0.f, c = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
      a += red[0][i];
      c += red[1][i];
    }
    mse[b] = a * inv;
    tT[b] = c * inv * sa_last * sa_last;
  }
}

template <bool OUT_BF16>
__global__ void __launch_bounds__(256) diff_loss_bwd_kernel(
    const float* __restrict__ x_start, const void* __restrict__ out_, const int64_t* __restrict__ ids,
    const int64_t* __restrict__ t, const float* __restrict__ W, const float* __restrict__ dmse,
    const float* __restrict__ dtT, int B, int L, int E, int V, float sa_last,
    void* __restrict__ d_out_, float* __restrict__ d_xs, float* __restrict__ dW, bool fold_t0) {
  const int vpr = E >> 2;
  const int64_t n = (int64_t)B * L * vpr;
  const float inv = 1.f / (float)(L * E);
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t tok = q / vpr;
    const int c = (int)(q - tok * vpr) * 4;
    const int b = (int)(tok / L);
    const int64_t o = tok * E + c;
    const f32x4 xs = *reinterpret_cast<const f32x4*>(x_start + o);
    f32x4 y;
    if (OUT_BF16) y = load4_bf(reinterpret_cast<const bf16_t*>(out_) + o);
    else y = *reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(out_) + o);
    const bool t0 = t[b] == 0;
    const float gm = dmse ? dmse[b] * 2.f * inv : 0.f;
    const float gt = dtT ? dtT[b] * 2.f * inv * sa_last * sa_last : 0.f;
    f32x4 tg = xs;
    const int64_t id = ids[tok];
    const bool id_ok = id >= 0 && id < V;
    if (t0) tg = id_ok ? *reinterpret_cast<const f32x4*>(W + id * E + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 dy, dx;
    // fold_t0: x_start = W[id] + noise (emb_qsample), so the t == 0 branch's gradient into the
    // embedding row, -dy, rides on d_xs and reaches dW through the sorted, deterministic
    // emb_qsample backward instead of fp32 atomics here
    const bool sub = !t0 || (fold_t0 && id_ok);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float r = y[k] - tg[k];
      dy[k] = gm * r;
      dx[k] = gt * xs[k] - (sub ? gm * r : 0.f);
    }
    if (d_out_) {
      if (OUT_BF16) store4_bf(reinterpret_cast<bf16_t*>(d_out_) + o, dy);
      else *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(d_out_) + o) = dy;
    }
    if (d_xs) *reinterpret_cast<f32x4*>(d_xs + o) = dx;
    if (t0 && dW && id_ok && !fold_t0) {  // d x0_mean of the t == 0 branch -> tied embedding rows
#pragma unroll
      for (int k = 0; k < 4; ++k) atomicAdd(dW + id * E + c + k, -dy[k]);
    }
  }
}

__global__ void __launch_bounds__(256) timestep_emb_kernel(const float* __restrict__ ts, int B, int dim,
                                                           float log_max_period,
                                                           bf16_t* __restrict__ out) {
  const int half = dim >> 1;
  const int64_t n = (int64_t)B * dim;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int b = (int)(i / dim), j = (int)(i - (int64_t)b * dim);
    float v = 0.f;
    if (j < 2 * half) {
      const int jj = j < half ? j : j - half;
      const float f = expf(-log_max_period * (float)jj / (float)half);
      const float a = ts[b] * f;
      v = j < half ? cosf(a) : sinf(a);
    }
    out[i] = f2bf(v);
  }
}

static inline unsigned grid_cap(int64_t n, int cap) {
  int64_t g = (n + 255) / 256;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

bool launch_emb_qsample_fwd(const int64_t* ids, const int64_t* mask, const int64_t* t, const float* W,
                            const float* sa, const float* s1a, int64_t NT, int L, int E, int V,
                            float std0, uint32_t seed, uint32_t offset, float* x_start,
                            uint16_t* x_start16, uint16_t* x_t, hipStream_t s) {
  if (E % 4 != 0 || L <= 0) return false;
  hipLaunchKernelGGL(emb_qsample_fwd_kernel, dim3(grid_cap(NT * (E / 4), 256 * 16)), dim3(256), 0, s,
                     ids, mask, t, W, sa, s1a, NT, L, E, V, std0, seed, offset, x_start,
                     (bf16_t*)x_start16, (bf16_t*)x_t);
  return true;
}

bool launch_emb_qsample_bwd(const int64_t* ids, const int64_t* mask, const int64_t* t, const float* sa,
                            const float* d_xs, const uint16_t* d_xs16, const uint16_t* d_xt16,
                            const float* d_xt32, int64_t NT, int L, int E, int V, float* dW,
                            hipStream_t s, const int64_t* sorted_ids,
                            const int64_t* perm, float* part) {
  if (L <= 0 || E <= 0) return false;
  if (sorted_ids && perm && part && (E == 128 || E == 256)) {
    const int CHUNK = emb_chunk(NT, true);
    const int64_t ng = emb_groups(NT, true);
    if (E == 128)
      launch_emb_sorted<2>(sorted_ids, perm, mask, t, sa, d_xs, (const bf16_t*)d_xs16, (const bf16_t*)d_xt16, d_xt32,
                           NT, L, V, dW, CHUNK, part, ng, s);
    else
      launch_emb_sorted<4>(sorted_ids, perm, mask, t, sa, d_xs, (const bf16_t*)d_xs16, (const bf16_t*)d_xt16, d_xt32,
                           NT, L, V, dW, CHUNK, part, ng, s);
    return true;
  }
  hipLaunchKernelGGL(emb_qsample_bwd_kernel, dim3(grid_cap(NT * E, 256 * 16)), dim3(256), 0, s, ids,
                     mask, t, sa, d_xs, (const bf16_t*)d_xs16, (const bf16_t*)d_xt16, d_xt32, NT, L,
                     E, V, dW);
  return true;
}

// Plain token-embedding backward over sorted ids (GPT-2 wte / wpe): the same sorted
// segment-sum kernel with only the upstream gradient as input.
bool launch_emb_grad(const int64_t* sorted_ids, const int64_t* perm, const float* dy32, const uint16_t* dy16,
                     int64_t NT, int E, int V, float* dW, float* part, hipStream_t s) {
  const int CHUNK = emb_chunk(NT, false);
  const int64_t ng = emb_groups(NT, false);
#define DPA_EMB_GO(CPL)                                                                                      \
  launch_emb_sorted<CPL>(sorted_ids, perm, nullptr, nullptr, nullptr, dy32, (const bf16_t*)dy16, nullptr, nullptr, \
                         NT, 1, V, dW, CHUNK, part, ng, s)
  switch (E) {
    case 128: DPA_EMB_GO(2); return true;
    case 256: DPA_EMB_GO(4); return true;
    case 768: DPA_EMB_GO(12); return true;
    case 1024: DPA_EMB_GO(16); return true;
    case 2048: DPA_EMB_GO(32); return true;
    default: return false;
  }
#undef DPA_EMB_GO
}

bool launch_diff_loss_fwd(const float* x_start, const void* out, bool out_bf16, const int64_t* ids,
                          const int64_t* t, const float* W, int B, int L, int E, int V, float sa_last,
                          float* mse, float* tT, hipStream_t s) {
  if (E % 4 != 0 || B <= 0) return false;
  if (out_bf16)
    hipLaunchKernelGGL(diff_loss_fwd_kernel<true>, dim3(B), dim3(256), 0, s, x_start, out, ids, t, W, L,
                       E, V, sa_last, mse, tT);
  else
    hipLaunchKernelGGL(diff_loss_fwd_kernel<false>, dim3(B), dim3(256), 0, s, x_start, out, ids, t, W,
                       L, E, V, sa_last, mse, tT);
  return true;
}

bool launch_diff_loss_bwd(const float* x_start, const void* out, bool out_bf16, const int64_t* ids,
                          const int64_t* t, const float* W, const float* dmse, const float* dtT, int B,
                          int L, int E, int V, float sa_last, void* d_out, float* d_xs, float* dW,
                          hipStream_t s, bool fold_t0) {
  if (E % 4 != 0 || B <= 0 || (fold_t0 && d_xs == nullptr)) return false;
  const unsigned g = grid_cap((int64_t)B * L * (E / 4), 256 * 16);
  if (out_bf16)
    hipLaunchKernelGGL(diff_loss_bwd_kernel<true>, dim3(g), dim3(256), 0, s, x_start, out, ids, t, W,
                       dmse, dtT, B, L, E, V, sa_last, d_out, d_xs, dW, fold_t0);
  else
    hipLaunchKernelGGL(diff_loss_bwd_kernel<false>, dim3(g), dim3(256), 0, s, x_start, out, ids, t, W,
                       dmse, dtT, B, L, E, V, sa_last, d_out, d_xs, dW, fold_t0);
  return true;
}

void launch_timestep_emb(const float* ts, int B, int dim, float max_period, uint16_t* out,
                         hipStream_t s) {
  hipLaunchKernelGGL(timestep_emb_kernel, dim3(grid_cap((int64_t)B * dim, 1024)), dim3(256), 0, s, ts,
                     B, dim, logf(max_period), (bf16_t*)out);
}

DPA_RNG_BASE_EXPORT(diffusion)

}  // namespace dpa
