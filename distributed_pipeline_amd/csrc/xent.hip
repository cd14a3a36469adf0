// Fused linear + cross-entropy for a tied rounding head (SURVEY K-M12):
//
//   logits[t][v] = x[t] . W[v] + b[v]        x: [N, E] bf16, W: [V, E] bf16
//   loss[t]      = logsumexp_v logits[t] - logits[t][target[t]]
//
// The [N, V] logits (1 GB fp32 per 8192x30522 call) are never written: every
// kernel recomputes 32x32 logit tiles on the matrix cores and consumes them
// in registers.
//
//   fwd : workgroup = 128 tokens, sweeps (a split of) the vocabulary in
//         64-row W tiles staged through LDS; S = W x^T so the token sits on
//         the MFMA lane and the vocabulary in the 16 accumulator registers:
//         the online log-sum-exp is lane-local (one cross-half merge at the end).
//   dx  : same sweep; dS = g (softmax - onehot) is rebuilt per tile and fed,
//         still in registers, as the A operand of dx = dS^T W (the W B-operand
//         comes from the same LDS tile through ds_read_b64_tr_b16).
//   dW  : workgroup = 256 vocabulary rows (W in registers), sweeps tokens in
//         64-row x tiles; S' = x W^T, dS' rebuilt, dW += dS'^T x with x read
//         transposed from LDS; partial dW / db are added with fp32 atomics
//         (token splits), two 128-B row segments per wave instruction.
//
// Out-of-range targets (< 0 or >= V) are ignored (loss 0, no gradient).
#include <cstdlib>

#include <type_traits>

#include "common.h"
#include "launchers.h"
#include "mfma.h"

namespace dpa {

static constexpr float LOG2E = 1.4426950408889634f;
static constexpr float LN2 = 0.6931471805599453f;

// ---------------------------------------------------------------------------
// W-tile staging (64 rows x E) into a swizzled LDS image, register-staged.
// ---------------------------------------------------------------------------
template <int E, int NT>
struct WTile {
  static constexpr int CH = E / 8;             // 16-byte chunks per row
  static constexpr int ROWB = E * 2;
  static constexpr int PER = 64 * CH / NT;     // chunks per thread
  uint4 r[PER];

  __device__ __forceinline__ void load(const bf16_t* __restrict__ W, int v0, int V, int tid) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * NT;
      const int row = c / CH, ch = c % CH;
      const int v = v0 + row;
      if (v < V)
        r[i] = *reinterpret_cast<const uint4*>(W + (int64_t)v * E + ch * 8);
      else
        r[i] = make_uint4(0, 0, 0, 0);
    }
  }
  __device__ __forceinline__ void store(char* lds, int tid) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * NT;
      const int row = c / CH, ch = c % CH;
      *reinterpret_cast<uint4*>(lds + swz<ROWB>(row, ch)) = r[i];
    }
  }
};

__device__ __forceinline__ float sel16(const f32x16& a, int i) {
  float v = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) v = (k == i) ? a[k] : v;
  return v;
}

// ---------------------------------------------------------------------------
// Forward
// ---------------------------------------------------------------------------
template <int E>
__global__ void __launch_bounds__(256) lxent_fwd_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ W, const bf16_t* __restrict__ bias,
    const int64_t* __restrict__ target, int N, int V, int v_per_split, float* __restrict__ loss,
    float* __restrict__ lse_out, float* __restrict__ part_m, float* __restrict__ part_s,
    float* __restrict__ tgt_logit, int xsplit) {
  constexpr int KS = E / 16, ROWB = E * 2;
  __shared__ __attribute__((aligned(16))) char smem[64 * ROWB + 64 * 4];
  char* wt = smem;
  float* bt = reinterpret_cast<float*>(smem + 64 * ROWB);

  // xsplit > 1: vocabulary split s = blockIdx.x % xsplit, i.e. (with the round-robin
  // workgroup -> XCD dispatch) every XCD sweeps only its 1/8 of W, which then stays
  // resident in that XCD's L2 instead of streaming all of W from the MALL per workgroup
  const int split = xsplit > 1 ? (int)(blockIdx.x % xsplit) : (int)blockIdx.y;
  const int tblk = xsplit > 1 ? (int)(blockIdx.x / xsplit) : (int)blockIdx.x;
  const int nsplit = xsplit > 1 ? xsplit : (int)gridDim.y;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
  const int t = tblk * 128 + w * 32 + (lane & 31);
  const bool tok_ok = t < N;
  bf16x8 xf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (tok_ok) xf[s] = ld_frag(x + (int64_t)t * E + 16 * s + 8 * h);
    else for (int j = 0; j < 8; ++j) xf[s][j] = 0;
  }
  const int64_t tg = tok_ok ? target[t] : -1;

  const int vbeg = split * v_per_split;
  const int vend = min(V, vbeg + v_per_split);
  // a block of only ignored targets (e.g. the unmasked tokens of the logged nll, sorted
  // to the end by the caller) skips the vocabulary sweep: loss 0, neutral statistics
  if (!__syncthreads_or(tg >= 0 && tg < V)) {
    if (h == 0 && tok_ok) {
      if (nsplit == 1) {
        loss[t] = 0.f;
        lse_out[t] = 0.f;
      } else {
        part_m[(int64_t)split * N + t] = 0.f;
        part_s[(int64_t)split * N + t] = 1.f;
      }
    }
    return;
  }
  float m = -1e30f, ssum = 0.f, tl = -INFINITY;

  WTile<E, 256> stage;
  if (vbeg < vend) stage.load(W, vbeg, V, tid);
  for (int v0 = vbeg; v0 < vend; v0 += 64) {
    stage.store(wt, tid);
    if (tid < 64) {
      const int v = v0 + tid;
      bt[tid] = (v < vend) ? (bias ? bf2f(bias[v]) : 0.f) : -INFINITY;
    }
    __syncthreads();
    if (v0 + 64 < vend) stage.load(W, v0 + 64, V, tid);  // prefetch next tile behind the MFMAs

    // Accumulators start at the bias of their vocabulary rows (-inf for rows past
    // the split / vocabulary), so no per-element bias add or tail test remains.
    f32x16 acc[2];
#pragma unroll
    for (int vt = 0; vt < 2; ++vt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 bv = *reinterpret_cast<const f32x4*>(bt + vt * 32 + 8 * g + 4 * h);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[vt][4 * g + r] = bv[r];
      }
#pragma unroll
      for (int s = 0; s < KS; ++s)
        acc[vt] = mfma32(lds_frag<ROWB>(wt, vt * 32 + (lane & 31), 2 * s + h), xf[s], acc[vt]);
    }
    float tmax = -INFINITY;
#pragma unroll
    for (int vt = 0; vt < 2; ++vt)
#pragma unroll
      for (int i = 0; i < 16; i += 2) tmax = fmaxf(tmax, fmaxf(acc[vt][i], acc[vt][i + 1]));
    const float mn = fmaxf(m, tmax * LOG2E);
    float add = 0.f;
#pragma unroll
    for (int vt = 0; vt < 2; ++vt)
#pragma unroll
      for (int i = 0; i < 16; ++i) add += fexp2(fmaf(acc[vt][i], LOG2E, -mn));
    ssum = ssum * fexp2(m - mn) + add;
    m = mn;
    const int64_t r = tg - v0;
    if (r >= 0 && r < 64 && v0 + r < vend) {
      const int rr = (int)r & 31, vt = (int)r >> 5;
      if (((rr >> 2) & 1) == h) {
        const int i = (rr & 3) + 4 * (rr >> 3);
        tl = vt ? sel16(acc[1], i) : sel16(acc[0], i);
      }
    }
    __syncthreads();
  }
  // merge the two lane halves that share a token
  const float m2 = __shfl_xor(m, 32, 64), s2 = __shfl_xor(ssum, 32, 64);
  const float tl2 = __shfl_xor(tl, 32, 64);
  const float M = fmaxf(m, m2);
  const float S = ssum * fexp2(m - M) + s2 * fexp2(m2 - M);
  tl = fmaxf(tl, tl2);
  if (h == 0 && tok_ok) {
    if (nsplit == 1) {
      const bool valid = tg >= 0 && tg < V;
      const float lse = (M + log2f(S)) * LN2;
      loss[t] = valid ? lse - tl : 0.f;
      lse_out[t] = lse;
    } else {
      part_m[(int64_t)split * N + t] = M;
      part_s[(int64_t)split * N + t] = S;
      if (tl > -INFINITY) tgt_logit[t] = tl;
    }
  }
}

__global__ void __launch_bounds__(256) lxent_combine_kernel(
    const float* __restrict__ part_m, const float* __restrict__ part_s,
    const float* __restrict__ tgt_logit, const int64_t* __restrict__ target, int N, int V, int S,
    float* __restrict__ loss, float* __restrict__ lse_out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N) return;
  float M = -1e30f;
  for (int s = 0; s < S; ++s) M = fmaxf(M, part_m[(int64_t)s * N + t]);
  float sum = 0.f;
  for (int s = 0; s < S; ++s) sum += part_s[(int64_t)s * N + t] * fexp2(part_m[(int64_t)s * N + t] - M);
  const float lse = (M + log2f(sum)) * LN2;
  const int64_t tg = target[t];
  const bool valid = tg >= 0 && tg < V;
  loss[t] = valid ? lse - tgt_logit[t] : 0.f;
  lse_out[t] = lse;
}

// ---------------------------------------------------------------------------
// Backward: dx
// ---------------------------------------------------------------------------
template <int E>
__global__ void __launch_bounds__(256) lxent_dx_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ W, const bf16_t* __restrict__ bias,
    const int64_t* __restrict__ target, const float* __restrict__ lse, const float* __restrict__ dloss,
    int N, int V, int v_per_split, bf16_t* __restrict__ dx, float* __restrict__ dx_acc) {
  constexpr int KS = E / 16, ROWB = E * 2, KT = E / 32;
  __shared__ __attribute__((aligned(16))) char smem[64 * ROWB + 64 * 4];
  char* wt = smem;
  float* bt = reinterpret_cast<float*>(smem + 64 * ROWB);

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
  const int t = blockIdx.x * 128 + w * 32 + (lane & 31);
  const bool tok_ok = t < N;
  bf16x8 xf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (tok_ok) xf[s] = ld_frag(x + (int64_t)t * E + 16 * s + 8 * h);
    else for (int j = 0; j < 8; ++j) xf[s][j] = 0;
  }
  const int64_t tg = tok_ok ? target[t] : -1;
  const bool valid = tok_ok && tg >= 0 && tg < V;
  const float g = valid ? dloss[t] : 0.f;
  const float lse2 = tok_ok ? lse[t] * LOG2E : 0.f;

  const int vbeg = blockIdx.y * v_per_split;
  const int vend = min(V, vbeg + v_per_split);
  f32x16 dacc[KT];
#pragma unroll
  for (int k = 0; k < KT; ++k) dacc[k] = zero16();

  WTile<E, 256> stage;
  if (vbeg < vend) stage.load(W, vbeg, V, tid);
  for (int v0 = vbeg; v0 < vend; v0 += 64) {
    stage.store(wt, tid);
    if (tid < 64) {
      const int v = v0 + tid;
      bt[tid] = (v < vend) ? (bias ? bf2f(bias[v]) : 0.f) : -INFINITY;
    }
    __syncthreads();
    if (v0 + 64 < vend) stage.load(W, v0 + 64, V, tid);

#pragma unroll
    for (int vt = 0; vt < 2; ++vt) {
      f32x16 acc;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const f32x4 bv = *reinterpret_cast<const f32x4*>(bt + vt * 32 + 8 * g4 + 4 * h);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[4 * g4 + r] = bv[r];
      }
#pragma unroll
      for (int s = 0; s < KS; ++s)
        acc = mfma32(lds_frag<ROWB>(wt, vt * 32 + (lane & 31), 2 * s + h), xf[s], acc);
      // dS = g * (softmax - onehot(target)); rows past the split come out as 0
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = g * fexp2(fmaf(acc[i], LOG2E, -lse2));
      const int64_t rt = tg - (v0 + vt * 32);
      if (rt >= 0 && rt < 32 && tg < vend && ((rt >> 2) & 1) == h) {
        const int it = ((int)rt & 3) + 4 * ((int)rt >> 3);
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] -= (i == it) ? g : 0.f;
      }
      // dx[t][k] += sum_v dS[v][t] W[v][k]   (dS as A operand, W read transposed)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 af = acc_to_frag(acc, s);
#pragma unroll
        for (int kt = 0; kt < KT; ++kt)
          dacc[kt] = mfma32(af, lds_tr_frag<ROWB>(wt, vt * 32 + 16 * s, kt * 32, lane), dacc[kt]);
      }
    }
    __syncthreads();
  }
  // dacc[kt] reg i: row = token (w*32 + acc_row(i,h)), col = k (kt*32 + lane&31)
  const int tb = blockIdx.x * 128 + w * 32;
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
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
}

// ---------------------------------------------------------------------------
// Forward + input gradient in one vocabulary sweep (training): the loss of token t
// is lse_t - s_t[target], and its gradient w.r.t. x_t does not depend on the upstream
// scalar g_t except as a factor:  dx_t = g_t (sum_v p_tv W_v - W_target).  So the
// forward accumulates  u_t = sum_v exp(s_tv - m_t) W_v  with an online max m_t (the
// flash-attention recurrence; lazy rescale, |growth| <= 2^8 between rescales) and
// writes dxu_t = u_t / l_t - W_target in fp32; the backward only multiplies by g_t.
// Versus lxent_fwd + lxent_dx this removes one full recompute of the logits and their
// exponentials (the dx kernel's S = W x^T pass).
// ---------------------------------------------------------------------------
template <int E>
__global__ void __launch_bounds__(256, E == 128 ? 2 : 1) lxent_fwd_dx_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ W, const bf16_t* __restrict__ bias,
    const int64_t* __restrict__ target, int N, int V, float* __restrict__ loss,
    float* __restrict__ lse_out, float* __restrict__ dxu, int vps, float* __restrict__ part) {
  constexpr int KS = E / 16, ROWB = E * 2, KT = E / 32;
  __shared__ __attribute__((aligned(16))) char smem[64 * ROWB + 64 * 4];
  // vocabulary split (part != nullptr, few token blocks): this block sweeps rows
  // [v_lo, v_hi) and leaves (m, l, target logit, unnormalised u) for lxent_fwd_dx_combine
  const int v_lo = part ? (int)blockIdx.y * vps : 0;
  const int v_hi = part ? min(V, v_lo + vps) : V;
  char* wt = smem;
  float* bt = reinterpret_cast<float*>(smem + 64 * ROWB);

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
  const int t = blockIdx.x * 128 + w * 32 + (lane & 31);
  const bool tok_ok = t < N;
  bf16x8 xf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (tok_ok) xf[s] = ld_frag(x + (int64_t)t * E + 16 * s + 8 * h);
    else for (int j = 0; j < 8; ++j) xf[s][j] = 0;
  }
  const int64_t tg = tok_ok ? target[t] : -1;
  f32x16 dacc[KT];
#pragma unroll
  for (int k = 0; k < KT; ++k) dacc[k] = zero16();
  float m = -1e30f, l = 0.f, tl = -INFINITY;  // m in the log2 domain

  WTile<E, 256> stage;
  stage.load(W, v_lo, V, tid);
  for (int v0 = v_lo; v0 < v_hi; v0 += 64) {
    stage.store(wt, tid);
    if (tid < 64) {
      const int v = v0 + tid;
      bt[tid] = (v < v_hi) ? (bias ? bf2f(bias[v]) : 0.f) : -INFINITY;
    }
    __syncthreads();
    if (v0 + 64 < v_hi) stage.load(W, v0 + 64, V, tid);  // prefetch behind the MFMAs

    // one 32-row vocabulary subtile at a time (a single live logit accumulator keeps
    // the kernel at 2 waves / SIMD); each subtile is one online-softmax step
#pragma unroll
    for (int vt = 0; vt < 2; ++vt) {
      f32x16 acc;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 bv = *reinterpret_cast<const f32x4*>(bt + vt * 32 + 8 * g + 4 * h);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[4 * g + r] = bv[r];
      }
#pragma unroll
      for (int s = 0; s < KS; ++s)
        acc = mfma32(lds_frag<ROWB>(wt, vt * 32 + (lane & 31), 2 * s + h), xf[s], acc);
      // the target's logit, from whichever lane half holds its row
      const int64_t r = tg - (v0 + vt * 32);
      if (r >= 0 && r < 32 && ((((int)r >> 2) & 1) == h)) tl = sel16(acc, ((int)r & 3) + 4 * ((int)r >> 3));
      // running max over both lane halves of the token (they feed the same dacc rows)
      float tmax = -INFINITY;
#pragma unroll
      for (int i = 0; i < 16; ++i) tmax = fmaxf(tmax, acc[i]);
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64)) * LOG2E;
      if (__any(tmax > m + 8.f)) {
        const float mn = fmaxf(m, tmax);
        const float alpha = fexp2(m - mn);
        m = mn;
        l *= alpha;
        // dacc rows are tokens (register i <-> token acc_row(i, h)): fetch their alpha
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float f = __shfl(alpha, acc_row(i, h), 64);
#pragma unroll
          for (int kt = 0; kt < KT; ++kt) dacc[kt][i] *= f;
        }
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float pr = fexp2(fmaf(acc[i], LOG2E, -m));
        l += pr;
        acc[i] = pr;
      }
      // u[t][k] += sum_v p[v][t] W[v][k]   (p as A operand, W read transposed)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 af = acc_to_frag(acc, s);
#pragma unroll
        for (int kt = 0; kt < KT; ++kt)
          dacc[kt] = mfma32(af, lds_tr_frag<ROWB>(wt, vt * 32 + 16 * s, kt * 32, lane), dacc[kt]);
      }
    }
    __syncthreads();
  }
  l += __shfl_xor(l, 32, 64);
  tl = fmaxf(tl, __shfl_xor(tl, 32, 64));
  if (part) {
    const int S = gridDim.y, sp = blockIdx.y;
    float* pm = part;
    float* pl = pm + (int64_t)S * N;
    float* pt = pl + (int64_t)S * N;
    float* pu = pt + (int64_t)S * N;
    if (h == 0 && tok_ok) {
      pm[(int64_t)sp * N + t] = m;
      pl[(int64_t)sp * N + t] = l;
      pt[(int64_t)sp * N + t] = tl;
    }
    const int tb0 = blockIdx.x * 128 + w * 32;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int tt = tb0 + acc_row(i, h);
      if (tt < N) {
#pragma unroll
        for (int kt = 0; kt < KT; ++kt) pu[((int64_t)sp * N + tt) * E + kt * 32 + (lane & 31)] = dacc[kt][i];
      }
    }
    return;
  }
  const bool valid = tok_ok && tg >= 0 && tg < V;
  const float lse = (m + log2f(l)) * LN2;
  if (h == 0 && tok_ok) {
    loss[t] = valid ? lse - tl : 0.f;
    lse_out[t] = lse;
  }
  // dxu[t][k] = u[t][k] / l_t - W[target_t][k]   (0 for ignored targets)
  const float inv_l = valid ? 1.f / l : 0.f;
  const int tb = blockIdx.x * 128 + w * 32;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int src = acc_row(i, h);
    const float f = __shfl(inv_l, src, 64);
    const int64_t tgi = __shfl(tg, src, 64);
    const int tt = tb + src;
    if (tt < N) {
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        const int k = kt * 32 + (lane & 31);
        float vv = 0.f;
        if (f != 0.f) vv = dacc[kt][i] * f - bf2f(W[tgi * E + k]);
        dxu[(int64_t)tt * E + k] = vv;
      }
    }
  }
}

// Merge of the vocabulary splits of lxent_fwd_dx_kernel: per token the split maxima
// (log2 domain) give M, L = sum_s l_s 2^(m_s - M), lse = (M + log2 L) ln 2, and
// dxu = sum_s 2^(m_s - M) u_s / L - W[target].  One thread per (token, column).
template <int E>
__global__ void __launch_bounds__(256) lxent_fwd_dx_combine_kernel(
    const float* __restrict__ part, int S, const bf16_t* __restrict__ W, const int64_t* __restrict__ target,
    int N, int V, float* __restrict__ loss, float* __restrict__ lse_out, float* __restrict__ dxu) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)N * E) return;
  const int t = (int)(idx / E), k = (int)(idx % E);
  const float* pm = part;
  const float* pl = pm + (int64_t)S * N;
  const float* pt = pl + (int64_t)S * N;
  const float* pu = pt + (int64_t)S * N;
  float M = -1e30f, tl = -INFINITY;
  for (int s = 0; s < S; ++s) {
    M = fmaxf(M, pm[(int64_t)s * N + t]);
    tl = fmaxf(tl, pt[(int64_t)s * N + t]);
  }
  float L = 0.f, u = 0.f;
  for (int s = 0; s < S; ++s) {
    const float f = fexp2(pm[(int64_t)s * N + t] - M);
    L += pl[(int64_t)s * N + t] * f;
    u += pu[((int64_t)s * N + t) * E + k] * f;
  }
  const int64_t tg = target[t];
  const bool valid = tg >= 0 && tg < V;
  const float lse = (M + log2f(L)) * LN2;
  if (k == 0) {
    loss[t] = valid ? lse - tl : 0.f;
    lse_out[t] = lse;
  }
  dxu[(int64_t)t * E + k] = valid ? u / L - bf2f(W[tg * E + k]) : 0.f;
}

// ---------------------------------------------------------------------------
// Backward: dW (+ db)
// ---------------------------------------------------------------------------
// ONEHOT: subtract the target's one-hot inside the kernel (a compare, subtract and select per
// logit); false: the caller adds dW[target] -= g x and db[target] -= g as a sorted scatter
// (bindings.cpp lxent_bwd), which leaves the per-logit work at exp, scale and column sum.
template <int E, bool ONEHOT = true>
__global__ void __launch_bounds__(512) lxent_dw_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ W, const bf16_t* __restrict__ bias,
    const int64_t* __restrict__ target, const float* __restrict__ lse, const float* __restrict__ dloss,
    int N, int V, int t_per_split, float* __restrict__ dW, float* __restrict__ db, float* __restrict__ ws) {
  constexpr int KS = E / 16, ROWB = E * 2, KT = E / 32, CH = E / 8;
  __shared__ __attribute__((aligned(16))) char smem[64 * ROWB + 3 * 64 * 4];
  char* xt = smem;
  float* s_lse = reinterpret_cast<float*>(smem + 64 * ROWB);
  float* s_g = s_lse + 64;
  int* s_tg = reinterpret_cast<int*>(s_g + 64);

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
  // waves w and w + 4 share a SIMD and run the same MFMA -> VALU -> MFMA chain between the same
  // barriers; a static priority for the first lets it run ahead, so the second's VALU work
  // fills the first's MFMA phases instead of colliding with its own
  if (w < 4) __builtin_amdgcn_s_setprio(1);
  const int vw = blockIdx.x * 256 + w * 32;       // this wave's 32 vocabulary rows
  const int v = vw + (lane & 31);                 // this lane's column (vocab)
  const bool v_ok = v < V;
  bf16x8 wf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (v_ok) wf[s] = ld_frag(W + (int64_t)v * E + 16 * s + 8 * h);
    else for (int j = 0; j < 8; ++j) wf[s][j] = 0;
  }
  // rows past the vocabulary start at -inf: their softmax (and gradient) is 0
  const float bv = v_ok ? (bias ? bf2f(bias[v]) : 0.f) : -INFINITY;

  f32x16 dacc[KT];
#pragma unroll
  for (int k = 0; k < KT; ++k) dacc[k] = zero16();
  float dbs = 0.f;

  const int tbeg = blockIdx.y * t_per_split;
  const int tend = min(N, tbeg + t_per_split);
  // x tile [64 tokens][E] + per-token scalars, register-staged one tile ahead so the
  // global loads of tile i+1 fly behind the MFMAs of tile i
  constexpr int PER = 64 * CH / 512;
  uint4 xr[PER];
  float r_lse = 0.f, r_g = 0.f;
  int r_tg = -1;
  auto load_tile = [&](int t0) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * 512;
      const int t = t0 + c / CH;
      xr[i] = t < tend ? *reinterpret_cast<const uint4*>(x + (int64_t)t * E + (c % CH) * 8)
                       : make_uint4(0, 0, 0, 0);
    }
    if (tid < 64) {
      const int t = t0 + tid;
      const bool ok = t < tend;
      const int64_t tg = ok ? target[t] : -1;
      const bool valid = ok && tg >= 0 && tg < V;
      r_lse = ok ? lse[t] * LOG2E : 0.f;
      r_g = valid ? dloss[t] : 0.f;
      r_tg = valid ? (int)tg : -1;
    }
  };
  if (tbeg < tend) load_tile(tbeg);
  for (int t0 = tbeg; t0 < tend; t0 += 64) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * 512;
      *reinterpret_cast<uint4*>(xt + swz<ROWB, true>(c / CH, c % CH)) = xr[i];
    }
    if (tid < 64) {
      s_lse[tid] = r_lse;
      s_g[tid] = r_g;
      s_tg[tid] = r_tg;
    }
    __syncthreads();
    if (t0 + 64 < tend) load_tile(t0 + 64);
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      f32x16 acc;  // S'[t][v]: rows = tokens, cols = vocab (lane); starts at the bias
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = bv;
#pragma unroll
      for (int s = 0; s < KS; ++s)
        acc = mfma32(lds_frag<ROWB, true>(xt, tt * 32 + (lane & 31), 2 * s + h), wf[s], acc);
      // the one-hot term lands on (token, vocab row) pairs whose target is one of this wave's 32
      // rows: ~32 x 32 / V of the subtiles (3% at V = 30522).  One wave-uniform test per subtile
      // (lane l checks token l) lets the others skip the per-logit compare and select.
      auto softmax_grad = [&](auto oh) {
        constexpr bool OH = decltype(oh)::value;
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          // per-token scalars of rows tt*32 + 8 g4 + 4 h + r, one 16-byte read each
          const int rb = tt * 32 + 8 * g4 + 4 * h;
          const f32x4 l4 = *reinterpret_cast<const f32x4*>(s_lse + rb);
          const f32x4 g4v = *reinterpret_cast<const f32x4*>(s_g + rb);
          int tgs[4] = {-1, -1, -1, -1};
          if constexpr (OH) {
            const int4 t4 = *reinterpret_cast<const int4*>(s_tg + rb);
            tgs[0] = t4.x; tgs[1] = t4.y; tgs[2] = t4.z; tgs[3] = t4.w;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = 4 * g4 + r;
            const float gp = g4v[r] * fexp2(fmaf(acc[i], LOG2E, -l4[r]));
            const float d = (OH && tgs[r] == v) ? gp - g4v[r] : gp;
            acc[i] = d;
            dbs += d;
          }
        }
      };
      bool hit = false;
      if constexpr (ONEHOT) {
        const int tgl = s_tg[tt * 32 + (lane & 31)];
        hit = __any(tgl >= vw && tgl < vw + 32);
      }
      if (hit) softmax_grad(std::true_type{});
      else softmax_grad(std::false_type{});
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 af = acc_to_frag(acc, s);
#pragma unroll
        for (int kt = 0; kt < KT; ++kt)
          dacc[kt] = mfma32(af, lds_tr_frag<ROWB, true>(xt, tt * 32 + 16 * s, kt * 32, lane), dacc[kt]);
      }
    }
    __syncthreads();
  }
  dbs += __shfl_xor(dbs, 32, 64);
  // ws: this token split's partials, plain stores into slab blockIdx.y ([V][E] then [V] for the
  // bias), summed in split order by xent_split_reduce_kernel - deterministic.  Without ws (one
  // token split) the block is the only adder of its rows.
  float* const pw = ws ? ws + (int64_t)blockIdx.y * V * (E + 1) : nullptr;
  if (h == 0 && v_ok && db) {
    if (pw) pw[(int64_t)V * E + v] = dbs;
    else db[v] += dbs;
  }
  // dacc[kt] reg i: row = vocab vw + acc_row(i,h), col = k
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int vv = vw + acc_row(i, h);
      if (vv < V) {
        const int64_t o = (int64_t)vv * E + kt * 32 + (lane & 31);
        if (pw) pw[o] = dacc[kt][i];
        else dW[o] += dacc[kt][i];
      }
    }
  }
}

// dst[i] += sum_s slab_s[i] in split order (slabs of `stride` floats; i < n)
__global__ void __launch_bounds__(256) xent_split_reduce_kernel(const float* __restrict__ ws, int64_t stride,
                                                                int splits, int64_t n, float* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float a = dst[i];
  for (int sp = 0; sp < splits; ++sp) a += ws[(int64_t)sp * stride + i];
  dst[i] = a;
}

__global__ void __launch_bounds__(256) f32_to_bf16_kernel(const float* __restrict__ a,
                                                         bf16_t* __restrict__ b, int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 3 < n) {
    f32x4 v = *reinterpret_cast<const f32x4*>(a + i);
    uint2 p;
    p.x = pack_bf2(v[0], v[1]);
    p.y = pack_bf2(v[2], v[3]);
    *reinterpret_cast<uint2*>(b + i) = p;
  } else {
    for (int64_t k = i; k < n; ++k) b[k] = f2bf(a[k]);
  }
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
static int pick_splits(int blocks, int chunks, int target_wgs) {
  int s = (target_wgs + blocks - 1) / blocks;
  if (s < 1) s = 1;
  if (s > chunks) s = chunks;
  return s;
}

// vocabulary splits of the forward: at least 8 (one per XCD, see the kernel) once the
// vocabulary has 8 x 64 rows, more when there are too few token blocks to fill the chip
static int fwd_splits(int N, int V) {
  const int tb = (N + 127) / 128;
  const int vchunks = (V + 63) / 64;
  int S = pick_splits(tb, vchunks, 1024);
  constexpr int xs = 8;
  if (xs > 1 && vchunks >= xs) S = (S + xs - 1) / xs * xs;
  return S;
}

template <int E>
static void fwd_impl(const bf16_t* x, const bf16_t* W, const bf16_t* b, const int64_t* tgt, int N,
                     int V, float* loss, float* lse, float* ws, hipStream_t st) {
  const int tb = (N + 127) / 128;
  const int vchunks = (V + 63) / 64;
  const int S = fwd_splits(N, V);
  const int vps = ((vchunks + S - 1) / S) * 64;
  const int Sx = (V + vps - 1) / vps;
  float* pm = ws;
  float* ps = ws + (int64_t)Sx * N;
  float* tl = ws + 2 * (int64_t)Sx * N;
  if (Sx == 8)  // one split per XCD: 1-D grid, split = blockIdx % 8
    hipLaunchKernelGGL(lxent_fwd_kernel<E>, dim3(tb * 8), dim3(256), 0, st, x, W, b, tgt, N, V, vps, loss,
                       lse, pm, ps, tl, 8);
  else
    hipLaunchKernelGGL(lxent_fwd_kernel<E>, dim3(tb, Sx), dim3(256), 0, st, x, W, b, tgt, N, V, vps, loss,
                       lse, pm, ps, tl, 0);
  if (Sx > 1)
    hipLaunchKernelGGL(lxent_combine_kernel, dim3((N + 255) / 256), dim3(256), 0, st, pm, ps, tl,
                       tgt, N, V, Sx, loss, lse);
}

// Vocabulary splits of the fused forward + dx: one block per 128 tokens sweeps the whole
// vocabulary, so below ~3 blocks per CU (a reference-schedule micro-batch: 8192 tokens =
// 64 blocks for 256 CUs) the vocabulary is split over gridDim.y and merged afterwards.
static void fwd_dx_plan(int N, int V, int& S, int& vps) {
  const int tb = (N + 127) / 128, vchunks = (V + 63) / 64;
  S = 1;
  vps = vchunks * 64;
  if (tb >= 768) return;
  int want = (768 + tb - 1) / tb;
  if (want > vchunks) want = vchunks;
  if (want < 2) return;
  vps = ((vchunks + want - 1) / want) * 64;
  S = (V + vps - 1) / vps;
}

int64_t lxent_fwd_dx_workspace_floats(int N, int V, int E) {
  int S, vps;
  fwd_dx_plan(N, V, S, vps);
  return S > 1 ? (int64_t)S * N * (3 + E) : 0;
}

template <int E>
static void fwd_dx_impl(const bf16_t* x, const bf16_t* W, const bf16_t* b, const int64_t* tgt, int N, int V,
                        float* loss, float* lse, float* dxu, float* ws, hipStream_t s) {
  const unsigned tb = (unsigned)((N + 127) / 128);
  int S, vps;
  fwd_dx_plan(N, V, S, vps);
  if (S > 1 && ws != nullptr) {
    hipLaunchKernelGGL(lxent_fwd_dx_kernel<E>, dim3(tb, S), dim3(256), 0, s, x, W, b, tgt, N, V, loss, lse,
                       dxu, vps, ws);
    const int64_t n = (int64_t)N * E;
    hipLaunchKernelGGL(lxent_fwd_dx_combine_kernel<E>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, ws,
                       S, W, tgt, N, V, loss, lse, dxu);
  } else {
    hipLaunchKernelGGL(lxent_fwd_dx_kernel<E>, dim3(tb), dim3(256), 0, s, x, W, b, tgt, N, V, loss, lse, dxu,
                       V, nullptr);
  }
}

void launch_lxent_fwd_dx(const uint16_t* x, const uint16_t* W, const uint16_t* b, const int64_t* tgt,
                         int N, int V, int E, float* loss, float* lse, float* dxu, hipStream_t s, float* ws) {
  if (E == 128)
    fwd_dx_impl<128>((const bf16_t*)x, (const bf16_t*)W, (const bf16_t*)b, tgt, N, V, loss, lse, dxu, ws, s);
  else
    fwd_dx_impl<256>((const bf16_t*)x, (const bf16_t*)W, (const bf16_t*)b, tgt, N, V, loss, lse, dxu, ws, s);
}

int64_t lxent_workspace_floats(int N, int V) {
  const int vchunks = (V + 63) / 64;
  const int S = fwd_splits(N, V);
  const int vps = ((vchunks + S - 1) / S) * 64;
  const int Sx = (V + vps - 1) / vps;
  return (2 * (int64_t)Sx + 1) * N + 64;
}

void launch_lxent_fwd(const uint16_t* x, const uint16_t* W, const uint16_t* b, const int64_t* tgt,
                      int N, int V, int E, float* loss, float* lse, float* ws, hipStream_t s) {
  if (E == 128) fwd_impl<128>(x, W, b, tgt, N, V, loss, lse, ws, s);
  else fwd_impl<256>(x, W, b, tgt, N, V, loss, lse, ws, s);
}

template <int E>
static void dx_impl(const bf16_t* x, const bf16_t* W, const bf16_t* b, const int64_t* tgt,
                    const float* lse, const float* dl, int N, int V, uint16_t* dx, float* dx_acc,
                    hipStream_t st) {
  const int tb = (N + 127) / 128;
  const int vchunks = (V + 63) / 64;
  const int S = dx_acc ? pick_splits(tb, vchunks, 1024) : 1;
  const int vps = ((vchunks + S - 1) / S) * 64;
  const int Sx = (V + vps - 1) / vps;
  hipLaunchKernelGGL(lxent_dx_kernel<E>, dim3(tb, Sx), dim3(256), 0, st, x, W, b, tgt, lse, dl, N, V,
                     vps, (bf16_t*)dx, Sx > 1 ? dx_acc : nullptr);
  if (Sx > 1) {
    const int64_t n = (int64_t)N * E;
    hipLaunchKernelGGL(f32_to_bf16_kernel, dim3((unsigned)((n / 4 + 255) / 256 + 1)), dim3(256), 0,
                       st, dx_acc, (bf16_t*)dx, n);
  }
}

bool lxent_dx_needs_acc(int N) { return (N + 127) / 128 < 512; }

void launch_lxent_dx(const uint16_t* x, const uint16_t* W, const uint16_t* b, const int64_t* tgt,
                     const float* lse, const float* dloss, int N, int V, int E, uint16_t* dx,
                     float* dx_acc, hipStream_t s) {
  if (E == 128) dx_impl<128>(x, W, b, tgt, lse, dloss, N, V, dx, dx_acc, s);
  else dx_impl<256>(x, W, b, tgt, lse, dloss, N, V, dx, dx_acc, s);
}

// token splits of the weight-gradient kernel (enough workgroups to fill the chip)
static void lxent_dw_plan(int N, int V, int& vb, int& tps, int& TSx) {
  vb = (V + 255) / 256;
  const int tchunks = (N + 63) / 64;
  const int TS = pick_splits(vb, tchunks, 960);
  tps = ((tchunks + TS - 1) / TS) * 64;
  TSx = (N + tps - 1) / tps;
}

int64_t lxent_dw_ws_floats(int N, int V, int E) {
  int vb, tps, TSx;
  lxent_dw_plan(N, V, vb, tps, TSx);
  return TSx > 1 ? (int64_t)TSx * V * (E + 1) : 0;
}

// ws: lxent_dw_ws_floats of scratch (the token splits' partials, reduced in order: the tied
// embedding's head gradient is bitwise reproducible); required when that is > 0
void launch_lxent_dw(const uint16_t* x, const uint16_t* W, const uint16_t* b, const int64_t* tgt,
                     const float* lse, const float* dloss, int N, int V, int E, float* dW, float* db,
                     hipStream_t s, bool onehot, float* ws) {
  int vb, tps, TSx;
  lxent_dw_plan(N, V, vb, tps, TSx);
  float* wsp = TSx > 1 ? ws : nullptr;
#define DPA_LXDW(EE, OH)                                                                                \
  hipLaunchKernelGGL((lxent_dw_kernel<EE, OH>), dim3(vb, TSx), dim3(512), 0, s, (const bf16_t*)x,        \
                     (const bf16_t*)W, (const bf16_t*)b, tgt, lse, dloss, N, V, tps, dW, db, wsp)
  if (E == 128) {
    if (onehot) DPA_LXDW(128, true); else DPA_LXDW(128, false);
  } else {
    if (onehot) DPA_LXDW(256, true); else DPA_LXDW(256, false);
  }
#undef DPA_LXDW
  if (wsp) {
    const int64_t stride = (int64_t)V * (E + 1), nw = (int64_t)V * E;
    hipLaunchKernelGGL(xent_split_reduce_kernel, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s,
                       (const float*)wsp, stride, TSx, nw, dW);
    if (db)
      hipLaunchKernelGGL(xent_split_reduce_kernel, dim3((unsigned)((V + 255) / 256)), dim3(256), 0, s,
                         (const float*)(wsp + nw), stride, TSx, (int64_t)V, db);
  }
}

}  // namespace dpa
