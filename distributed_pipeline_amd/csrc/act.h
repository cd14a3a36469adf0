// Activation functions shared by the GEMM epilogues and the elementwise kernels.
//
// GELU is the exact (erf) form used by BERT, evaluated with the
// Abramowitz-Stegun 7.1.26 rational approximation of erf (|error| < 1.5e-7,
// far below bf16 resolution): one v_exp_f32 and one v_rcp_f32 instead of the
// libm erff, and the same exp(-z^2/2) term serves the derivative's pdf.
// Codes: 0 none, 1 gelu, 2 tanh, 3 silu; 4 = "the saved operand already IS act'(z)"
// (forward epilogues that store the derivative instead of the pre-activation, so the
// backward epilogue is one multiply instead of a second erf/exp evaluation).
#pragma once
#include <hip/hip_runtime.h>

#include "common.h"

namespace dpa {

// Phi(z) (standard normal cdf) and exp(-z^2/2)
__device__ __forceinline__ float phi_cdf(float z, float& e) {
  const float x = fabsf(z) * 0.70710678118654752f;
  e = fexp(-x * x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, x, 1.f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float erf_abs = fmaf(-p, e, 1.f);
  return 0.5f + 0.5f * copysignf(erf_abs, z);
}

__device__ __forceinline__ float gelu_f(float z) {
  float e;
  return z * phi_cdf(z, e);
}

__device__ __forceinline__ float dgelu_f(float z) {
  float e;
  const float c = phi_cdf(z, e);
  return fmaf(z * 0.39894228040143268f, e, c);
}

// Two-lane forms for the GEMM epilogues: the polynomial part runs on packed fp32
// (v_pk_fma_f32 / v_pk_mul_f32, two elements per instruction); the exp and rcp
// stay per element.  Same math as phi_cdf.
// (x = |z| / sqrt 2 folded into the constants: -x^2 log2 e = z * (-log2(e) / 2) * z, and
// 1 + 0.3275911 x = 1 + (0.3275911 / sqrt 2) |z|)
__device__ __forceinline__ f32x2 phi_cdf2(f32x2 z, f32x2& e) {
  const f32x2 az = {fabsf(z.x), fabsf(z.y)};
  const f32x2 nx2 = (z * -0.72134752044448170f) * z;
  e = f32x2{__builtin_amdgcn_exp2f(nx2.x), __builtin_amdgcn_exp2f(nx2.y)};
  const f32x2 d = az * (0.3275911f * 0.70710678118654752f) + 1.f;
  const f32x2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 p = t * 1.061405429f - 1.453152027f;
  p = p * t + 1.421413741f;
  p = p * t - 0.284496736f;
  p = p * t + 0.254829592f;
  p = p * t;
  const f32x2 ea = 1.f - p * e;
  const f32x2 sg = {copysignf(ea.x, z.x), copysignf(ea.y, z.y)};
  return sg * 0.5f + 0.5f;
}

// tanh(z) = 1 - 2 / (exp(2z) + 1): one v_exp and one v_rcp (the libm tanhf is a branchy
// polynomial); exp overflow gives 1, underflow -1; absolute error ~1e-7.  Below |z| = 2^-8
// that absolute error would be a visible relative one, and tanh(z) = z to 5e-6 there.
__device__ __forceinline__ float tanh_fast(float z) {
  const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(fexp2(z * 2.8853900817779268f) + 1.f);
  return fabsf(z) < 0.00390625f ? z : t;
}

template <int ACT>
__device__ __forceinline__ f32x2 act2(f32x2 z) {
  if constexpr (ACT == 1) {
    f32x2 e;
    return z * phi_cdf2(z, e);
  } else if constexpr (ACT == 2) {
    return f32x2{tanh_fast(z.x), tanh_fast(z.y)};
  } else if constexpr (ACT == 3) {
    const f32x2 d = {1.f + fexp(-z.x), 1.f + fexp(-z.y)};
    return z * f32x2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  } else {
    return z;
  }
}

// act(z) and act'(z) together (the shared erf/exp work done once), two lanes
template <int ACT>
__device__ __forceinline__ f32x2 act_dact2(f32x2 z, f32x2& d) {
  if constexpr (ACT == 1) {
    f32x2 e;
    const f32x2 c = phi_cdf2(z, e);
    d = z * 0.39894228040143268f * e + c;
    return z * c;
  } else if constexpr (ACT == 2) {
    const f32x2 y = {tanh_fast(z.x), tanh_fast(z.y)};
    d = 1.f - y * y;
    return y;
  } else if constexpr (ACT == 3) {
    const f32x2 den = {1.f + fexp(-z.x), 1.f + fexp(-z.y)};
    const f32x2 sg = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
    d = sg * (z * (1.f - sg) + 1.f);
    return z * sg;
  } else {
    d = f32x2{1.f, 1.f};
    return z;
  }
}

// d act / dz given aux = z (gelu, silu) or y = tanh(z) (tanh), two lanes
template <int ACT>
__device__ __forceinline__ f32x2 dact2(f32x2 a) {
  if constexpr (ACT == 4) {
    return a;
  } else if constexpr (ACT == 1) {
    f32x2 e;
    const f32x2 c = phi_cdf2(a, e);
    return a * 0.39894228040143268f * e + c;
  } else if constexpr (ACT == 2) {
    return 1.f - a * a;
  } else if constexpr (ACT == 3) {
    const f32x2 d = {1.f + fexp(-a.x), 1.f + fexp(-a.y)};
    const f32x2 sg = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
    return sg * (a * (1.f - sg) + 1.f);
  } else {
    return f32x2{1.f, 1.f};
  }
}

__device__ __forceinline__ float act_apply(float z, int act) {
  switch (act) {
    case 1: return gelu_f(z);
    case 2: return tanh_fast(z);
    case 3: return z * __builtin_amdgcn_rcpf(1.f + fexp(-z));
    default: return z;
  }
}

// d act / dz given aux = z (gelu, silu) or y = tanh(z) (tanh)
__device__ __forceinline__ float act_deriv(float a, int act) {
  switch (act) {
    case 1: return dgelu_f(a);
    case 2: return 1.f - a * a;
    case 3: {
      const float sg = __builtin_amdgcn_rcpf(1.f + fexp(-a));
      return sg * fmaf(a, 1.f - sg, 1.f);
    }
    case 4: return a;
    default: return 1.f;
  }
}

}  // namespace dpa
