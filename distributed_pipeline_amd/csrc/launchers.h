// Host-side launch entry points of the gfx950 kernels.  Kernels live in the
// .hip translation units (which include no torch headers, so they compile in
// seconds); bindings.cpp is the only TU that sees ATen.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dpa {

// ---- optim.hip -------------------------------------------------------------
void launch_sqnorm(const void* g, bool g_bf16, int64_t n, float* partial, int nparts, float scale,
                   float max_norm, float* out, hipStream_t s);
void launch_adamw_ema(float* p, const void* g, bool g_bf16, float* m, float* v, uint16_t* p16,
                      float* const* ema_bufs, const float* ema_rates, int n_ema, int64_t n, float lr,
                      float beta1, float beta2, float eps, float wd, int64_t step, float grad_scale,
                      const float* clip, hipStream_t s);
void launch_ema(float* e, const float* p, int64_t n, float rate, hipStream_t s);
void launch_cast_bf16(const float* src, uint16_t* dst, int64_t n, hipStream_t s);

}  // namespace dpa
