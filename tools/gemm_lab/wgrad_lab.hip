// Weight-gradient lab: the production split-K 8-phase kernel (gemm256_kernel<true, true, 2>,
// launch_gemm256_wgrad) against the one-wave-per-SIMD kernel (csrc/wgrad4w.hip) on the
// DiffuSeq-base Linear shapes at T tokens, same split-K plan (gemm256.hip wgrad_plan), same
// workspace merge, interleaved rounds on uniform random bf16; checks both against each other and
// an fp32 reference on sampled entries.
//
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../distributed_pipeline_amd/csrc wgrad_lab.hip -o wgrad_lab
// run:   ./wgrad_lab [T] [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "gemm.hip"
#include "gemm256.hip"
#include "wgrad4w.hip"

#define CK(x)                                                                                     \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) {                                                                       \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);      \
      exit(1);                                                                                    \
    }                                                                                             \
  } while (0)

__global__ void fill_rand(uint16_t* p, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    p[i] = dpa::f2bf(((x >> 8) * (1.0f / 16777216.0f) * 2.f - 1.f));
  }
}

// ref[s] = sum_t A[t][m_s] B[t][n_s] for sampled (m_s, n_s); one block per sample
__global__ void ref_entries(const uint16_t* A, const uint16_t* B, int T, int M, int N, const int* mn, float* out) {
  __shared__ float red[256];
  const int m = mn[2 * blockIdx.x], n = mn[2 * blockIdx.x + 1];
  float s = 0.f;
  for (int t = threadIdx.x; t < T; t += blockDim.x)
    s += dpa::bf2f(A[(int64_t)t * M + m]) * dpa::bf2f(B[(int64_t)t * N + n]);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}

struct Shape { const char* name; int M, N; };

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 262144;
  const int rounds = argc > 2 ? atoi(argv[2]) : 7;
  const Shape shapes[] = {{"qkv", 2304, 768}, {"attn_out", 768, 768}, {"ffn_in", 3072, 768}, {"ffn_out", 768, 3072}};
  uint16_t *A, *B;
  CK(hipMalloc(&A, (size_t)T * 3072 * 2));
  CK(hipMalloc(&B, (size_t)T * 3072 * 2));
  hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, A, (int64_t)T * 3072, 1u);
  hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, B, (int64_t)T * 3072, 2u);
  float *W0, *W1, *ws, *ref;
  CK(hipMalloc(&W0, (size_t)3072 * 768 * 4));
  CK(hipMalloc(&W1, (size_t)3072 * 768 * 4));
  CK(hipMalloc(&ref, 64 * 4));
  int* mn;
  CK(hipMalloc(&mn, 128 * 4));
  size_t wsmax = 0;
  for (const Shape& sh : shapes)
    wsmax = std::max(wsmax, (size_t)dpa::gemm256_wgrad_workspace_floats(T, sh.M, sh.N, 1));
  CK(hipMalloc(&ws, std::max<size_t>(wsmax, 1) * 4));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("T %d, CUs %d\n", T, dpa::device_cu_count());
  dpa::set_wgrad4w(false);  // "old" = launch_gemm256_wgrad on the 8-phase kernel
  for (const Shape& sh : shapes) {
    const int M = sh.M, N = sh.N;
    const dpa::WgradPlan p = dpa::wgrad_plan(T, M, N);
    const double fl = 2.0 * T * M * N;
    auto old_k = [&](float* dW) { dpa::launch_gemm256_wgrad(A, B, dW, nullptr, T, M, N, s, ws); };
    auto new_k = [&](float* dW) {
      const uint16_t* as[1] = {A};
      const uint16_t* bs[1] = {B};
      float* wsp = p.ws ? ws : nullptr;
      if (!dpa::launch_wgrad4w(as, bs, 1, T, M, N, p.splits, p.kps, dW, wsp, s)) {
        fprintf(stderr, "launch_wgrad4w refused\n");
        exit(1);
      }
      if (wsp) {
        const int64_t n4 = (int64_t)M * N / 4;
        hipLaunchKernelGGL(dpa::wgrad_reduce_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, wsp, dW, n4,
                           p.splits);
      }
    };
    // correctness: both from zero, then sampled fp32 reference
    CK(hipMemsetAsync(W0, 0, (size_t)M * N * 4, s));
    CK(hipMemsetAsync(W1, 0, (size_t)M * N * 4, s));
    old_k(W0);
    new_k(W1);
    std::vector<int> hmn(128);
    for (int i = 0; i < 64; ++i) {
      hmn[2 * i] = (int)((uint64_t)(i * 7919 + 13) * 2654435761u % M);
      hmn[2 * i + 1] = (int)((uint64_t)(i * 104729 + 7) * 2246822519u % N);
    }
    CK(hipMemcpy(mn, hmn.data(), 128 * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(ref_entries, dim3(64), dim3(256), 0, s, A, B, T, M, N, mn, ref);
    CK(hipStreamSynchronize(s));
    std::vector<float> h0((size_t)M * N), h1((size_t)M * N), hr(64);
    CK(hipMemcpy(h0.data(), W0, (size_t)M * N * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h1.data(), W1, (size_t)M * N * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hr.data(), ref, 64 * 4, hipMemcpyDeviceToHost));
    double dmax = 0, amax = 0, rerr = 0, rmax = 0;
    for (size_t i = 0; i < h0.size(); ++i) {
      dmax = std::max(dmax, (double)fabsf(h0[i] - h1[i]));
      amax = std::max(amax, (double)fabsf(h0[i]));
    }
    for (int i = 0; i < 64; ++i) {
      const size_t idx = (size_t)hmn[2 * i] * N + hmn[2 * i + 1];
      rerr = std::max(rerr, (double)fabsf(h1[idx] - hr[i]));
      rmax = std::max(rmax, (double)fabsf(hr[i]));
    }
    printf("check %-9s splits %d kps %d ws %d: new vs old max %.3e (rel %.3e), new vs fp32 ref rel %.3e\n", sh.name,
           p.splits, p.kps, (int)p.ws, dmax, dmax / (amax + 1e-30), rerr / (rmax + 1e-30));
    // timing, interleaved
    std::vector<float> t_old, t_new;
    for (int r = 0; r < rounds; ++r) {
      for (int v = 0; v < 2; ++v) {
        CK(hipEventRecord(e0, s));
        for (int k = 0; k < 5; ++k) {
          if (v) new_k(W1);
          else old_k(W0);
        }
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        (v ? t_new : t_old).push_back(ms / 5);
      }
    }
    auto med = [](std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
    const float mo = med(t_old), mnw = med(t_new);
    printf("%-9s old %.4f ms %.1f TF/s | new %.4f ms %.1f TF/s | new/old %.3f\n", sh.name, mo, fl / mo / 1e9, mnw,
           fl / mnw / 1e9, mnw / mo);
    fflush(stdout);
  }
  return 0;
}
