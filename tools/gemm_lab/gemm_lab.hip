// Standalone GEMM timing lab (no torch): times kernel variants of the Linear-layer
// GEMMs on the DiffuSeq-base shapes, interleaved in one process (rounds x variants,
// median reported), on uniform random [-1, 1) bf16 operands.
//
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I../../distributed_pipeline_amd/csrc -I. \
//          gemm_lab.hip -o gemm_lab
// run:   ./gemm_lab [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "gemm256.hip"
#include "gemm_pp.hip"
#include "gemm4w.hip"
#include "gemm4p.hip"

#include "gemm.hip"  // 128 x 128 kernels (and device_cu_count)


#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__global__ void fill_rand(uint16_t* p, int64_t n, uint32_t seed, float scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    const float f = ((x >> 8) * (1.0f / 16777216.0f) * 2.f - 1.f) * scale;
    p[i] = dpa::f2bf(f);
  }
}

// fp32 reference C[m][n] = sum_k A[m][k] * B[n][k] (B row form) or B[k][n] (B_TR) on a
// sample of rows; returns max |err| / max |ref|
__global__ void ref_rows(const uint16_t* A, const uint16_t* B, bool btr, int N, int K, const int* rows,
                         int nrows, float* out) {
  const int r = blockIdx.x, n = threadIdx.x + blockIdx.y * blockDim.x;
  if (r >= nrows || n >= N) return;
  const int m = rows[r];
  float s = 0.f;
  for (int k = 0; k < K; ++k)
    s += dpa::bf2f(A[(int64_t)m * K + k]) * dpa::bf2f(btr ? B[(int64_t)k * N + n] : B[(int64_t)n * K + k]);
  out[(int64_t)r * N + n] = s;
}

// Store-throughput probe: every workgroup (512 threads, one per CU) writes `tiles`
// 256 x 256 bf16 tiles of a [M][N] matrix with 16 dwordx4 stores per lane.
// mode 0: the persistent GEMM epilogue pattern (an instruction covers 16 rows x 64 B);
// mode 1: fully contiguous 1 KiB per instruction (2 rows x 512 B).
template <int MODE>
__global__ void __launch_bounds__(512) store_probe(uint16_t* C, int N, int tiles_per_wg, int ntiles) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = (w >> 2) & 1, wn = w & 3;
  const int NT = N / 256;
  for (int k = 0; k < tiles_per_wg; ++k) {
    const int t = (blockIdx.x + k * gridDim.x) % ntiles;
    const int mt = t / NT, nt = t % NT;
    const uint4 v = make_uint4(t, k, lane, w);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      int64_t row;
      int col;
      if (MODE == 0) {
        const int qb = s >> 3, qa = (s >> 2) & 1, i = s & 3, R = lane >> 4, li = lane & 15;
        row = (int64_t)mt * 256 + qa * 128 + wm * 64 + i * 16 + li;
        col = nt * 256 + qb * 128 + wn * 32 + (((R & 1) << 4) | ((R >> 1) << 3));
      } else if (MODE == 1) {
        const int idx = (s * 512 + tid);  // 16-B chunk index within the tile: 32 per row
        row = (int64_t)mt * 256 + (idx >> 5);
        col = nt * 256 + (idx & 31) * 8;
      } else {
        // MODE 2: a wave owns 64 rows x 64 cols (4 x 2 waves), an instruction covers 8 rows x 128 B
        const int wr = w & 3, wc = w >> 2;
        row = (int64_t)mt * 256 + (s >> 3) * 128 + wr * 32 + (s & 3) * 8 + (lane >> 3);
        col = nt * 256 + wc * 128 + ((s >> 2) & 1) * 64 + (lane & 7) * 8;
      }
      *reinterpret_cast<uint4*>(C + row * N + col) = v;
    }
  }
}

__global__ void maxdiff_k(const uint16_t* a, const uint16_t* b, int64_t n, float* out) {
  float m = 0.f, mx = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float x = dpa::bf2f(a[i]), y = dpa::bf2f(b[i]);
    m = fmaxf(m, fabsf(x - y));
    mx = fmaxf(mx, fabsf(x));
  }
  atomicMax(reinterpret_cast<int*>(out), __float_as_int(m));
  atomicMax(reinterpret_cast<int*>(out) + 1, __float_as_int(mx));
}

// max |a - b| / max |a| over n bf16 values
static double maxdiff(const uint16_t* a, const uint16_t* b, int64_t n) {
  float* d;
  CK(hipMalloc(&d, 8));
  CK(hipMemset(d, 0, 8));
  hipLaunchKernelGGL(maxdiff_k, dim3(1024), dim3(256), 0, 0, a, b, n, d);
  float h[2];
  CK(hipMemcpy(h, d, 8, hipMemcpyDeviceToHost));
  CK(hipFree(d));
  return h[0] / (h[1] + 1e-30);
}

__global__ void colsum_bf16(const uint16_t* x, int R, int N, float* out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= N) return;
  double acc = 0;
  for (int r = 0; r < R; ++r) acc += dpa::bf2f(x[(int64_t)r * N + c]);
  out[c] = (float)acc;
}
__global__ void colsum_f32(const float* x, int R, int N, float* out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= N) return;
  double acc = 0;
  for (int r = 0; r < R; ++r) acc += x[(int64_t)r * N + c];
  out[c] = (float)acc;
}

struct Variant {
  std::string name;
  std::function<void(hipStream_t)> fn;
  double flop;
  std::vector<float> ms;
};

static float time_it(Variant& v, hipStream_t s, int iters) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, s));
  for (int i = 0; i < iters; ++i) v.fn(s);
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / iters;
}

static double check(const uint16_t* A, const uint16_t* B, bool btr, const uint16_t* C, int M, int N, int K) {
  const int nrows = 64;
  std::vector<int> rows(nrows);
  for (int i = 0; i < nrows; ++i) rows[i] = (int)(((int64_t)i * 7919 + 13) % M);
  int* drows;
  float* dref;
  CK(hipMalloc(&drows, nrows * sizeof(int)));
  CK(hipMalloc(&dref, (size_t)nrows * N * sizeof(float)));
  CK(hipMemcpy(drows, rows.data(), nrows * sizeof(int), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(ref_rows, dim3(nrows, (N + 255) / 256), dim3(256), 0, 0, A, B, btr, N, K, drows, nrows, dref);
  CK(hipDeviceSynchronize());
  std::vector<float> ref((size_t)nrows * N);
  CK(hipMemcpy(ref.data(), dref, ref.size() * 4, hipMemcpyDeviceToHost));
  std::vector<uint16_t> c((size_t)N);
  double mx = 0, me = 0;
  for (int i = 0; i < nrows; ++i) {
    CK(hipMemcpy(c.data(), C + (int64_t)rows[i] * N, N * 2, hipMemcpyDeviceToHost));
    for (int n = 0; n < N; ++n) {
      uint32_t gb = ((uint32_t)c[n]) << 16; float got; memcpy(&got, &gb, 4);
      const float r = ref[(size_t)i * N + n];
      mx = std::max(mx, (double)fabsf(r));
      me = std::max(me, (double)fabsf(got - r));
    }
  }
  CK(hipFree(drows));
  CK(hipFree(dref));
  return me / (mx + 1e-30);
}

// persistent kernel with the lab knobs (store policy POL, tile grouping GM)
template <bool BTR, int EPI, int ACT, int POL, int GM>
static void gp(const uint16_t* a, int64_t lda, const uint16_t* b, int64_t ldb, int M, int N, int K, uint16_t* c,
               const uint16_t* bias, uint16_t* z, float* colpart, int ncu, hipStream_t st) {
  const int tiles = (M / 256) * (N / 256);
  const int grid = std::min(tiles, ncu);
  hipLaunchKernelGGL((dpa::g256::gemmp_kernel<BTR, EPI, ACT, POL, GM>), dim3(grid), dim3(512), 0, st,
                     (const dpa::bf16_t*)a, lda, (const dpa::bf16_t*)b, ldb, M, N, K / 64, (dpa::bf16_t*)c,
                     (int64_t)N, (const dpa::bf16_t*)bias, (dpa::bf16_t*)z, colpart, (int*)nullptr, 0);
}

// Study "policy": non-temporal epilogue stores / aux loads and grouped tile order on the
// model's persistent GEMMs (fwd: y[T][N] = x[T][K] W[N][K]^T; dgrad: dx[T][K] = dy[T][N] W[N][K])
template <int POL, int GM>
static void add_policy(std::vector<Variant>& vs, const std::string& tag, uint16_t* A, uint16_t* B, uint16_t* C,
                       uint16_t* Z, uint16_t* bias, float* CP, int T, int ncu) {
  auto fl = [&](int K, int N) { return 2.0 * T * K * N; };
  vs.push_back({"qkv/fwd_bias" + tag, [=](hipStream_t st) {
                  gp<false, 0, 0, POL, 1>(A, 768, B, 768, T, 2304, 768, C, bias, nullptr, nullptr, ncu, st);
                }, fl(768, 2304), {}});
  vs.push_back({"attn_out/fwd_bias" + tag, [=](hipStream_t st) {
                  gp<false, 0, 0, POL, 1>(A, 768, B, 768, T, 768, 768, C, bias, nullptr, nullptr, ncu, st);
                }, fl(768, 768), {}});
  vs.push_back({"ffn_in/fwd_gelu_d" + tag, [=](hipStream_t st) {
                  gp<false, 6, 1, POL, GM>(A, 768, B, 768, T, 3072, 768, C, bias, Z, nullptr, ncu, st);
                }, fl(768, 3072), {}});
  vs.push_back({"ffn_out/fwd_bias" + tag, [=](hipStream_t st) {
                  gp<false, 0, 0, POL, 1>(A, 3072, B, 3072, T, 768, 3072, C, bias, nullptr, nullptr, ncu, st);
                }, fl(3072, 768), {}});
  // dh[T][3072] = dy[T][768] W2[768][3072] * d, plus column-sum partials (EPI 4, act code 4)
  vs.push_back({"ffn_out/dgrad_dact_db" + tag, [=](hipStream_t st) {
                  gp<true, 4, 4, POL, GM>(A, 768, B, 3072, T, 3072, 768, C, nullptr, Z, CP, ncu, st);
                }, fl(768, 3072), {}});
  // dx[T][768] = dh[T][3072] W1[3072][768] + dx (EPI 5, in place)
  vs.push_back({"ffn_in/dgrad_res" + tag, [=](hipStream_t st) {
                  gp<true, 5, 0, POL, 1>(A, 3072, B, 768, T, 768, 3072, C, nullptr, C, nullptr, ncu, st);
                }, fl(3072, 768), {}});
}

// Study "stagger": start-phase offsets between workgroups (STG phases of DU x ~1 us) so the
// epilogue store bursts of the 256 persistent workgroups stop coinciding; q != nullptr runs
// the dynamic tile queue (a late workgroup takes fewer tiles).  Library store policy.
template <bool BTR, int EPI, int ACT, int POL, int GM, int STG, int DU>
static void gps(const uint16_t* a, int64_t lda, const uint16_t* b, int64_t ldb, int M, int N, int K, uint16_t* c,
                const uint16_t* bias, uint16_t* z, float* colpart, int ncu, int* q, hipStream_t st) {
  const int tiles = (M / 256) * (N / 256);
  const int grid = std::min(tiles, ncu);
  if (q) CK(hipMemsetAsync(q, 0, 8 * 16 * sizeof(int), st));
  hipLaunchKernelGGL((dpa::g256::gemmp_kernel<BTR, EPI, ACT, POL, GM, STG, DU>), dim3(grid), dim3(512), 0, st,
                     (const dpa::bf16_t*)a, lda, (const dpa::bf16_t*)b, ldb, M, N, K / 64, (dpa::bf16_t*)c,
                     (int64_t)N, (const dpa::bf16_t*)bias, (dpa::bf16_t*)z, colpart, q, 0);
}
template <int STG, int DU>
static void add_stag(std::vector<Variant>& vs, const std::string& tag, uint16_t* A, uint16_t* B, uint16_t* C,
                     uint16_t* Z, uint16_t* bias, float* CP, int T, int ncu, int* q) {
  auto fl = [&](int K, int N) { return 2.0 * T * K * N; };
  vs.push_back({"qkv/fwd_bias" + tag, [=](hipStream_t st) {
                  gps<false, 0, 0, 0, 1, STG, DU>(A, 768, B, 768, T, 2304, 768, C, bias, nullptr, nullptr, ncu, q, st);
                }, fl(768, 2304), {}});
  vs.push_back({"attn_out/fwd_bias" + tag, [=](hipStream_t st) {
                  gps<false, 0, 0, 0, 1, STG, DU>(A, 768, B, 768, T, 768, 768, C, bias, nullptr, nullptr, ncu, q, st);
                }, fl(768, 768), {}});
  vs.push_back({"ffn_in/fwd_gelu_d" + tag, [=](hipStream_t st) {
                  gps<false, 6, 1, 1, 8, STG, DU>(A, 768, B, 768, T, 3072, 768, C, bias, Z, nullptr, ncu, q, st);
                }, fl(768, 3072), {}});
  vs.push_back({"ffn_out/fwd_bias" + tag, [=](hipStream_t st) {
                  gps<false, 0, 0, 0, 1, STG, DU>(A, 3072, B, 3072, T, 768, 3072, C, bias, nullptr, nullptr, ncu, q, st);
                }, fl(3072, 768), {}});
  vs.push_back({"ffn_out/dgrad_dact_db" + tag, [=](hipStream_t st) {
                  gps<true, 4, 4, 1, 8, STG, DU>(A, 768, B, 3072, T, 3072, 768, C, nullptr, Z, CP, ncu, q, st);
                }, fl(768, 3072), {}});
  vs.push_back({"ffn_in/dgrad_res" + tag, [=](hipStream_t st) {
                  gps<true, 5, 0, 0, 1, STG, DU>(A, 3072, B, 768, T, 768, 3072, C, nullptr, C, nullptr, ncu, q, st);
                }, fl(3072, 768), {}});
  vs.push_back({"qkv/dgrad" + tag, [=](hipStream_t st) {
                  gps<true, 0, 0, 0, 1, STG, DU>(A, 2304, B, 768, T, 768, 2304, C, nullptr, nullptr, nullptr, ncu, q, st);
                }, fl(2304, 768), {}});
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 5;
  const int iters = 10;
  const int T = 262144;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  printf("CUs %d\n", ncu);

  struct Shape { const char* name; int K, N; };
  const Shape shapes[] = {{"qkv", 768, 2304}, {"attn_out", 768, 768}, {"ffn_in", 768, 3072}, {"ffn_out", 3072, 768}};
  uint16_t *A, *B, *C, *bias, *Z;
  float* CP;
  CK(hipMalloc(&CP, (size_t)(262144 / 256) * 2 * 3072 * 4));
  const int64_t maxA = (int64_t)T * 3072, maxB = 3072LL * 3072, maxC = (int64_t)T * 3072;
  CK(hipMalloc(&A, maxA * 2));
  CK(hipMalloc(&B, maxB * 2));
  CK(hipMalloc(&C, maxC * 2));
  CK(hipMalloc(&Z, maxC * 2));
  CK(hipMalloc(&bias, 4096 * 2));
  float* DW;
  CK(hipMalloc(&DW, 3072LL * 3072 * 4));
  hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, A, maxA, 1u, 1.f);
  hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, B, maxB, 2u, 0.05f);
  hipLaunchKernelGGL(fill_rand, dim3(16), dim3(256), 0, 0, bias, (int64_t)4096, 3u, 0.1f);
  hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, Z, maxC, 4u, 1.f);
  CK(hipDeviceSynchronize());

  if (argc > 2 && std::string(argv[2]) == "stagger") {
    int* q;
    CK(hipMalloc(&q, 8 * 16 * sizeof(int)));
    std::vector<Variant> pv;
    add_stag<0, 0>(pv, "", A, B, C, Z, bias, CP, T, ncu, nullptr);
    add_stag<4, 5>(pv, "_s4x5", A, B, C, Z, bias, CP, T, ncu, nullptr);
    add_stag<4, 10>(pv, "_s4x10", A, B, C, Z, bias, CP, T, ncu, nullptr);
    add_stag<8, 3>(pv, "_s8x3", A, B, C, Z, bias, CP, T, ncu, nullptr);
    add_stag<0, 0>(pv, "_dyn", A, B, C, Z, bias, CP, T, ncu, q);
    add_stag<4, 10>(pv, "_dyn_s4x10", A, B, C, Z, bias, CP, T, ncu, q);
    add_stag<8, 3>(pv, "_dyn_s8x3", A, B, C, Z, bias, CP, T, ncu, q);
    {  // bitwise: the stagger only moves start times
      const int K = 768, N = 3072;
      uint16_t *C2, *Z2;
      CK(hipMalloc(&C2, (size_t)T * N * 2));
      CK(hipMalloc(&Z2, (size_t)T * N * 2));
      gps<false, 6, 1, 1, 8, 0, 0>(A, K, B, K, T, N, K, C, bias, Z, nullptr, ncu, nullptr, s);
      gps<false, 6, 1, 1, 8, 8, 3>(A, K, B, K, T, N, K, C2, bias, Z2, nullptr, ncu, q, s);
      CK(hipStreamSynchronize(s));
      printf("check stagger gelu y maxdiff %.3e d maxdiff %.3e\n", maxdiff(C, C2, (int64_t)T * N),
             maxdiff(Z, Z2, (int64_t)T * N));
      CK(hipFree(C2));
      CK(hipFree(Z2));
      hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, Z, maxC, 4u, 1.f);
      CK(hipDeviceSynchronize());
    }
    for (auto& v : pv) time_it(v, s, 2);
    for (int r = 0; r < rounds; ++r)
      for (auto& v : pv) v.ms.push_back(time_it(v, s, iters));
    for (auto& v : pv) {
      std::sort(v.ms.begin(), v.ms.end());
      const float med = v.ms[v.ms.size() / 2];
      printf("%-32s median %.4f ms  min %.4f ms  %.1f TF/s\n", v.name.c_str(), med, v.ms[0], v.flop / med / 1e9);
    }
    return 0;
  }

  if (argc > 2 && std::string(argv[2]) == "small") {
    // reference-schedule micro-batch (64 x 128 = 8192 tokens): persistent 256 x 256 tiles
    // (96-384 tiles for 256 CUs) vs the 128 x 128 kernel (4x the tiles)
    const int Ts = 8192;
    std::vector<Variant> pv;
    for (const Shape& sh : shapes) {
      const int K = sh.K, N = sh.N;
      const double fl = 2.0 * Ts * K * N;
      const std::string nm = sh.name;
      pv.push_back({nm + "/fwd_gp256", [=](hipStream_t st) {
                      dpa::launch_gemmp_nt(A, B, bias, C, nullptr, Ts, N, K, 0, ncu, st);
                    }, fl, {}});
      pv.push_back({nm + "/fwd_t128", [=](hipStream_t st) {
                      hipLaunchKernelGGL((dpa::gemm_kernel<false, false, dpa::EPI_BIAS_ACT>), dim3((Ts / 128) * (N / 128)),
                                         dim3(256), 0, st, (const dpa::bf16_t*)A, (int64_t)K, (const dpa::bf16_t*)B,
                                         (int64_t)K, Ts, N, K, K, 1, (dpa::bf16_t*)C, (int64_t)N, nullptr,
                                         (const dpa::bf16_t*)bias, 0, nullptr, nullptr);
                    }, fl, {}});
      pv.push_back({nm + "/dgrad_gp256", [=](hipStream_t st) {
                      dpa::launch_gemmp_nn(A, B, C, nullptr, 0, Ts, N, K, ncu, st, nullptr);
                    }, fl, {}});
      pv.push_back({nm + "/dgrad_t128", [=](hipStream_t st) {
                      hipLaunchKernelGGL((dpa::gemm_kernel<false, true, dpa::EPI_BF16>), dim3((Ts / 128) * (K / 128)),
                                         dim3(256), 0, st, (const dpa::bf16_t*)A, (int64_t)N, (const dpa::bf16_t*)B,
                                         (int64_t)K, Ts, K, N, N, 1, (dpa::bf16_t*)C, (int64_t)K, nullptr, nullptr, 0,
                                         nullptr, nullptr);
                    }, fl, {}});
    }
    for (auto& v : pv) time_it(v, s, 2);
    for (int r = 0; r < rounds; ++r)
      for (auto& v : pv) v.ms.push_back(time_it(v, s, iters));
    for (auto& v : pv) {
      std::sort(v.ms.begin(), v.ms.end());
      const float med = v.ms[v.ms.size() / 2];
      printf("%-32s median %.4f ms  min %.4f ms  %.1f TF/s\n", v.name.c_str(), med, v.ms[0], v.flop / med / 1e9);
    }
    return 0;
  }

  if (argc > 2 && std::string(argv[2]) == "aux") {
    // epilogues that read an aux operand (EPI 5 residual-accumulating dgrad, EPI 4 dact dgrad
    // with bias column sums) vs the plain dgrad: build with -DDPA_GEMM_EARLY_AUX=0 / 1 to
    // compare the aux loads issued in the last K-iteration against after the main loop
    std::vector<Variant> pv;
    for (const Shape& sh : shapes) {
      const int K = sh.K, N = sh.N;
      const double fl = 2.0 * T * K * N;
      const std::string nm = sh.name;
      pv.push_back({nm + "/gp_dgrad", [=](hipStream_t st) {
                      gp<true, 0, 0, 0, 1>(A, N, B, K, T, K, N, C, nullptr, nullptr, nullptr, ncu, st);
                    }, fl, {}});
      pv.push_back({nm + "/gp_dgrad_res", [=](hipStream_t st) {
                      gp<true, 5, 0, 0, 1>(A, N, B, K, T, K, N, C, nullptr, Z, nullptr, ncu, st);
                    }, fl, {}});
      if (nm == "ffn_out")
        pv.push_back({nm + "/gp_dgrad_dact_db", [=](hipStream_t st) {
                        gp<true, 4, 4, 1, 8>(A, 768, B, 3072, T, 3072, 768, C, nullptr, Z, CP, ncu, st);
                      }, fl, {}});
    }
    printf("DPA_GEMM_EARLY_AUX=%d\n", DPA_GEMM_EARLY_AUX);
    for (auto& v : pv) time_it(v, s, 2);
    for (int r = 0; r < rounds; ++r)
      for (auto& v : pv) v.ms.push_back(time_it(v, s, iters));
    for (auto& v : pv) {
      std::sort(v.ms.begin(), v.ms.end());
      const float med = v.ms[v.ms.size() / 2];
      printf("%-32s median %.4f ms  min %.4f ms  %.1f TF/s\n", v.name.c_str(), med, v.ms[0], v.flop / med / 1e9);
    }
    return 0;
  }

  if (argc > 2 && std::string(argv[2]) == "4p") {
    // persistent one-wave-per-SIMD 256 x 128 kernel with the epilogue inside the next tile's
    // main loop (gemm4p.hip) vs the production persistent 8-wave kernel (gemmp_kernel)
    std::vector<Variant> pv;
    for (const Shape& sh : shapes) {
      const int K = sh.K, N = sh.N;
      const double fl = 2.0 * T * K * N;
      const std::string nm = sh.name;
      pv.push_back({nm + "/gp_bias", [=](hipStream_t st) {
                      dpa::launch_gemmp_nt(A, B, bias, C, nullptr, T, N, K, 0, ncu, st);
                    }, fl, {}});
      pv.push_back({nm + "/gp_bias_sc1", [=](hipStream_t st) {
                      gp<false, 0, 0, 4, 1>(A, K, B, K, T, N, K, C, bias, nullptr, nullptr, ncu, st);
                    }, fl, {}});
      pv.push_back({nm + "/4p_bias", [=](hipStream_t st) {
                      dpa::launch_gemm4p<0, 0>(A, B, bias, C, nullptr, T, N, K, ncu, st);
                    }, fl, {}});
      pv.push_back({nm + "/4p_nostore", [=](hipStream_t st) {
                      dpa::launch_gemm4p<-1, 0>(A, B, bias, C, nullptr, T, N, K, ncu, st);
                    }, fl, {}});
      // data gradient dx[T][K] = dy[T][N] W[N][K] (B transposed reads), plain and write-through stores
      pv.push_back({nm + "/gp_dgrad", [=](hipStream_t st) {
                      gp<true, 0, 0, 0, 1>(A, N, B, K, T, K, N, C, nullptr, nullptr, nullptr, ncu, st);
                    }, fl, {}});
      pv.push_back({nm + "/gp_dgrad_sc1", [=](hipStream_t st) {
                      gp<true, 0, 0, 4, 1>(A, N, B, K, T, K, N, C, nullptr, nullptr, nullptr, ncu, st);
                    }, fl, {}});
      if (nm == "ffn_out") {
        pv.push_back({nm + "/gp_dgrad_dact_db", [=](hipStream_t st) {
                        gp<true, 4, 4, 1, 8>(A, 768, B, 3072, T, 3072, 768, C, nullptr, Z, CP, ncu, st);
                      }, fl, {}});
        pv.push_back({nm + "/gp_dgrad_dact_db_sc1", [=](hipStream_t st) {
                        gp<true, 4, 4, 4, 8>(A, 768, B, 3072, T, 3072, 768, C, nullptr, Z, CP, ncu, st);
                      }, fl, {}});
      }
      if (nm == "ffn_in") {
        pv.push_back({nm + "/gp_gelu_d", [=](hipStream_t st) {
                        dpa::launch_gemmp_nt(A, B, bias, C, Z, T, N, K, 1, ncu, st, true);
                      }, fl, {}});
        pv.push_back({nm + "/gp_gelu_d_sc1", [=](hipStream_t st) {
                        gp<false, 6, 1, 4, 8>(A, K, B, K, T, N, K, C, bias, Z, nullptr, ncu, st);
                      }, fl, {}});
        pv.push_back({nm + "/4p_gelu_d", [=](hipStream_t st) {
                        dpa::launch_gemm4p<6, 1>(A, B, bias, C, Z, T, N, K, ncu, st);
                      }, fl, {}});
      }
    }
    for (const Shape& sh : shapes) {
      dpa::launch_gemm4p<0, 0>(A, B, nullptr, C, nullptr, T, sh.N, sh.K, ncu, s);
      CK(hipStreamSynchronize(s));
      printf("check %s 4p relerr %.3e\n", sh.name, check(A, B, false, C, T, sh.N, sh.K));
    }
    {  // bias and GELU epilogues vs the production kernel's (same accumulation order)
      const int K = 768, N = 3072;
      uint16_t *C2, *Z2;
      CK(hipMalloc(&C2, (size_t)T * N * 2));
      CK(hipMalloc(&Z2, (size_t)T * N * 2));
      dpa::launch_gemmp_nt(A, B, bias, C, nullptr, T, N, K, 0, ncu, s);
      dpa::launch_gemm4p<0, 0>(A, B, bias, C2, nullptr, T, N, K, ncu, s);
      CK(hipStreamSynchronize(s));
      printf("check 4p bias vs gp maxdiff %.3e\n", maxdiff(C, C2, (int64_t)T * N));
      dpa::launch_gemmp_nt(A, B, bias, C, Z, T, N, K, 1, ncu, s, true);
      dpa::launch_gemm4p<6, 1>(A, B, bias, C2, Z2, T, N, K, ncu, s);
      CK(hipStreamSynchronize(s));
      printf("check 4p gelu vs gp y maxdiff %.3e d maxdiff %.3e\n", maxdiff(C, C2, (int64_t)T * N),
             maxdiff(Z, Z2, (int64_t)T * N));
      CK(hipFree(C2));
      CK(hipFree(Z2));
      hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, Z, maxC, 4u, 1.f);
      CK(hipDeviceSynchronize());
    }
    for (auto& v : pv) time_it(v, s, 2);
    for (int r = 0; r < rounds; ++r)
      for (auto& v : pv) v.ms.push_back(time_it(v, s, iters));
    for (auto& v : pv) {
      std::sort(v.ms.begin(), v.ms.end());
      const float med = v.ms[v.ms.size() / 2];
      printf("%-32s median %.4f ms  min %.4f ms  %.1f TF/s\n", v.name.c_str(), med, v.ms[0], v.flop / med / 1e9);
    }
    return 0;
  }

  if (argc > 2 && std::string(argv[2]) == "4w") {
    // one wave per SIMD (gemm4w.hip) vs the two-wave 8-phase template, main loop only (no
    // epilogue stores), one tile per workgroup in both (non-persistent)
    std::vector<Variant> pv;
    for (const Shape& sh : shapes) {
      const int K = sh.K, N = sh.N;
      const double fl = 2.0 * T * K * N;
      const std::string nm = sh.name;
      pv.push_back({nm + "/g256_nostore", [=](hipStream_t st) {
                      hipLaunchKernelGGL((dpa::g256::gemm256_kernel<false, false, dpa::g256::EPI_NONE>),
                                         dim3((T / 256) * (N / 256)), dim3(512), 0, st, (const dpa::bf16_t*)A,
                                         (int64_t)K, (const dpa::bf16_t*)B, (int64_t)K, T, N, K / 64, K / 64, 1,
                                         (dpa::bf16_t*)C, (int64_t)N, nullptr, nullptr, 0, nullptr, nullptr);
                    }, fl, {}});
      pv.push_back({nm + "/4w_nostore", [=](hipStream_t st) {
                      dpa::launch_gemm4w(A, B, C, T, N, K, false, st);
                    }, fl, {}});
      pv.push_back({nm + "/fwd_gp", [=](hipStream_t st) {
                      dpa::launch_gemmp_nt(A, B, nullptr, C, nullptr, T, N, K, 0, ncu, st);
                    }, fl, {}});
    }
    for (const Shape& sh : shapes) {
      dpa::launch_gemm4w(A, B, C, T, sh.N, sh.K, true, s);
      CK(hipStreamSynchronize(s));
      printf("check %s 4w relerr %.3e\n", sh.name, check(A, B, false, C, T, sh.N, sh.K));
    }
    for (auto& v : pv) time_it(v, s, 2);
    for (int r = 0; r < rounds; ++r)
      for (auto& v : pv) v.ms.push_back(time_it(v, s, iters));
    for (auto& v : pv) {
      std::sort(v.ms.begin(), v.ms.end());
      const float med = v.ms[v.ms.size() / 2];
      printf("%-32s median %.4f ms  min %.4f ms  %.1f TF/s\n", v.name.c_str(), med, v.ms[0], v.flop / med / 1e9);
    }
    return 0;
  }

  if (argc > 2 && std::string(argv[2]) == "policy") {
    std::vector<Variant> pv;
    add_policy<0, 1>(pv, "", A, B, C, Z, bias, CP, T, ncu);
    add_policy<1, 1>(pv, "_nt", A, B, C, Z, bias, CP, T, ncu);
    add_policy<3, 1>(pv, "_nt_ntaux", A, B, C, Z, bias, CP, T, ncu);
    add_policy<0, 8>(pv, "_gm8", A, B, C, Z, bias, CP, T, ncu);
    add_policy<0, 4>(pv, "_gm4", A, B, C, Z, bias, CP, T, ncu);
    add_policy<1, 8>(pv, "_nt_gm8", A, B, C, Z, bias, CP, T, ncu);
    {  // bitwise: every policy / grouping writes the same y and d as the default
      const int K = 768, N = 3072;
      uint16_t *C2, *Z2;
      CK(hipMalloc(&C2, (size_t)T * N * 2));
      CK(hipMalloc(&Z2, (size_t)T * N * 2));
      gp<false, 6, 1, 0, 1>(A, K, B, K, T, N, K, C, bias, Z, nullptr, ncu, s);
      gp<false, 6, 1, 1, 8>(A, K, B, K, T, N, K, C2, bias, Z2, nullptr, ncu, s);
      CK(hipStreamSynchronize(s));
      printf("check nt_gm8 gelu y maxdiff %.3e d maxdiff %.3e\n", maxdiff(C, C2, (int64_t)T * N),
             maxdiff(Z, Z2, (int64_t)T * N));
      gp<true, 4, 4, 0, 1>(A, 768, B, 3072, T, 3072, 768, C, nullptr, Z, CP, ncu, s);
      gp<true, 4, 4, 3, 8>(A, 768, B, 3072, T, 3072, 768, C2, nullptr, Z, CP, ncu, s);
      CK(hipStreamSynchronize(s));
      printf("check nt_gm8 dact maxdiff %.3e\n", maxdiff(C, C2, (int64_t)T * N));
      CK(hipFree(C2));
      CK(hipFree(Z2));
      hipLaunchKernelGGL(fill_rand, dim3(4096), dim3(256), 0, 0, Z, maxC, 4u, 1.f);
      CK(hipDeviceSynchronize());
    }
    for (auto& v : pv) time_it(v, s, 2);
    for (int r = 0; r < rounds; ++r)
      for (auto& v : pv) v.ms.push_back(time_it(v, s, iters));
    for (auto& v : pv) {
      std::sort(v.ms.begin(), v.ms.end());
      const float med = v.ms[v.ms.size() / 2];
      printf("%-32s median %.4f ms  min %.4f ms  %.1f TF/s\n", v.name.c_str(), med, v.ms[0], v.flop / med / 1e9);
    }
    return 0;
  }

  std::vector<Variant> vs;
  // shape (K = layer input width, N = layer output width)
  for (const Shape& sh : shapes) {
    const int K = sh.K, N = sh.N;
    const double fl = 2.0 * T * K * N;
    const std::string nm = sh.name;
    vs.push_back({nm + "/fwd_g256", [=](hipStream_t st) {
                    dpa::launch_gemm256_nt(A, B, bias, C, nullptr, T, N, K, 0, st);
                  }, fl, {}});
    vs.push_back({nm + "/fwd_nostore", [=](hipStream_t st) {
                    hipLaunchKernelGGL((dpa::g256::gemm256_kernel<false, false, dpa::g256::EPI_NONE>),
                                       dim3((T / 256) * (N / 256)), dim3(512), 0, st, (const dpa::bf16_t*)A,
                                       (int64_t)K, (const dpa::bf16_t*)B, (int64_t)K, T, N, K / 64, K / 64, 1,
                                       (dpa::bf16_t*)C, (int64_t)N, nullptr, nullptr, 0, nullptr, nullptr);
                  }, fl, {}});
    vs.push_back({nm + "/fwd_gp", [=](hipStream_t st) {
                    dpa::launch_gemmp_nt(A, B, bias, C, nullptr, T, N, K, 0, ncu, st);
                  }, fl, {}});
    // data gradient of this layer: dx[T][K] = dy[T][N] . W[N][K]
    vs.push_back({nm + "/dgrad_g256", [=](hipStream_t st) {
                    dpa::launch_gemm256_nn(A, B, C, T, N, K, st);
                  }, fl, {}});
    vs.push_back({nm + "/dgrad_gp", [=](hipStream_t st) {
                    dpa::launch_gemmp_nn(A, B, C, nullptr, 0, T, N, K, ncu, st, nullptr);
                  }, fl, {}});
    if (nm == "ffn_in") {
      vs.push_back({nm + "/fwd_gelu_z_g256", [=](hipStream_t st) {
                      dpa::launch_gemm256_nt(A, B, bias, C, Z, T, N, K, 1, st);
                    }, fl, {}});
      vs.push_back({nm + "/fwd_gelu_z_gp", [=](hipStream_t st) {
                      dpa::launch_gemmp_nt(A, B, bias, C, Z, T, N, K, 1, ncu, st);
                    }, fl, {}});
    }
    if (nm == "ffn_out") {  // dh = (dy . W2) * gelu'(z1): the MLP's fused dgrad
      vs.push_back({nm + "/dgrad_dgelu_g256", [=](hipStream_t st) {
                      dpa::launch_gemm256_nn_dact(A, B, Z, C, T, N, K, 1, st);
                    }, fl, {}});
      vs.push_back({nm + "/dgrad_dgelu_gp", [=](hipStream_t st) {
                      dpa::launch_gemmp_nn(A, B, C, Z, 1, T, N, K, ncu, st, nullptr);
                    }, fl, {}});
      vs.push_back({nm + "/dgrad_dgelu_db_gp", [=](hipStream_t st) {
                      dpa::launch_gemmp_nn(A, B, C, Z, 1, T, N, K, ncu, st, CP);
                    }, fl, {}});
    }
  }
  // ping-pong kernel (gemm_pp.hip): main loop alone, plain bias epilogue, GELU epilogue, dgrad
  for (const Shape& sh : shapes) {
    const int K = sh.K, N = sh.N;
    const double fl = 2.0 * T * K * N;
    const std::string nm = sh.name;
    vs.push_back({nm + "/pp_fwd_nostore", [=](hipStream_t st) {
                    dpa::launch_gemm_pp_nt(A, B, bias, C, nullptr, T, N, K, 0, ncu, st, -1);
                  }, fl, {}});
    vs.push_back({nm + "/pp_fwd", [=](hipStream_t st) {
                    dpa::launch_gemm_pp_nt(A, B, bias, C, nullptr, T, N, K, 0, ncu, st, 0);
                  }, fl, {}});
    vs.push_back({nm + "/pp_dgrad_nostore", [=](hipStream_t st) {
                    dpa::launch_gemm_pp_nn(A, B, C, T, N, K, ncu, st, -1);
                  }, fl, {}});
    vs.push_back({nm + "/pp_dgrad", [=](hipStream_t st) {
                    dpa::launch_gemm_pp_nn(A, B, C, T, N, K, ncu, st, 0);
                  }, fl, {}});
    if (nm == "ffn_in")
      vs.push_back({nm + "/pp_fwd_gelu", [=](hipStream_t st) {
                      dpa::launch_gemm_pp_nt(A, B, bias, C, Z, T, N, K, 1, ncu, st, 0);
                    }, fl, {}});
  }
  // epilogue cost split: ldc = 0 makes every row of a column band hit the same L2 lines
  // (stores still issue, the HBM drain is ~gone) - issue/VALU cost vs drain cost
  {
    const int K = 768, N = 3072;
    const double fl = 2.0 * T * K * N;
    const int grid = std::min((T / 256) * (N / 256), ncu);
    vs.push_back({"ffn_in/fwd_gp_ldc0", [=](hipStream_t st) {
                    hipLaunchKernelGGL((dpa::g256::gemmp_kernel<false, 0, 0>), dim3(grid), dim3(512), 0, st,
                                       (const dpa::bf16_t*)A, (int64_t)K, (const dpa::bf16_t*)B, (int64_t)K, T, N,
                                       K / 64, (dpa::bf16_t*)C, (int64_t)0, (const dpa::bf16_t*)bias,
                                       (dpa::bf16_t*)nullptr, (float*)nullptr, (int*)nullptr, 0);
                  }, fl, {}});
    vs.push_back({"ffn_in/fwd_gelu_z_gp_ldc0", [=](hipStream_t st) {
                    hipLaunchKernelGGL((dpa::g256::gemmp_kernel<false, 2, 1>), dim3(grid), dim3(512), 0, st,
                                       (const dpa::bf16_t*)A, (int64_t)K, (const dpa::bf16_t*)B, (int64_t)K, T, N,
                                       K / 64, (dpa::bf16_t*)C, (int64_t)0, (const dpa::bf16_t*)bias,
                                       (dpa::bf16_t*)Z, (float*)nullptr, (int*)nullptr, 0);
                  }, fl, {}});
    vs.push_back({"ffn_in/fwd_z_noact_gp_ldc0", [=](hipStream_t st) {
                    hipLaunchKernelGGL((dpa::g256::gemmp_kernel<false, 2, 0>), dim3(grid), dim3(512), 0, st,
                                       (const dpa::bf16_t*)A, (int64_t)K, (const dpa::bf16_t*)B, (int64_t)K, T, N,
                                       K / 64, (dpa::bf16_t*)C, (int64_t)0, (const dpa::bf16_t*)bias,
                                       (dpa::bf16_t*)Z, (float*)nullptr, (int*)nullptr, 0);
                  }, fl, {}});
    vs.push_back({"ffn_in/fwd_z_noact_gp", [=](hipStream_t st) {
                    hipLaunchKernelGGL((dpa::g256::gemmp_kernel<false, 2, 0>), dim3(grid), dim3(512), 0, st,
                                       (const dpa::bf16_t*)A, (int64_t)K, (const dpa::bf16_t*)B, (int64_t)K, T, N,
                                       K / 64, (dpa::bf16_t*)C, (int64_t)N, (const dpa::bf16_t*)bias,
                                       (dpa::bf16_t*)Z, (float*)nullptr, (int*)nullptr, 0);
                  }, fl, {}});
    vs.push_back({"ffn_out/dgrad_dact_noact_gp_ldc0", [=](hipStream_t st) {
                    hipLaunchKernelGGL((dpa::g256::gemmp_kernel<true, 3, 0>), dim3(grid), dim3(512), 0, st,
                                       (const dpa::bf16_t*)A, (int64_t)768, (const dpa::bf16_t*)B, (int64_t)3072, T,
                                       3072, 768 / 64, (dpa::bf16_t*)C, (int64_t)0, (const dpa::bf16_t*)nullptr,
                                       (dpa::bf16_t*)Z, (float*)nullptr, (int*)nullptr, 0);
                  }, fl, {}});
    // dgrad of ffn_out with dgelu: dh[T][3072] = dy[T][768] . W2[768][3072] * gelu'(z)
    vs.push_back({"ffn_out/dgrad_dgelu_gp_ldc0", [=](hipStream_t st) {
                    hipLaunchKernelGGL((dpa::g256::gemmp_kernel<true, 3, 1>), dim3(grid), dim3(512), 0, st,
                                       (const dpa::bf16_t*)A, (int64_t)768, (const dpa::bf16_t*)B, (int64_t)3072, T,
                                       3072, 768 / 64, (dpa::bf16_t*)C, (int64_t)0, (const dpa::bf16_t*)nullptr,
                                       (dpa::bf16_t*)Z, (float*)nullptr, (int*)nullptr, 0);
                  }, fl, {}});
    vs.push_back({"ffn_out/dgrad_nostore_g256", [=](hipStream_t st) {
                    hipLaunchKernelGGL((dpa::g256::gemm256_kernel<false, true, dpa::g256::EPI_NONE>),
                                       dim3((T / 256) * (3072 / 256)), dim3(512), 0, st, (const dpa::bf16_t*)A,
                                       (int64_t)768, (const dpa::bf16_t*)B, (int64_t)3072, T, 3072, 768 / 64,
                                       768 / 64, 1, (dpa::bf16_t*)C, (int64_t)3072, nullptr, nullptr, 0, nullptr,
                                       nullptr);
                  }, fl, {}});
  }
  // weight gradients dW[N][K] += dy[T][N]^T . x[T][K] (split-K, fp32 atomics) and the
  // same grid without the atomic epilogue (main loop with both operands transposed)
  for (const Shape& sh : shapes) {
    const int K = sh.K, N = sh.N;
    const double fl = 2.0 * T * K * N;
    const std::string nm = sh.name;
    vs.push_back({nm + "/wgrad", [=](hipStream_t st) {
                    dpa::launch_gemm256_wgrad(A, Z, DW, nullptr, T, N, K, st);
                  }, fl, {}});
    vs.push_back({nm + "/wgrad_nostore", [=](hipStream_t st) {
                    const int tiles = (N / 256) * (K / 256), ktot = T / 64;
                    const int splits = std::max(1, (2 * ncu + tiles - 1) / tiles);
                    int kps = (ktot + splits - 1) / splits;
                    kps += kps & 1;
                    const int sp = (ktot + kps - 1) / kps;
                    hipLaunchKernelGGL((dpa::g256::gemm256_kernel<true, true, dpa::g256::EPI_NONE>),
                                       dim3(tiles * sp), dim3(512), 0, st, (const dpa::bf16_t*)A, (int64_t)N,
                                       (const dpa::bf16_t*)Z, (int64_t)K, N, K, ktot, kps, sp, nullptr, (int64_t)K,
                                       DW, nullptr, 0, nullptr, nullptr);
                  }, fl, {}});
  }
  {  // per-CU store rate vs number of storing CUs (each WG writes 36 tiles of 128 KiB)
    const int N = 2304;
    const int ntiles = (T / 256) * (N / 256);
    for (int g : {8, 32, 64, 128, 256}) {
      const double bytes = (double)g * 36 * 131072;
      vs.push_back({"store_probe_gemmpat_wg" + std::to_string(g), [=](hipStream_t st) {
                      hipLaunchKernelGGL(store_probe<0>, dim3(g), dim3(512), 0, st, C, N, 36, ntiles);
                    }, bytes * 1e3 / g /* TF/s column = TB/s per WG x 1000 = GB/s per CU */, {}});
      vs.push_back({"store_probe_rows_wg" + std::to_string(g), [=](hipStream_t st) {
                      hipLaunchKernelGGL(store_probe<1>, dim3(g), dim3(512), 0, st, C, N, 36, ntiles);
                    }, bytes * 1e3 / g, {}});
      vs.push_back({"store_probe_8x128_wg" + std::to_string(g), [=](hipStream_t st) {
                      hipLaunchKernelGGL(store_probe<2>, dim3(g), dim3(512), 0, st, C, N, 36, ntiles);
                    }, bytes * 1e3 / g, {}});
    }
  }
  // correctness of the new kernels (fwd: B row form [N][K]; dgrad: B [N][K] read as [k][n])
  for (const Shape& sh : shapes) {
    const int K = sh.K, N = sh.N;
    CK(hipMemset(C, 0, (size_t)T * N * 2));
    dpa::launch_gemmp_nt(A, B, nullptr, C, nullptr, T, N, K, 0, ncu, s);
    CK(hipStreamSynchronize(s));
    printf("check %s gp_fwd relerr %.3e\n", sh.name, check(A, B, false, C, T, N, K));
    CK(hipMemset(C, 0, (size_t)T * K * 2));
    dpa::launch_gemmp_nn(A, B, C, nullptr, 0, T, N, K, ncu, s, nullptr);
    CK(hipStreamSynchronize(s));
    // dx[T][K] = dy[T][N] . W[N][K]: reference with reduction N, output width K, B = [N][K] as [k][n]
    printf("check %s gp_dgrad relerr %.3e\n", sh.name, check(A, B, true, C, T, K, N));
    fflush(stdout);
  }
  for (const Shape& sh : shapes) {  // ping-pong kernel correctness
    const int K = sh.K, N = sh.N;
    CK(hipMemset(C, 0, (size_t)T * N * 2));
    dpa::launch_gemm_pp_nt(A, B, nullptr, C, nullptr, T, N, K, 0, ncu, s, 0);
    CK(hipStreamSynchronize(s));
    printf("check %s pp_fwd relerr %.3e\n", sh.name, check(A, B, false, C, T, N, K));
    CK(hipMemset(C, 0, (size_t)T * K * 2));
    dpa::launch_gemm_pp_nn(A, B, C, T, N, K, ncu, s, 0);
    CK(hipStreamSynchronize(s));
    printf("check %s pp_dgrad relerr %.3e\n", sh.name, check(A, B, true, C, T, K, N));
    fflush(stdout);
  }
  {  // ping-pong bias and GELU epilogues against the 256 x 256 persistent kernel
    const int K = 768, N = 3072;
    uint16_t *C2, *Z2;
    CK(hipMalloc(&C2, (size_t)T * N * 2));
    CK(hipMalloc(&Z2, (size_t)T * N * 2));
    dpa::launch_gemmp_nt(A, B, bias, C, nullptr, T, N, K, 0, ncu, s);
    dpa::launch_gemm_pp_nt(A, B, bias, C2, nullptr, T, N, K, 0, ncu, s, 0);
    CK(hipStreamSynchronize(s));
    printf("check pp bias y maxdiff %.3e\n", maxdiff(C, C2, (int64_t)T * N));
    dpa::launch_gemmp_nt(A, B, bias, C, Z, T, N, K, 1, ncu, s, true);
    dpa::launch_gemm_pp_nt(A, B, bias, C2, Z2, T, N, K, 1, ncu, s, 0);
    CK(hipStreamSynchronize(s));
    printf("check pp gelu y maxdiff %.3e d maxdiff %.3e\n", maxdiff(C, C2, (int64_t)T * N), maxdiff(Z, Z2, (int64_t)T * N));
    CK(hipFree(C2));
    CK(hipFree(Z2));
    fflush(stdout);
  }
  {  // fused epilogues against the unfused g256 kernels (bitwise-close: same bf16 rounding points)
    const int K = 768, N = 3072;
    uint16_t *C2, *Z2;
    CK(hipMalloc(&C2, (size_t)T * N * 2));
    CK(hipMalloc(&Z2, (size_t)T * N * 2));
    dpa::launch_gemm256_nt(A, B, bias, C, Z, T, N, K, 1, s);
    dpa::launch_gemmp_nt(A, B, bias, C2, Z2, T, N, K, 1, ncu, s);
    CK(hipStreamSynchronize(s));
    printf("check gelu_fwd y maxdiff %.3e z maxdiff %.3e\n", maxdiff(C, C2, (int64_t)T * N), maxdiff(Z, Z2, (int64_t)T * N));
    // dgrad dact: dh[T][3072] = dy[T][768] . W2[768][3072] * gelu'(z)
    dpa::launch_gemm256_nn_dact(A, B, Z, C, T, 768, 3072, 1, s);
    dpa::launch_gemmp_nn(A, B, C2, Z, 1, T, 768, 3072, ncu, s, nullptr);
    CK(hipStreamSynchronize(s));
    printf("check dgelu_dgrad maxdiff %.3e\n", maxdiff(C, C2, (int64_t)T * 3072));
    // EPI 4: the column-sum partials reduce to the column sums of the (bf16) result
    dpa::launch_gemmp_nn(A, B, C2, Z, 1, T, 768, 3072, ncu, s, CP);
    CK(hipStreamSynchronize(s));
    printf("check dgelu_dgrad(EPI4) maxdiff %.3e\n", maxdiff(C, C2, (int64_t)T * 3072));
    float *cs_ref, *cs_got;
    CK(hipMalloc(&cs_ref, 3072 * 4));
    CK(hipMalloc(&cs_got, 3072 * 4));
    hipLaunchKernelGGL(colsum_bf16, dim3(12), dim3(256), 0, 0, C2, T, 3072, cs_ref);
    hipLaunchKernelGGL(colsum_f32, dim3(12), dim3(256), 0, 0, CP, (T / 256) * 2, 3072, cs_got);
    CK(hipDeviceSynchronize());
    std::vector<float> a(3072), b(3072);
    CK(hipMemcpy(a.data(), cs_ref, 3072 * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), cs_got, 3072 * 4, hipMemcpyDeviceToHost));
    double me = 0, mx = 0;
    for (int i = 0; i < 3072; ++i) { me = std::max(me, (double)fabsf(a[i] - b[i])); mx = std::max(mx, (double)fabsf(a[i])); }
    printf("check dgelu_dgrad colsum maxdiff %.3e (max %.3e)\n", me / (mx + 1e-30), mx);
    CK(hipFree(C2));
    CK(hipFree(Z2));
    fflush(stdout);
  }
  for (auto& v : vs) time_it(v, s, 2);  // warm
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vs) v.ms.push_back(time_it(v, s, iters));
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    printf("%-28s median %.4f ms  min %.4f ms  %.1f TF/s\n", v.name.c_str(), med, v.ms[0], v.flop / med / 1e9);
  }
  return 0;
}
