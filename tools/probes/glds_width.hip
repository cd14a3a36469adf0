// Probe: LDS layout written by global_load_lds with 1/2/4-byte widths
// (is the LDS destination base + lane*size or base + lane*4?).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void glob_void;

template <int SZ>
__global__ void probe(const uint8_t* src, uint32_t* out) {
  __shared__ uint32_t lds[128];
  for (int i = threadIdx.x; i < 128; i += 64) lds[i] = 0xdeadbeefu;
  __syncthreads();
  if constexpr (SZ == 2)
    __builtin_amdgcn_global_load_lds((glob_void*)(src + threadIdx.x * SZ), (lds_void*)lds, 2, 0, 0);
  else
    __builtin_amdgcn_global_load_lds((glob_void*)(src + threadIdx.x * SZ), (lds_void*)lds, 1, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 128; i += 64) out[i] = lds[i];
}

int main() {
  uint8_t h[512];
  for (int i = 0; i < 512; ++i) h[i] = (uint8_t)i;
  uint8_t* d; uint32_t* o; uint32_t ho[128];
  (void)hipMalloc(&d, 512); (void)hipMalloc(&o, 512);
  (void)hipMemcpy(d, h, 512, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe<2>, dim3(1), dim3(64), 0, 0, d, o);
  (void)hipMemcpy(ho, o, 512, hipMemcpyDeviceToHost);
  printf("size2:"); for (int i = 0; i < 8; ++i) printf(" %08x", ho[i]); printf(" ... [64]=%08x\n", ho[64]);
  hipLaunchKernelGGL(probe<1>, dim3(1), dim3(64), 0, 0, d, o);
  (void)hipMemcpy(ho, o, 512, hipMemcpyDeviceToHost);
  printf("size1:"); for (int i = 0; i < 8; ++i) printf(" %08x", ho[i]); printf(" ... [32]=%08x\n", ho[32]);
  return 0;
}
