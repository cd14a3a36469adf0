// Simulated data plane: a one-GPU PROJECTION of the W > 1 gradient all-reduce (SURVEY 5.8, §4
// item 6; the reference's overlap is DDP's, /root/reference/utils/trainer.py:115-128, 216-220).
//
// The C++ reducer's sim mode (csrc/comm/reducer.cpp, BucketReducer::init_sim) launches, in place
// of each bucket's RCCL all-reduce, ONE comm_sim_kernel on the reducer's own high-priority comm
// stream, ordered after the bucket's grad-ready event exactly like the real collective:
//
// * `cus` workgroups (RCCL runs one workgroup per channel), each holding a CU slot for as long
//   as the collective would: t = latency + 2 (W - 1) / W x bytes / busbw, measured from the
//   workgroup's own start on the constant 100 MHz clock (s_memrealtime) - so a workgroup that
//   only gets a CU late (persistent GEMMs hold every CU) finishes late, as RCCL's would;
// * the HBM traffic of a ring all-reduce's local side: it reads and writes back 2 (W - 1) / W x
//   the bucket (values unchanged: the gradients stay this rank's, the world-1 math);
// * a timeline per bucket (first workgroup start, last workgroup end) in device memory, next
//   to the grad-ready time that a one-thread marker kernel stamps on the producing stream, so
//   the queueing delay and the exposed tail after the backward are measured, not inferred.
//
// Timeline words are written with global (vector) atomics only.
#include "common.h"
#include "launchers.h"

namespace dpa {

__device__ __forceinline__ uint64_t rt_now() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ uint32_t opaque_zero(uint32_t x) {
  uint32_t y;
  asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
  return y;
}

// tl[0] = min over workgroups of the start time, tl[1] = min over workgroups of ~(end time)
// (both start as all-ones, so one memset resets them)
__global__ void __launch_bounds__(256) comm_sim_kernel(uint4* __restrict__ buf, int64_t n16, int64_t touch16,
                                                      uint64_t ticks, unsigned long long* __restrict__ tl) {
  const uint64_t t0 = rt_now();
  if (threadIdx.x == 0) atomicMin(tl, (unsigned long long)t0);
  // the local side of the ring's HBM traffic: read + write back (unchanged) touch16 16-B words
  const uint32_t z = opaque_zero(0u);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < touch16; i += stride) {
    const int64_t j = i < n16 ? i : i % n16;
    uint4 v = buf[j];
    v.x += z;  // the compiler cannot prove the store writes back what it read
    buf[j] = v;
  }
  // hold the CU slot until this workgroup's share of the collective's time has passed
  while (rt_now() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  __syncthreads();
  if (threadIdx.x == 0) atomicMin(tl + 1, ~(unsigned long long)rt_now());
}

// one thread stamps the constant-clock time at which its stream reached this point
__global__ void time_marker_kernel(unsigned long long* __restrict__ slot) {
  if (threadIdx.x == 0) atomicMin(slot, (unsigned long long)rt_now());
}

// After a step's finalize (compute stream, behind the wait on the comm stream): per-step sums
// over its buckets, all in 10 ns ticks -
//   acc[0] += steps, acc[1] += exposed tail = max(0, last bucket end - backward end),
//   acc[2] += sum over buckets of (first workgroup start - grad ready),
//   acc[3] += sum over buckets of (last end - first start), acc[4] += busy span of the comm
//   stream (last end - first start over the step), acc[5] = last step's tail.
__global__ void comm_sim_stats_kernel(const unsigned long long* __restrict__ tl, int nb,
                                      const unsigned long long* __restrict__ bwd_end,
                                      unsigned long long* __restrict__ acc) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  unsigned long long last_end = 0, first_start = ~0ull, delay = 0, busy = 0;
  for (int b = 0; b < nb; ++b) {
    const unsigned long long ready = tl[b * 4 + 2], st = tl[b * 4], en = ~tl[b * 4 + 1];
    if (st == ~0ull) continue;  // not launched this step
    if (ready != ~0ull && st > ready) delay += st - ready;
    busy += en - st;
    last_end = en > last_end ? en : last_end;
    first_start = st < first_start ? st : first_start;
  }
  const unsigned long long be = *bwd_end;
  const unsigned long long tail = (be != ~0ull && last_end > be) ? last_end - be : 0ull;
  acc[0] += 1;
  acc[1] += tail;
  acc[2] += delay;
  acc[3] += busy;
  acc[4] += (first_start != ~0ull && last_end > first_start) ? last_end - first_start : 0ull;
  acc[5] = tail;
}

void launch_comm_sim(void* buf, int64_t bytes, int64_t touch_bytes, uint64_t ticks, int cus,
                     unsigned long long* tl, hipStream_t s) {
  const int64_t n16 = bytes / 16;
  hipLaunchKernelGGL(comm_sim_kernel, dim3(cus > 0 ? cus : 1), dim3(256), 0, s, reinterpret_cast<uint4*>(buf),
                     n16, n16 > 0 ? touch_bytes / 16 : 0, ticks, tl);
}

void launch_time_marker(unsigned long long* slot, hipStream_t s) {
  hipLaunchKernelGGL(time_marker_kernel, dim3(1), dim3(64), 0, s, slot);
}

void launch_comm_sim_stats(const unsigned long long* tl, int nb, const unsigned long long* bwd_end,
                           unsigned long long* acc, hipStream_t s) {
  hipLaunchKernelGGL(comm_sim_stats_kernel, dim3(1), dim3(64), 0, s, tl, nb, bwd_end, acc);
}

}  // namespace dpa
