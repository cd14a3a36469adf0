// Direct single-node all-reduce over xGMI through IPC-mapped peer buffers
// (SURVEY 5.8 / 7.4 item 4): the opt-in alternative to RCCL rings for the
// gradient buckets (DPA_IPC_ALLREDUCE=1, csrc/comm/reducer.cpp).
//
// A ring all-reduce crosses ONE xGMI link per hop, so on a fully connected
// 8-GPU MI355X node it runs at one link's bandwidth (~153 GB/s x N/(2(N-1))).
// Here every rank reads its peers' buffers directly, so all 7 links of a GPU
// carry traffic at once:
//   one-shot (small buckets): every rank stages its slice, then sums the same
//     slice of all W staging buffers ((W-1) n remote reads per rank, 1 launch,
//     lowest latency);
//   two-shot (large buckets): slice b is reduced only by its owner rank b % W
//     (reduce-scatter: (W-1)/W n reads), written back into the owner's staging
//     buffer, then every other rank copies it (all-gather: (W-1)/W n reads).
//
// Signalling (MI355X_MICROARCH "Valid forms", at SYSTEM scope because the
// consumers sit on other devices): a block's stores -> s_waitcnt vmcnt(0) ->
// barrier -> lane 0 release fence + relaxed flag store (an epoch counter);
// consumer lane 0 polls the flag relaxed, one acquire fence, barrier, then
// plain loads.  Flags are per (rank, parity, phase, block): block b of rank r
// only ever reads slice b, so "block b of every peer posted call e+1" implies
// "they finished reading call e's slice b", and two parity halves of the staging
// buffer make reuse safe without an extra barrier.  Every spin is bounded
// (20 s): on timeout the kernel sets *err and returns instead of hanging; the fused
// AdamW then skips the step and the DDP engine raises (parallel/ddp.py).
//
// Single-GPU testing: gridDim.y = W simulated ranks in ONE launch (all blocks
// co-resident), each block y acting as rank y - the exact per-rank code path.
#include "common.h"
#include "launchers.h"

namespace dpa {

constexpr int IPC_NBMAX = 1024;  // flag slots per (parity, phase)

__device__ __forceinline__ void ipc_publish(uint32_t* flag, uint32_t epoch) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// lane 0 of the block waits until every flag in flags[0..n) (stride apart) equals
// epoch; returns false on timeout.  All threads return the same value.
__device__ __forceinline__ bool ipc_wait(uint32_t* const* flags, int n, int64_t idx, uint32_t epoch,
                                         int* err, int* sh) {
  if (threadIdx.x == 0) {
    int ok = 1;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int s = 0; s < n && ok; ++s) {
      while (__hip_atomic_load(flags[s] + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
        __builtin_amdgcn_s_sleep(2);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000000ull) {  // 20 s at 100 MHz
          ok = 0;
          atomicOr(err, 1);
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    *sh = ok;
  }
  __syncthreads();
  return *sh != 0;
}

__global__ void __launch_bounds__(256) ipc_allreduce_kernel(IpcPeers peers, IpcData data, int W, int rank,
                                                            int64_t n, int64_t cap, uint32_t epoch,
                                                            int two_shot, int* err) {
  __shared__ int sh;
  const int R = gridDim.y > 1 ? (int)blockIdx.y : rank;
  const int b = blockIdx.x, NB = gridDim.x;
  const int par = epoch & 1;
  const int64_t per = ((n + NB - 1) / NB + 3) & ~(int64_t)3;
  const int64_t lo = (int64_t)b * per, hi = lo + per < n ? lo + per : n;
  float* io = data.p[R];
  float* mine = peers.stage[R] + par * cap;
  // 1. stage this rank's slice b where the peers can read it
  for (int64_t i = lo + threadIdx.x * 4; i < hi; i += blockDim.x * 4)
    *reinterpret_cast<f32x4*>(mine + i) = *reinterpret_cast<const f32x4*>(io + i);
  const int64_t f0 = (int64_t)(par * 2 + 0) * IPC_NBMAX + b, f1 = (int64_t)(par * 2 + 1) * IPC_NBMAX + b;
  ipc_publish(peers.flags[R] + f0, epoch);
  if (!two_shot) {
    if (!ipc_wait(peers.flags, W, f0, epoch, err, &sh)) return;
    for (int64_t i = lo + threadIdx.x * 4; i < hi; i += blockDim.x * 4) {
      f32x4 acc = *reinterpret_cast<const f32x4*>(peers.stage[0] + par * cap + i);
      for (int s = 1; s < W; ++s) acc += *reinterpret_cast<const f32x4*>(peers.stage[s] + par * cap + i);
      *reinterpret_cast<f32x4*>(io + i) = acc;
    }
    return;
  }
  const int owner = b % W;
  if (owner == R) {
    // reduce-scatter: the owner sums slice b of every rank into its own staging slice
    if (!ipc_wait(peers.flags, W, f0, epoch, err, &sh)) return;
    for (int64_t i = lo + threadIdx.x * 4; i < hi; i += blockDim.x * 4) {
      f32x4 acc = *reinterpret_cast<const f32x4*>(peers.stage[0] + par * cap + i);
      for (int s = 1; s < W; ++s) acc += *reinterpret_cast<const f32x4*>(peers.stage[s] + par * cap + i);
      *reinterpret_cast<f32x4*>(mine + i) = acc;
      *reinterpret_cast<f32x4*>(io + i) = acc;
    }
    ipc_publish(peers.flags[R] + f1, epoch);
  } else {
    // all-gather: copy the owner's reduced slice
    uint32_t* const owner_flags[1] = {peers.flags[owner]};
    if (!ipc_wait(owner_flags, 1, f1, epoch, err, &sh)) return;
    const float* src = peers.stage[owner] + par * cap;
    for (int64_t i = lo + threadIdx.x * 4; i < hi; i += blockDim.x * 4)
      *reinterpret_cast<f32x4*>(io + i) = *reinterpret_cast<const f32x4*>(src + i);
  }
}

int ipc_allreduce_blocks(int64_t n, int W, bool two_shot) {
  // ~64 KiB per block; two-shot wants a multiple of W blocks so every rank owns slices
  int64_t nb = (n * 4 + 65535) / 65536;
  if (two_shot) nb = (nb + W - 1) / W * W;
  if (nb < 1) nb = 1;
  if (nb > IPC_NBMAX) nb = IPC_NBMAX / W * W;
  return (int)nb;
}

bool launch_ipc_allreduce(const IpcPeers& peers, const IpcData& data, int W, int rank, int sim_ranks,
                          int64_t n, int64_t cap, uint32_t epoch, bool two_shot, int* err, hipStream_t s) {
  if (W < 1 || W > IPC_MAXW || n % 4 || cap % 4 || n > cap || (sim_ranks != 1 && sim_ranks != W)) return false;
  for (int r = 0; r < W; ++r) {
    const float* io = data.p[sim_ranks == 1 ? rank : r];
    if (!io || (reinterpret_cast<uintptr_t>(io) & 15) || !peers.stage[r] || !peers.flags[r] ||
        (reinterpret_cast<uintptr_t>(peers.stage[r]) & 15))
      return false;
  }
  const int nb = ipc_allreduce_blocks(n, W, two_shot);
  hipLaunchKernelGGL(ipc_allreduce_kernel, dim3(nb, sim_ranks), dim3(256), 0, s, peers, data, W, rank, n, cap,
                     epoch, two_shot ? 1 : 0, err);
  return true;
}

}  // namespace dpa
