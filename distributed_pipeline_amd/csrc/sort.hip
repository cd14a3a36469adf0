// Sort-free orderings of token ids (SURVEY K-M1: the embedding gradient's segment order;
// the logged nll's masked-first order), replacing two general-purpose device sorts per step
// (at::sort of the 262144 ids: a rocprim merge sort, 2.85 ms/step, and a stable argsort of
// the 0/1 target mask) with passes whose cost is a few reads of the ids:
//
//   id_bucket_sort : counting sort of ids < 2^17 into V + 1 buckets (bucket V collects the
//                    out-of-range ids, which the segment-sum kernels skip):
//                    histogram -> exclusive scan -> scatter.  Histogram and scatter aggregate
//                    per wave: lanes holding the same bucket are found with 17 ballots (one
//                    per key bit) and one lane issues the wave's atomic for the group, so a
//                    frequent id (a padding token in real data) costs one atomic per wave, not
//                    one per token.  The order inside a bucket is the atomics' order (not
//                    stable); the embedding gradient only needs equal ids adjacent.
//   partition01    : stable partition of a 0/1 mask (nonzero first) -> the permutation.  Block
//                    counts, then each block scans the counts before it and places its
//                    elements with wave ballots (one 64-lane prefix per instruction).
#include "common.h"
#include "launchers.h"

namespace dpa {

constexpr int SORT_KEY_BITS = 17;

__device__ __forceinline__ uint64_t lanemask_lt() {
  const int lane = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  return (1ull << lane) - 1ull;
}

// lanes of the wave (among the active ones) whose key equals this lane's
__device__ __forceinline__ uint64_t match_key(uint32_t key) {
  uint64_t m = __ballot(1);
#pragma unroll
  for (int b = 0; b < SORT_KEY_BITS; ++b) {
    const bool bit = (key >> b) & 1u;
    const uint64_t bal = __ballot(bit);
    m &= bit ? bal : ~bal;
  }
  return m;
}

__device__ __forceinline__ uint32_t bucket_of(int64_t id, int V) {
  return (id >= 0 && id < V) ? (uint32_t)id : (uint32_t)V;
}

// grid-stride over ids: cnt[bucket] += 1 (one atomic per distinct bucket per wave)
__global__ void __launch_bounds__(256) id_hist_kernel(const int64_t* __restrict__ ids, int64_t n, int V,
                                                      int* __restrict__ cnt) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  // whole waves iterate together (every lane runs the same number of iterations; tail lanes
  // are inactive inside the body) so the ballots see the full wave
  const int64_t base0 = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63);
  for (int64_t base = base0; base < n; base += stride) {
    const int64_t i = base + (threadIdx.x & 63);
    if (i < n) {
      const uint32_t b = bucket_of(ids[i], V);
      const uint64_t m = match_key(b);
      if ((m & lanemask_lt()) == 0) atomicAdd(cnt + b, (int)__popcll(m));
    }
  }
}

// exclusive scan of cnt[0..nb) into off[0..nb) by one 1024-thread block: thread t owns the
// contiguous run [t * PER, t * PER + PER) (PER = 0: ceil(nb / 1024), generic loops); off doubles
// as the scatter cursor.  PER = 32 (nb <= 32768: BERT's 30522 + 1 buckets) loads and stores its
// run as 8 int4 issued back to back - one memory latency per pass instead of PER dependent
// ones (24 us -> a few per call; the reference schedule sorts twice per micro-batch).
template <int PER>
__global__ void __launch_bounds__(1024) bucket_scan_kernel(const int* __restrict__ cnt, int nb,
                                                           int* __restrict__ off) {
  __shared__ int wsum[16];
  const int t = threadIdx.x;
  const int per = PER > 0 ? PER : (nb + 1023) / 1024;
  const int b0 = t * per, b1 = min(nb, b0 + per);
  int v[PER > 0 ? PER : 1];
  int s = 0;
  if constexpr (PER > 0) {
#pragma unroll
    for (int q = 0; q < PER / 4; ++q) {
      const int b = b0 + 4 * q;
      if (b + 3 < nb) {
        const int4 x = *reinterpret_cast<const int4*>(cnt + b);
        v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * q + e] = b + e < nb ? cnt[b + e] : 0;
      }
    }
#pragma unroll
    for (int e = 0; e < PER; ++e) s += v[e];
  } else {
    for (int b = b0; b < b1; ++b) s += cnt[b];
  }
  // inclusive scan of s over the block: wave scan by shuffles, then the 16 wave totals
  const int lane = t & 63, w = t >> 6;
  int x = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  int wpre = 0;
  for (int k = 0; k < w; ++k) wpre += wsum[k];
  int run = wpre + x - s;  // exclusive prefix of this thread's run
  if constexpr (PER > 0) {
#pragma unroll
    for (int q = 0; q < PER / 4; ++q) {
      const int b = b0 + 4 * q;
      int o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] = run;
        run += v[4 * q + e];
      }
      if (b + 3 < nb) {
        *reinterpret_cast<int4*>(off + b) = make_int4(o[0], o[1], o[2], o[3]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (b + e < nb) off[b + e] = o[e];
      }
    }
  } else {
    for (int b = b0; b < b1; ++b) {
      off[b] = run;
      run += cnt[b];
    }
  }
}

// pos = cur[bucket]++ per token (one atomic per distinct bucket per wave): sorted[pos] = id,
// perm[pos] = token index
__global__ void __launch_bounds__(256) id_scatter_kernel(const int64_t* __restrict__ ids, int64_t n, int V,
                                                         int* __restrict__ cur, int64_t* __restrict__ sorted,
                                                         int64_t* __restrict__ perm) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t base0 = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63);
  for (int64_t base = base0; base < n; base += stride) {
    const int64_t i = base + (threadIdx.x & 63);
    if (i < n) {
      const int64_t id = ids[i];
      const uint32_t b = bucket_of(id, V);
      const uint64_t m = match_key(b);
      const uint64_t lt = m & lanemask_lt();
      const int leader = __ffsll((unsigned long long)m) - 1;
      int p0 = 0;
      if (lt == 0) p0 = atomicAdd(cur + b, (int)__popcll(m));
      p0 = __shfl(p0, leader, 64);
      const int64_t pos = (int64_t)p0 + __popcll(lt);
      sorted[pos] = id;
      perm[pos] = i;
    }
  }
}

// cnt[0..nb) then off at the next multiple of 4 ints (16-byte aligned for the int4 scan)
static int64_t id_sort_off(int V) { return ((int64_t)V + 1 + 3) / 4 * 4; }
int64_t id_sort_workspace_ints(int V) { return id_sort_off(V) + V + 1; }

bool launch_id_bucket_sort(const int64_t* ids, int64_t n, int V, int* ws, int64_t* sorted, int64_t* perm,
                           hipStream_t s) {
  if (V < 1 || V >= (1 << SORT_KEY_BITS) || n <= 0 || n > (int64_t)INT32_MAX) return false;
  const int nb = V + 1;
  int* cnt = ws;
  int* off = ws + id_sort_off(V);
  if (hipMemsetAsync(cnt, 0, sizeof(int) * nb, s) != hipSuccess) return false;
  int64_t g = (n + 255) / 256;
  const unsigned grid = (unsigned)(g > 2048 ? 2048 : g);
  hipLaunchKernelGGL(id_hist_kernel, dim3(grid), dim3(256), 0, s, ids, n, V, cnt);
  // (the int4 path needs 16-byte aligned cnt / off: ws from the caching allocator is)
  if (nb <= 32 * 1024 && (reinterpret_cast<uintptr_t>(ws) & 15) == 0)
    hipLaunchKernelGGL(bucket_scan_kernel<32>, dim3(1), dim3(1024), 0, s, (const int*)cnt, nb, off);
  else
    hipLaunchKernelGGL(bucket_scan_kernel<0>, dim3(1), dim3(1024), 0, s, (const int*)cnt, nb, off);
  hipLaunchKernelGGL(id_scatter_kernel, dim3(grid), dim3(256), 0, s, ids, n, V, off, sorted, perm);
  return true;
}

// ---- stable 0/1 partition ---------------------------------------------------------------
constexpr int PART_TILE = 1024;  // elements per block (4 rounds of 256 threads)

__global__ void __launch_bounds__(256) part_count_kernel(const int64_t* __restrict__ mask, int64_t n,
                                                         int* __restrict__ blk) {
  __shared__ int ws[4];
  const int64_t t0 = (int64_t)blockIdx.x * PART_TILE;
  int c = 0;
  for (int r = 0; r < PART_TILE / 256; ++r) {
    const int64_t i = t0 + r * 256 + threadIdx.x;
    c += (i < n && mask[i] != 0) ? 1 : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) blk[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ void __launch_bounds__(256) part_place_kernel(const int64_t* __restrict__ mask, int64_t n, int nblk,
                                                         const int* __restrict__ blk, int64_t* __restrict__ order) {
  __shared__ int red[2][4];
  __shared__ int wc[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // ones before this block and in total (each block scans the per-block counts itself)
  int before = 0, total = 0;
  for (int b = threadIdx.x; b < nblk; b += 256) {
    const int v = blk[b];
    total += v;
    before += b < (int)blockIdx.x ? v : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    before += __shfl_xor(before, o, 64);
    total += __shfl_xor(total, o, 64);
  }
  if (lane == 0) {
    red[0][w] = before;
    red[1][w] = total;
  }
  __syncthreads();
  int64_t ones = red[0][0] + red[0][1] + red[0][2] + red[0][3];
  const int64_t tot = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  const int64_t t0 = (int64_t)blockIdx.x * PART_TILE;
  int64_t zeros = tot + (t0 - ones);  // zeros go after every one, in index order
  for (int r = 0; r < PART_TILE / 256; ++r) {
    const int64_t i = t0 + r * 256 + threadIdx.x;
    const bool in = i < n;
    const bool one = in && mask[i] != 0;
    const uint64_t b1 = __ballot(one), bin = __ballot(in);
    if (lane == 0) wc[w] = (int)__popcll(b1);
    __syncthreads();
    int pre1 = 0, pre_in = 0;
    for (int k = 0; k < w; ++k) {
      pre1 += wc[k];
      pre_in += 64;
    }
    const int r1 = pre1 + (int)__popcll(b1 & lanemask_lt());
    const int rin = pre_in + (int)__popcll(bin & lanemask_lt());
    if (in) order[one ? ones + r1 : zeros + (rin - r1)] = i;
    const int round1 = wc[0] + wc[1] + wc[2] + wc[3];
    __syncthreads();  // wc is rewritten by the next round
    ones += round1;
    zeros += 256 - round1;
  }
}

bool launch_partition01(const int64_t* mask, int64_t n, int* blk_ws, int64_t* order, hipStream_t s) {
  if (n <= 0) return false;
  const int64_t nblk = (n + PART_TILE - 1) / PART_TILE;
  if (nblk > (1 << 20)) return false;
  hipLaunchKernelGGL(part_count_kernel, dim3((unsigned)nblk), dim3(256), 0, s, mask, n, blk_ws);
  hipLaunchKernelGGL(part_place_kernel, dim3((unsigned)nblk), dim3(256), 0, s, mask, n, (int)nblk,
                     (const int*)blk_ws, order);
  return true;
}

int64_t partition01_workspace_ints(int64_t n) { return (n + PART_TILE - 1) / PART_TILE; }

}  // namespace dpa
