// Sort-free orderings of token ids (SURVEY K-M1: the embedding gradient's segment order;
// the logged nll's masked-first order), replacing two general-purpose device sorts per step
// (at::sort of the 262144 ids: a rocprim merge sort, 2.85 ms/step, and a stable argsort of
// the 0/1 target mask) with passes whose cost is a few reads of the ids:
//
//   id_bucket_sort : STABLE counting sort of ids < 2^17 into V + 1 buckets (bucket V collects
//                    the out-of-range ids, which the segment-sum kernels skip), so that the
//                    embedding gradient's fp32 segment sums are bitwise reproducible (SURVEY 7.4
//                    hard part 2; reference utils/trainer.py:235):
//                      1. per-block histograms of SORT_BLK = 2048 tokens (LDS counters as 16-bit
//                         pairs, so a 50257-token vocabulary fits the 160 KiB LDS), dense
//                         [nblk][V + 1];
//                      2. per bucket, the exclusive prefix over blocks (one thread per bucket);
//                      3. exclusive scan of the bucket totals (bucket_scan_kernel);
//                      4. one wave per block places its tokens in index order: lanes holding the
//                         same bucket are found with 17 ballots and the group's leader takes the
//                         bucket's block-local cursor with one LDS atomic, so a token's position
//                         is off[b] + (tokens of b in earlier blocks) + (earlier tokens of b in
//                         this block) - the same on every run.
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

// ---- stable counting sort -------------------------------------------------------------
constexpr int SORT_BLK = 2048;         // tokens per block (< 2^16: counts fit 16-bit LDS halves)
constexpr int SORT_LDS_WORDS = 40960;  // 160 KiB: two 16-bit counters per word -> V + 1 <= 81920

__device__ __forceinline__ uint32_t half_of(uint32_t w, uint32_t b) { return (w >> ((b & 1u) * 16u)) & 0xffffu; }

// 1. hist[blk][b] = tokens of bucket b in block blk
__global__ void __launch_bounds__(256) id_blockhist_kernel(const int64_t* __restrict__ ids, int64_t n, int V,
                                                           int* __restrict__ hist) {
  __shared__ uint32_t c32[SORT_LDS_WORDS];
  const int nb = V + 1, nw = (nb + 1) / 2;
  for (int q = threadIdx.x; q < nw; q += blockDim.x) c32[q] = 0u;
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * SORT_BLK;
  for (int r = threadIdx.x; r < SORT_BLK; r += blockDim.x) {
    const int64_t i = t0 + r;
    if (i < n) {
      const uint32_t b = bucket_of(ids[i], V);
      atomicAdd(c32 + (b >> 1), 1u << ((b & 1u) * 16u));  // counts are order-free
    }
  }
  __syncthreads();
  int* row = hist + (int64_t)blockIdx.x * nb;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) row[b] = (int)half_of(c32[b >> 1], (uint32_t)b);
}

// 2. hist[k][b] <- sum over blocks k' < k of hist[k'][b]; tot[b] = sum over all blocks
__global__ void __launch_bounds__(256) id_colscan_kernel(int* __restrict__ hist, int nblk, int nb,
                                                         int* __restrict__ tot) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  int run = 0;
  int k = 0;
  for (; k + 8 <= nblk; k += 8) {  // 8 loads in flight per thread
    int v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = hist[(int64_t)(k + u) * nb + b];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      hist[(int64_t)(k + u) * nb + b] = run;
      run += v[u];
    }
  }
  for (; k < nblk; ++k) {
    const int v = hist[(int64_t)k * nb + b];
    hist[(int64_t)k * nb + b] = run;
    run += v;
  }
  tot[b] = run;
}

// 4. one wave per block walks its tokens in index order (32 rounds of 64)
__global__ void __launch_bounds__(64) id_stable_scatter_kernel(const int64_t* __restrict__ ids, int64_t n, int V,
                                                               const int* __restrict__ pre,
                                                               const int* __restrict__ off,
                                                               int64_t* __restrict__ sorted,
                                                               int64_t* __restrict__ perm) {
  __shared__ uint32_t c32[SORT_LDS_WORDS];
  const int nb = V + 1, nw = (nb + 1) / 2;
  const int lane = threadIdx.x;
  for (int q = lane; q < nw; q += 64) c32[q] = 0u;
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * SORT_BLK;
  const int* prow = pre + (int64_t)blockIdx.x * nb;
  constexpr int ROUNDS = SORT_BLK / 64, GROUP = 8;
  for (int r0 = 0; r0 < ROUNDS; r0 += GROUP) {
    int64_t idv[GROUP];
#pragma unroll
    for (int u = 0; u < GROUP; ++u) {  // a group of rounds' ids in flight at once
      const int64_t i = t0 + (int64_t)(r0 + u) * 64 + lane;
      idv[u] = i < n ? ids[i] : -1;
    }
#pragma unroll
    for (int u = 0; u < GROUP; ++u) {
      const int64_t base = t0 + (int64_t)(r0 + u) * 64;
      if (base < n) {  // wave-uniform
        const int64_t i = base + lane;
        const bool in = i < n;
        // tail lanes carry key 2^17 - 1 (no bucket: V + 1 <= 2^17 - 1), matching only each other
        const uint32_t b = in ? bucket_of(idv[u], V) : (1u << SORT_KEY_BITS) - 1u;
        const uint64_t m = match_key(b);
        const uint64_t lt = m & lanemask_lt();
        const int leader = __ffsll((unsigned long long)m) - 1;
        uint32_t old = 0u;
        if (in && lt == 0) old = atomicAdd(c32 + (b >> 1), (uint32_t)__popcll(m) << ((b & 1u) * 16u));
        old = __shfl(old, leader, 64);
        if (in) {
          const int64_t pos = (int64_t)off[b] + prow[b] + half_of(old, b) + __popcll(lt);
          sorted[pos] = idv[u];
          perm[pos] = i;
        }
      }
    }
  }
}

// ws: hist [nblk][V + 1], then tot and off (each 16-byte aligned)
static int64_t nblk_of(int64_t n) { return (n + SORT_BLK - 1) / SORT_BLK; }
static int64_t pad4(int64_t x) { return (x + 3) / 4 * 4; }
int64_t id_sort_workspace_ints(int64_t n, int V) { return pad4(nblk_of(n) * (V + 1)) + 2 * pad4(V + 1); }

bool launch_id_bucket_sort(const int64_t* ids, int64_t n, int V, int* ws, int64_t* sorted, int64_t* perm,
                           hipStream_t s) {
  if (V < 1 || V + 1 > 2 * SORT_LDS_WORDS || V + 1 >= (1 << SORT_KEY_BITS) - 1 || n <= 0 ||
      n > (int64_t)INT32_MAX)
    return false;
  const int nb = V + 1;
  const int64_t nblk = nblk_of(n);
  int* hist = ws;
  int* tot = ws + pad4(nblk * nb);
  int* off = tot + pad4(nb);
  hipLaunchKernelGGL(id_blockhist_kernel, dim3((unsigned)nblk), dim3(256), 0, s, ids, n, V, hist);
  hipLaunchKernelGGL(id_colscan_kernel, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, s, hist, (int)nblk, nb,
                     tot);
  // (the int4 path needs 16-byte aligned tot / off: ws from the caching allocator is)
  if (nb <= 32 * 1024 && (reinterpret_cast<uintptr_t>(tot) & 15) == 0)
    hipLaunchKernelGGL(bucket_scan_kernel<32>, dim3(1), dim3(1024), 0, s, (const int*)tot, nb, off);
  else
    hipLaunchKernelGGL(bucket_scan_kernel<0>, dim3(1), dim3(1024), 0, s, (const int*)tot, nb, off);
  hipLaunchKernelGGL(id_stable_scatter_kernel, dim3((unsigned)nblk), dim3(64), 0, s, ids, n, V, (const int*)hist,
                     (const int*)off, sorted, perm);
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
