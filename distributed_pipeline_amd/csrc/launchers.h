// Host-side launch entry points of the gfx950 kernels.  Kernels live in the
// .hip translation units (which include no torch headers, so they compile in
// seconds); bindings.cpp is the only TU that sees ATen.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dpa {

// ---- ipc_allreduce.hip: direct xGMI all-reduce over IPC-mapped peer buffers ----
constexpr int IPC_MAXW = 8;
struct IpcPeers {            // per rank: staging buffer (2 parity halves of `cap` floats) and flags
  float* stage[IPC_MAXW];
  uint32_t* flags[IPC_MAXW];
};
struct IpcData {             // in/out buffer of each (simulated) rank; real runs use p[rank]
  float* p[IPC_MAXW];
};
constexpr int64_t IPC_FLAG_WORDS = 4 * 1024;  // [2 parity][2 phase][IPC_NBMAX]
int ipc_allreduce_blocks(int64_t n, int W, bool two_shot);
// sim_ranks == W: one launch plays all W ranks on one device (tests); 1: this rank only.
bool launch_ipc_allreduce(const IpcPeers& peers, const IpcData& data, int W, int rank, int sim_ranks,
                          int64_t n, int64_t cap, uint32_t epoch, bool two_shot, int* err, hipStream_t s);

// ---- comm_sim.hip: one-GPU projection of the W > 1 data plane (reducer sim mode) ----
// tl: this bucket's timeline words {first start, ~last end} (both reset to all-ones)
void launch_comm_sim(void* buf, int64_t bytes, int64_t touch_bytes, uint64_t ticks, int cus,
                     unsigned long long* tl, hipStream_t s);
void launch_time_marker(unsigned long long* slot, hipStream_t s);
void launch_comm_sim_stats(const unsigned long long* tl, int nb, const unsigned long long* bwd_end,
                           unsigned long long* acc, hipStream_t s);

// ---- wgrad4w.hip: one-wave-per-SIMD weight gradient (both operands token-major) ----
bool launch_wgrad4w(const uint16_t* const* as, const uint16_t* const* bs, int nseg, int T, int M, int N, int splits,
                    int kps, float* dW, float* ws, hipStream_t s);
void set_wgrad4w(bool on);  // gemm256.hip: route db-free weight gradients to wgrad4w (default off: measured no faster)

// ---- optim.hip -------------------------------------------------------------
void launch_sqnorm(const void* g, bool g_bf16, int64_t n, float* partial, int nparts, float scale,
                   float max_norm, float* out, hipStream_t s);
void launch_adamw_ema(float* p, const void* g, bool g_bf16, float* m, float* v, uint16_t* p16,
                      float* const* ema_bufs, const float* ema_rates, int n_ema, int64_t n, float lr,
                      float beta1, float beta2, float eps, float wd, int64_t step, float grad_scale,
                      const float* clip, hipStream_t s,
                      const int* skip = nullptr);
void launch_ema(float* e, const float* p, int64_t n, float rate, hipStream_t s);
void launch_cast_bf16(const float* src, uint16_t* dst, int64_t n, hipStream_t s);
// dst_i = src_i^T for up to MAXN bf16 matrices [rows_i][cols_i] (multiples of 64), one launch;
// tile_start = prefix sums of (rows / 64) * (cols / 64), tile_start[n] = total
struct TransposeBatch {
  static constexpr int MAXN = 96;
  const uint16_t* src[MAXN];
  uint16_t* dst[MAXN];
  int rows[MAXN], cols[MAXN], tile_start[MAXN + 1];
  int n;
};
bool launch_transpose_bf16_batch(const TransposeBatch& d, hipStream_t s);
void launch_cast_f32(const uint16_t* src, float* dst, int64_t n, hipStream_t s);  // n % 4 == 0

// ---- xent.hip (fused linear + cross-entropy) ----------------------------------
int64_t lxent_workspace_floats(int N, int V);
// forward + unscaled input gradient in one sweep: dxu[t] = softmax_t . W - W[target_t] (fp32)
void launch_lxent_fwd_dx(const uint16_t* x, const uint16_t* W, const uint16_t* b, const int64_t* tgt,
                         int N, int V, int E, float* loss, float* lse, float* dxu, hipStream_t s,
                         float* ws = nullptr);
// fp32 workspace of the vocabulary-split fused forward (0: no split for this shape)
int64_t lxent_fwd_dx_workspace_floats(int N, int V, int E);
bool lxent_dx_needs_acc(int N);
void launch_lxent_fwd(const uint16_t* x, const uint16_t* W, const uint16_t* b, const int64_t* tgt,
                      int N, int V, int E, float* loss, float* lse, float* ws, hipStream_t s);
void launch_lxent_dx(const uint16_t* x, const uint16_t* W, const uint16_t* b, const int64_t* tgt,
                     const float* lse, const float* dloss, int N, int V, int E, uint16_t* dx,
                     float* dx_acc, hipStream_t s);
// dW (+ db) += the head gradient; ws: lxent_dw_ws_floats(N, V, E) floats of scratch when that is
// > 0 (the token splits' partials, summed in split order: deterministic)
int64_t lxent_dw_ws_floats(int N, int V, int E);
void launch_lxent_dw(const uint16_t* x, const uint16_t* W, const uint16_t* b, const int64_t* tgt,
                     const float* lse, const float* dloss, int N, int V, int E, float* dW, float* db,
                     hipStream_t s, bool onehot, float* ws);

// ---- norm.hip (fused dropout + residual + LayerNorm) ---------------------------
bool launch_add_ln_fwd(const uint16_t* y, const uint16_t* res, const uint16_t* g, const uint16_t* b,
                       uint16_t* out, uint16_t* hsave, float* mean, float* rstd, int64_t R, int D,
                       float p, float eps, uint32_t seed, uint32_t off, hipStream_t s,
                       const uint16_t* pos = nullptr, const uint16_t* temb = nullptr, int L = 1,
                       bool post = false, bool hguard = false);  // hguard: write hsave only if some |gamma| is small
int ln_bwd_blocks(int64_t R);
// dyb (nullable): column sums of dy (the bias gradient of the layer producing y)
bool launch_add_ln_bwd(const uint16_t* dout, const uint16_t* hsave, const float* mean,
                       const float* rstd, const uint16_t* g, uint16_t* dres, uint16_t* dy, float* dyb,
                       float* dg, float* db, int64_t R, int D, float p, uint32_t seed, uint32_t off,
                       hipStream_t s, const uint16_t* dh_in = nullptr, bool post = false,
                       int zero_mask = 7, float* ws = nullptr, int part_mode = 0,
                       const uint16_t* beta = nullptr,    // beta: `hsave` is the LN output ...
                       const uint16_t* hcopy = nullptr,   // ... and hcopy the guarded h copy
                       bool pair_hash = false);           // dy's dropout bits: common.h pair_hash
// the deferred second stage of part_mode 1/2 (R = the rows of each summed micro-batch); consumes
// the partials (ordered two-pass sums, no atomics)
bool launch_ln_colreduce(float* part, int64_t R, int D, float* dg, float* db, float* dyb, hipStream_t s);
// dpos[L][H] (zeroed; += sum over b) and dtemb[B][H] (= sum over l) of a [B][L][H] bf16 gradient in
// one read; part: seq_pos_groups(B) * L * H floats of workspace.  L in {64, 128, 256}, H % 64 == 0.
int seq_pos_groups(int B);
bool launch_seq_pos_sums(const uint16_t* d, int B, int L, int H, float* dpos, float* dtemb, float* part,
                         hipStream_t s);
// dst[c] += sum_r part[r][c] in a fixed order (deterministic); consumes part
bool launch_colsum_acc(float* part, int rows, int cols, float* dst, hipStream_t s);
// fp32 workspace (floats) the small-R two-stage column sums of launch_add_ln_bwd use (0: none)
int64_t ln_bwd_ws_floats(int64_t R, int D);

// ---- elementwise.hip (bias + activation epilogues) -------------------------------
void launch_bias_act_fwd(uint16_t* z, const uint16_t* bias, uint16_t* y, int64_t R, int N, int act,
                         hipStream_t s);
// db (nullable) += column sums of dz, through ws = bias_act_bwd_ws_floats(R, N) floats of scratch
// (row-block partials summed in order: deterministic); ws is required when db is given
int64_t bias_act_bwd_ws_floats(int64_t R, int N);
void launch_bias_act_bwd(const uint16_t* dy, const uint16_t* zy, uint16_t* dz, float* db, int64_t R,
                         int N, int act, hipStream_t s, float* ws);

// ---- attention.hip (head_dim 64 or 128, dropout, causal) ---------------------------------
// head_major: qkv is [B, 3H, L, D] (QKV GEMM head-major store; L == 128, D == 64, bidirectional only)
bool launch_attn_fwd(const uint16_t* qkv, uint16_t* out, float* lse, int B, int L, int H, int D,
                     float p, bool causal, uint32_t seed, uint32_t offset, hipStream_t s,
                     bool head_major = false);
bool attn128_supports(int L, int D, bool causal);
bool attn_bwd_needs_dq_acc(int L);
// attention128.hip: persistent L = 128 bidirectional kernels (false: not applicable)
bool launch_attn128_bwd_d128(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout, const float* lse,
                             float* delta, uint16_t* dqkv, int B, int L, int H, float p, bool causal,
                             uint32_t seed, uint32_t offset, hipStream_t s, float* colpart = nullptr);
// attention backward bias-gradient partials: rows of the colpart scratch ([rows][3 D] fp32) and
// the reduce pass db[3 H D] += column sums
int64_t attn_colpart_rows(int B, int L, int H, int D, bool causal);
void launch_colpart_reduce(float* colpart, float* db, int R, int H, int D, hipStream_t s);  // consumes colpart
bool launch_attn128_fwd_d128(const uint16_t* qkv, uint16_t* out, float* lse, int B, int L, int H,
                             float p, bool causal, uint32_t seed, uint32_t offset, hipStream_t s);
bool launch_attn128_fwd(const uint16_t* qkv, uint16_t* out, float* lse, int B, int L, int H,
                        float p, bool causal, uint32_t seed, uint32_t offset, hipStream_t s,
                        bool head_major = false);
// colpart [B*H][192] fp32 scratch; when dbias != nullptr also writes the column sums of
// dqkv (the qkv bias gradient) into dbias [3*H*64] (overwritten).
bool launch_attn128_bwd(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout,
                        const float* lse, uint16_t* dqkv, float* colpart, float* dbias, int B,
                        int L, int H, float p, bool causal, uint32_t seed, uint32_t offset,
                        hipStream_t s, bool head_major = false, bool db_accumulate = false,
                        bool defer_reduce = false);
// Returns true when the column sums of dqkv were written to dbias (L == 128 path).  defer_reduce:
// the column-sum partials stay in colpart (dbias untouched) for one launch_colpart_reduce over
// several calls' partials (the reference schedule's deferral window).
bool launch_attn_bwd(const uint16_t* qkv, const uint16_t* out, const uint16_t* dout, const float* lse,
                     float* delta, uint16_t* dqkv, float* dq_acc, float* colpart, float* dbias, int B,
                     int L, int H, int D, float p, bool causal, uint32_t seed, uint32_t offset,
                     hipStream_t s, bool head_major = false, bool db_accumulate = false,
                     bool defer_reduce = false);

// ---- xent_rows.hip: row softmax-CE over materialised logits (wide-E chunked path) ----
// forward that leaves softmax - onehot (unscaled) in place of the logits (false: row too long)
bool launch_xent_rows_fwd_grad(uint16_t* lg, int64_t ld, int V, const int64_t* tgt, int64_t R, float* loss,
                               float* lse, hipStream_t s);
bool launch_xent_rows_fwd(const uint16_t* lg, int64_t ld, int V, const int64_t* tgt, int64_t R,
                          float* loss, float* lse, hipStream_t s);
bool launch_xent_rows_bwd(uint16_t* lg, int64_t ld, int V, const int64_t* tgt, const float* lse,
                          const float* dloss, int64_t R, hipStream_t s);

// ---- diffusion.hip: DiffuSeq q_sample / diffusion losses / timestep embedding ------
bool launch_emb_qsample_fwd(const int64_t* ids, const int64_t* mask, const int64_t* t, const float* W,
                            const float* sa, const float* s1a, int64_t NT, int L, int E, int V,
                            float std0, uint32_t seed, uint32_t offset, float* x_start,
                            uint16_t* x_start16, uint16_t* x_t, hipStream_t s);
// Deterministic segment sums over a STABLE sort: part = emb_grad_part_floats(NT, E, qsample) fp32
// scratch (qsample: for launch_emb_qsample_bwd, else launch_emb_grad)
int64_t emb_grad_part_floats(int64_t NT, int E, bool qsample);
bool launch_emb_grad(const int64_t* sorted_ids, const int64_t* perm, const float* dy32, const uint16_t* dy16,
                     int64_t NT, int E, int V, float* dW, float* part, hipStream_t s);
bool launch_emb_qsample_bwd(const int64_t* ids, const int64_t* mask, const int64_t* t, const float* sa,
                            const float* d_xs, const uint16_t* d_xs16, const uint16_t* d_xt16,
                            const float* d_xt32, int64_t NT, int L, int E, int V, float* dW,
                            hipStream_t s, const int64_t* sorted_ids = nullptr,
                            const int64_t* perm = nullptr, float* part = nullptr);
bool launch_diff_loss_fwd(const float* x_start, const void* out, bool out_bf16, const int64_t* ids,
                          const int64_t* t, const float* W, int B, int L, int E, int V, float sa_last,
                          float* mse, float* tT, hipStream_t s);
bool launch_diff_loss_bwd(const float* x_start, const void* out, bool out_bf16, const int64_t* ids,
                          const int64_t* t, const float* W, const float* dmse, const float* dtT, int B,
                          int L, int E, int V, float sa_last, void* d_out, float* d_xs, float* dW,
                          hipStream_t s, bool fold_t0 = false);  // fold_t0: the t == 0 W term into d_xs
void launch_timestep_emb(const float* ts, int B, int dim, float max_period, uint16_t* out,
                         hipStream_t s);

// ---- sort.hip: counting sort of token ids, stable 0/1 partition ---------------------
// STABLE counting sort of ids into V + 1 buckets (out-of-range ids -> bucket V); ws:
// id_sort_workspace_ints(n, V) ints.  Equal ids end up adjacent in index order (the same
// permutation on every run).  false: V + 1 > 81920 or n == 0.
int64_t id_sort_workspace_ints(int64_t n, int V);
bool launch_id_bucket_sort(const int64_t* ids, int64_t n, int V, int* ws, int64_t* sorted, int64_t* perm,
                           hipStream_t s);
// order = indices of the nonzero mask entries, then of the zero ones, each in index order
int64_t partition01_workspace_ints(int64_t n);
bool launch_partition01(const int64_t* mask, int64_t n, int* blk_ws, int64_t* order, hipStream_t s);

// ---- gemm.hip (bf16 MFMA GEMMs of Linear layers) ----------------------------------
bool launch_gemm_nt(const uint16_t* x, const uint16_t* W, const uint16_t* bias, uint16_t* y,
                    uint16_t* z, int T, int N, int K, int act, hipStream_t s,
                    bool* zderiv = nullptr, int hm = 0);
bool launch_gemm_nn(const uint16_t* dy, const uint16_t* W, uint16_t* dx, int T, int N, int K,
                    hipStream_t s, const uint16_t* WT = nullptr);
bool launch_gemm_wgrad(const uint16_t* dy, const uint16_t* x, float* dW, float* db, int T, int N,
                       int K, hipStream_t s, float* ws = nullptr);
// gemm256.hip: 256x256 8-phase variants (return false when the shape does not tile
// or DPA_GEMM256=0); the launch_gemm_* entry points try them first.
bool launch_gemm256_nt(const uint16_t* x, const uint16_t* W, const uint16_t* bias, uint16_t* y,
                       uint16_t* z, int T, int N, int K, int act, hipStream_t s);
bool launch_gemm256_nn(const uint16_t* dy, const uint16_t* W, uint16_t* dx, int T, int N, int K,
                       hipStream_t s);
void set_gemm256(bool on);
void set_gemmp_dynamic(bool on);  // dynamic tile schedule of the persistent GEMMs (world > 1)
void set_gemmp_grid_cap(int cap);  // persistent-GEMM grid cap (0 = #CUs)
void set_gemmp_half(int mode);     // 128-row tiles: 0 off, 1 auto (occupancy rule), 2 always
bool launch_gemm256_nn_dact(const uint16_t* dy, const uint16_t* W, const uint16_t* aux,
                            uint16_t* dz, int T, int N, int K, int act, hipStream_t s);
bool launch_gemm256_wgrad(const uint16_t* dy, const uint16_t* x, float* dW, float* db, int T,
                          int N, int K, hipStream_t s, float* ws = nullptr);
// fp32 workspace the split-K weight gradient merges through (0: atomics / no split)
int64_t gemm256_wgrad_workspace_floats(int T, int N, int K, int nseg = 1);
// dW += sum_s dy_s^T x_s over nseg (<= 8) equal token segments in one split-K launch
bool launch_gemm256_wgrad_multi(const uint16_t* const* dys, const uint16_t* const* xs, int nseg, float* dW,
                                float* db, int T, int N, int K, hipStream_t s, float* ws);
// Grouped weight gradient of several Linears (the deferral flush): site i adds
// sum_s a[s]^T b[s] (a: dy [T][M], b: x [T][N], bf16) into dW [M][N] fp32 (+ colsum[M] += column
// sums of the dy segments when colsum != null); one workgroup per 256 x 256 tile, no token split.
// The table is filled on the host (wgrad_group_prepare: tile0, returns the tile total or -1 when a
// site does not tile) and passed in device memory.
struct WgGroupSite {
  const uint16_t* a[8];
  const uint16_t* b[8];
  float* dW;
  float* colsum;
  int nseg, M, N, ktiles, tile0, pad[3];
};
int wgrad_group_prepare(WgGroupSite* sites, int nsites);
bool launch_wgrad_group(const WgGroupSite* d_sites, int nsites, int ntiles, hipStream_t s);
// gemm256.hip persistent forward / data-gradient kernels with fused epilogues (false when
// the shape does not tile).  ncu: compute units (grid = min(tiles, ncu)).
//   nt: y[T][N] = act(x[T][K] W[N][K]^T + bias); z (nullable) = pre-activation, or act'(it)
//       when zderiv (backward act code 4 multiplies by it)
//   nn: dx[T][K] = dy[T][N] W[N][K] (* act'(aux[T][K]) when aux; act 4: * aux); colpart (nullable, needs
//       aux): per-tile column-sum partials [(T/256)*2][K] of dx (the bias gradient)
//       z8 (with zderiv): act'(z) as u8 codes in a tile-native layout ([T * N] bytes; only the
//       persistent data-gradient kernel reads it: launch_gemmp_nn act 5)
bool launch_gemmp_nt(const uint16_t* x, const uint16_t* W, const uint16_t* bias, uint16_t* y,
                     uint16_t* z, int T, int N, int K, int act, int ncu, hipStream_t s,
                     bool zderiv = false, int hm = 0, bool z8 = false);
//   nt_res: h[T][N] = res + dropout_p(x W^T + bias), pair-hash dropout bits (common.h pair_hash)
bool launch_gemmp_nt_res(const uint16_t* x, const uint16_t* W, const uint16_t* bias, const uint16_t* res,
                         uint16_t* h, int T, int N, int K, int ncu, hipStream_t s, float p, uint32_t seed,
                         uint32_t offset);
// WT (optional): W^T [K][N] bf16 - the data gradient then takes the row-form operand path
bool launch_gemmp_nn(const uint16_t* dy, const uint16_t* W, uint16_t* dx, const uint16_t* aux, int act,
                     int T, int N, int K, int ncu, hipStream_t s, float* colpart, const uint16_t* WT = nullptr);
bool launch_gemmp_nn_acc(const uint16_t* dy, const uint16_t* W, uint16_t* dx, int T, int N, int K, int ncu,
                         hipStream_t s, const uint16_t* WT = nullptr);
int device_cu_count();
// bump the device-side Philox offset base of each translation unit that draws numbers
// (common.h g_rng_base: graph replays)
void rng_base_add_attention(uint32_t d, hipStream_t s);
void rng_base_add_attention128(uint32_t d, hipStream_t s);
void rng_base_add_diffusion(uint32_t d, hipStream_t s);
void rng_base_add_norm(uint32_t d, hipStream_t s);
void rng_base_add_gemm256(uint32_t d, hipStream_t s);

}  // namespace dpa
