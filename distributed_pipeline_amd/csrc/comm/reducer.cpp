// Native bucket reducer of the DDP engine (SURVEY N-1: the role of torch's C++
// DDP Reducer, reference utils/trainer.py:115-128; SURVEY N-2: its data plane),
// designed around the flat gradient buffer instead of per-parameter copies:
//
// * Buckets are contiguous [begin, end) slices of ONE flat fp32 gradient buffer
//   (the parameters' .grad are views into it), so a bucket is reduced in place:
//   no copy-in / copy-out, no per-bucket staging.
// * mark_ready(param) is called from the parameters' post-accumulate-grad hooks
//   (autograd worker thread).  A per-bucket pending counter reaches zero when
//   the bucket's last gradient has been accumulated; ready buckets are launched
//   strictly in bucket order so every rank issues the same collective sequence
//   (one all-reduce per bucket per step, RCCL over xGMI on the GPU).
// * Optional bf16 wire format: the slice is packed into a persistent bf16 comm
//   buffer, reduced, and unpacked at finalize (fp32 master gradients keep full
//   precision locally; only the wire is narrow).
// * The 1/world average is NOT applied here: the fused AdamW kernel folds it
//   into its gradient scale.
// * ZeRO-1 mode (a shard buffer is given): each bucket is REDUCE-SCATTERED
//   instead: this rank's summed chunk of bucket b lands at shard_offsets[b] of
//   the compact shard buffer (bucket lengths are multiples of the world size).
//
// Two data planes:
// * direct (default on RCCL): the reducer owns an RCCL communicator (unique id
//   handed out by rank 0 over the c10d store) and a HIGHEST-priority HIP stream.
//   A bucket launch records an event on the producing (compute) stream at the
//   grad-ready point, the comm stream waits on it, packs (bf16 wire) and runs
//   ncclAllReduce / ncclReduceScatter; finalize() makes the compute stream wait on
//   the comm stream's completion event - nothing blocks the host, and the
//   all-reduce kernels get the CUs first when they contend with backward GEMMs.
// * process group (gloo, fake PG, or DPA_REDUCER_COMM=pg): collectives through the
//   c10d ProcessGroup the Python side created; ordering follows the backend.
// * opt-in on top of direct (DPA_IPC_ALLREDUCE=1, fp32 all-reduce buckets): peers map
//   each other's staging buffers (hipIpc handles exchanged once) and the buckets are
//   reduced by csrc/ipc_allreduce.hip on the same comm stream - all 7 xGMI links of a
//   GPU carry traffic at once instead of one ring neighbour's link.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>
#include <torch/csrc/distributed/c10d/Work.hpp>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../launchers.h"

#define DPA_RCCL_CHECK(cmd)                                                                  \
  do {                                                                                       \
    ncclResult_t r_ = (cmd);                                                                 \
    TORCH_CHECK(r_ == ncclSuccess, "RCCL error '", ncclGetErrorString(r_), "' in ", #cmd);   \
  } while (0)
#define DPA_HIP_CHECK(cmd)                                                                   \
  do {                                                                                       \
    hipError_t e_ = (cmd);                                                                   \
    TORCH_CHECK(e_ == hipSuccess, "HIP error '", hipGetErrorString(e_), "' in ", #cmd);      \
  } while (0)

namespace dpa {

// Single-device test of the IPC all-reduce protocol: the W tensors play W ranks in
// ONE launch (csrc/ipc_allreduce.hip, gridDim.y = W); every call replaces each
// tensor by the sum of all W.  mode: 0 one-shot, 1 two-shot, 2 alternate per call
// (flag slots reused across the two modes' block counts).  Returns the kernel's error
// word (0 = ok, 1 = a bounded spin timed out).
static int64_t ipc_allreduce_sim(std::vector<at::Tensor> ts, int64_t mode, int64_t calls) {
  const int W = (int)ts.size();
  TORCH_CHECK(W >= 1 && W <= IPC_MAXW, "1..8 simulated ranks");
  const int64_t n = ts[0].numel();
  for (auto& t : ts)
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == n,
                "equal-size contiguous fp32 device tensors");
  const c10::DeviceGuard guard(ts[0].device());
  auto opt = ts[0].options();
  at::Tensor stage = at::zeros({W, 2 * n}, opt);
  at::Tensor flags = at::zeros({W, IPC_FLAG_WORDS}, opt.dtype(at::kInt));
  at::Tensor err = at::zeros({1}, opt.dtype(at::kInt));
  IpcPeers peers{};
  IpcData data{};
  for (int r = 0; r < W; ++r) {
    peers.stage[r] = stage[r].data_ptr<float>();
    peers.flags[r] = reinterpret_cast<uint32_t*>(flags[r].data_ptr<int>());
    data.p[r] = ts[r].data_ptr<float>();
  }
  // all W x blocks must be co-resident (the simulated ranks spin on each other)
  TORCH_CHECK(mode >= 0 && mode <= 2, "mode: 0 one-shot, 1 two-shot, 2 alternate");
  TORCH_CHECK((int64_t)ipc_allreduce_blocks(n, W, true) * W <= 1024, "ipc_allreduce_sim: n too large");
  hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  for (int64_t c = 0; c < calls; ++c)
    TORCH_CHECK(launch_ipc_allreduce(peers, data, W, 0, W, n, n, (uint32_t)(c + 1),
                                     mode == 2 ? (c & 1) != 0 : mode == 1,
                                     err.data_ptr<int>(), s), "ipc_allreduce_sim: bad arguments");
  return err.item<int>();
}

// The reducer's issue pattern on one device: steps x buckets of different sizes through ONE
// staging buffer of 2 x cap floats per rank (cap = the largest bucket), the epoch advancing
// per bucket across steps (so the parity half alternates bucket to bucket) and one-shot /
// two-shot chosen per bucket exactly as BucketReducer::launch_direct does.  buckets[b][r] is
// rank r's slice of bucket b; each bucket is all-reduced `steps` times in bucket order.
static int64_t ipc_allreduce_sim_buckets(std::vector<std::vector<at::Tensor>> buckets, int64_t steps) {
  TORCH_CHECK(!buckets.empty() && steps >= 1, "buckets and steps");
  const int W = (int)buckets[0].size();
  TORCH_CHECK(W >= 1 && W <= IPC_MAXW, "1..8 simulated ranks");
  int64_t cap = 0;
  for (auto& b : buckets) {
    TORCH_CHECK((int)b.size() == W, "every bucket has one tensor per rank");
    for (auto& t : b)
      TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == b[0].numel(),
                  "equal-size contiguous fp32 device tensors per bucket");
    cap = std::max<int64_t>(cap, b[0].numel());
    TORCH_CHECK((int64_t)ipc_allreduce_blocks(b[0].numel(), W, true) * W <= 1024,
                "ipc_allreduce_sim_buckets: bucket too large to co-schedule its simulated ranks");
  }
  const c10::DeviceGuard guard(buckets[0][0].device());
  auto opt = buckets[0][0].options();
  at::Tensor stage = at::zeros({W, 2 * cap}, opt);
  at::Tensor flags = at::zeros({W, IPC_FLAG_WORDS}, opt.dtype(at::kInt));
  at::Tensor err = at::zeros({1}, opt.dtype(at::kInt));
  IpcPeers peers{};
  for (int r = 0; r < W; ++r) {
    peers.stage[r] = stage[r].data_ptr<float>();
    peers.flags[r] = reinterpret_cast<uint32_t*>(flags[r].data_ptr<int>());
  }
  hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
  uint32_t epoch = 0;
  for (int64_t st = 0; st < steps; ++st)
    for (auto& b : buckets) {
      IpcData data{};
      for (int r = 0; r < W; ++r) data.p[r] = b[r].data_ptr<float>();
      const int64_t n = b[0].numel();
      TORCH_CHECK(launch_ipc_allreduce(peers, data, W, 0, W, n, cap, epoch + 1, n * 4 > (256 << 10),
                                       err.data_ptr<int>(), s),
                  "ipc_allreduce_sim_buckets: bad arguments");
      ++epoch;
    }
  return err.item<int>();
}

// 128 opaque bytes for ncclCommInitRank, created by one rank and shared by all.
static pybind11::bytes rccl_unique_id() {
  ncclUniqueId id;
  DPA_RCCL_CHECK(ncclGetUniqueId(&id));
  return pybind11::bytes(id.internal, NCCL_UNIQUE_ID_BYTES);
}

class BucketReducer {
 public:
  BucketReducer(c10::intrusive_ptr<c10d::ProcessGroup> pg, at::Tensor grad_flat,
                std::vector<int64_t> bounds, std::vector<int64_t> param_bucket, bool bf16_wire,
                c10::optional<at::Tensor> shard_out, std::vector<int64_t> shard_offsets,
                std::string rccl_uid, int64_t rank, int64_t world, int64_t comm_stream = 0)
      : given_cs_(reinterpret_cast<hipStream_t>(comm_stream)), pg_(std::move(pg)), grad_(std::move(grad_flat)), bounds_(std::move(bounds)),
        bucket_of_(std::move(param_bucket)), bf16_(bf16_wire) {
    TORCH_CHECK(grad_.is_contiguous() && grad_.dim() == 1, "grad_flat must be a 1-D contiguous tensor");
    TORCH_CHECK(bounds_.size() >= 2 && bounds_.front() == 0 && bounds_.back() <= grad_.numel(),
                "bucket bounds must start at 0 and stay inside the flat buffer");
    const int nb = (int)bounds_.size() - 1;
    size_.assign(nb, 0);
    for (int64_t b : bucket_of_) {
      TORCH_CHECK(b >= 0 && b < nb, "param bucket index out of range");
      size_[b] += 1;
    }
    for (int b = 0; b < nb; ++b) TORCH_CHECK(size_[b] > 0, "empty bucket ", b);
    pending_ = size_;
    work_.resize(nb);
    launched_.assign(nb, false);
    world_ = pg_ ? pg_->getSize() : world;
    if (bf16_) comm_ = at::empty({grad_.numel()}, grad_.options().dtype(at::kBFloat16));
    if (shard_out.has_value() && shard_out->defined()) {
      rs_ = true;
      shard_ = *shard_out;
      shard_off_ = std::move(shard_offsets);
      TORCH_CHECK(shard_.is_contiguous() && shard_.scalar_type() == grad_.scalar_type(),
                  "shard buffer must be contiguous and of the gradient dtype");
      TORCH_CHECK((int)shard_off_.size() == nb, "one shard offset per bucket");
      for (int b = 0; b < nb; ++b) {
        const int64_t n = bounds_[b + 1] - bounds_[b];
        TORCH_CHECK(n % world_ == 0, "bucket ", b, " is not divisible by the world size");
        TORCH_CHECK(shard_off_[b] >= 0 && shard_off_[b] + n / world_ <= shard_.numel(),
                    "shard offset out of range");
      }
      if (bf16_) comm_out_ = at::empty({shard_.numel()}, grad_.options().dtype(at::kBFloat16));
    }
    if (!rccl_uid.empty()) init_direct(rccl_uid, (int)rank, (int)world);
  }

  ~BucketReducer() {
    // abort (not destroy): never blocks on peers that already left at shutdown
    if (rcomm_) ncclCommAbort(rcomm_);
    for (int r = 0; r < world_; ++r)
      if (r != rank_ && peers_.stage[r]) {
        (void)hipIpcCloseMemHandle(peers_.stage[r]);
        (void)hipIpcCloseMemHandle(peers_.flags[r]);
      }
    if (ipc_stage_) (void)hipFree(ipc_stage_);
    if (ipc_flags_) (void)hipFree(ipc_flags_);
    for (hipEvent_t e : ready_) if (e) (void)hipEventDestroy(e);
    if (done_) (void)hipEventDestroy(done_);
    if (gather_ev_) (void)hipEventDestroy(gather_ev_);
    if (cs_ && own_cs_) (void)hipStreamDestroy(cs_);
  }

  // Called at forward time when gradient synchronisation is enabled (torch-DDP
  // semantics: the no_sync decision is taken when the graph is built).
  //
  // ``stream``: the stream the armed backward produces its gradients on (0: the calling
  // thread's current stream NOW - which may be the null stream, handle 0 too).  The grad-ready
  // hooks do NOT run on it reliably: autograd runs a leaf's AccumulateGrad - and its hook - on
  // the stream of the forward that first used the leaf, which in the overlapped micro-batch
  // schedule is often the other stream; an event recorded there would not follow the gradient
  // kernels.  (Deferring the choice to launch time, as before round 6, took the HOOK thread's
  // stream whenever the trainer ran on the null stream, whose handle is 0.)
  void arm(int64_t stream = 0) {
    std::lock_guard<std::mutex> g(mu_);
    if (grad_.is_cuda())
      arm_c10_ = stream ? c10::hip::getStreamFromExternalMasqueradingAsCUDA(reinterpret_cast<hipStream_t>(stream),
                                                                             grad_.device().index())
                        : c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(grad_.device().index());
    arm_stream_ = arm_c10_ ? arm_c10_->stream() : nullptr;
    pending_ = size_;
    std::fill(launched_.begin(), launched_.end(), false);
    for (auto& w : work_) w.reset();
    next_ = 0;
    armed_ = true;
    if (sim_)  // fresh timeline: every word all-ones (the kernels keep minima)
      DPA_HIP_CHECK(hipMemsetAsync(sim_tl_.data_ptr(), 0xff, sim_tl_.nbytes(), producer()));
  }

  // Abandon a partially run backward (out-of-memory retry).  Buckets its hooks already
  // launched keep running on the comm stream and write the flat gradient in place, so
  // the compute stream (the retry's zero_grad and backward) is ordered after them.
  void disarm() {
    std::lock_guard<std::mutex> g(mu_);
    if (armed_ && cs_ && next_ > 0) {
      DPA_HIP_CHECK(hipEventRecord(done_, cs_));
      DPA_HIP_CHECK(hipStreamWaitEvent(compute_stream(), done_, 0));
    }
    armed_ = false;
  }
  // Buckets launches the hooks had already made since the last arm().
  int64_t launched_count() const { return next_; }

  bool armed() const { return armed_; }
  bool direct() const { return rcomm_ != nullptr; }

  void mark_ready(int64_t param_index) {
    std::lock_guard<std::mutex> g(mu_);
    if (!armed_) return;
    TORCH_CHECK(param_index >= 0 && param_index < (int64_t)bucket_of_.size(), "bad param index");
    const int b = (int)bucket_of_[param_index];
    TORCH_CHECK(pending_[b] > 0, "parameter ", param_index, " marked ready twice in one backward");
    if (--pending_[b] == 0) launch_ready_in_order();
  }

  // Launch whatever has not been launched (e.g. unused parameters, or graph
  // replays without hooks), then order the reduced gradients before the current
  // stream's next work (direct: a stream-side event wait, no host block; process
  // group: wait on the Work handles), unpacking the bf16 wire.
  void finalize() {
    std::lock_guard<std::mutex> g(mu_);
    if (!armed_) return;
    const int nb = (int)launched_.size();
    // a bucket still waiting for gradients here had a parameter whose hook never fired
    // (unused in this step's graph): it is reduced now, after backward, without overlap
    late_.clear();
    for (int b = next_; b < nb; ++b) {
      if (pending_[b] > 0) late_.push_back(b);
      launch(b);
    }
    next_ = nb;
    if (cs_) {
      if (bf16_) {
        for (int b = 0; b < nb; ++b) {
          if (rs_) {
            const int64_t c = (bounds_[b + 1] - bounds_[b]) / world_;
            launch_cast_f32(bf_ptr(comm_out_) + shard_off_[b], shard_.data_ptr<float>() + shard_off_[b], c, cs_);
          } else {
            launch_cast_f32(bf_ptr(comm_) + bounds_[b], grad_.data_ptr<float>() + bounds_[b],
                            bounds_[b + 1] - bounds_[b], cs_);
          }
        }
      }
      if (sim_) launch_time_marker(sim_end_slot(), compute_stream());  // the backward's end
      DPA_HIP_CHECK(hipEventRecord(done_, cs_));
      DPA_HIP_CHECK(hipStreamWaitEvent(compute_stream(), done_, 0));
      if (sim_)
        launch_comm_sim_stats(sim_slot(0, 0), (int)launched_.size(), sim_end_slot(),
                              reinterpret_cast<unsigned long long*>(sim_acc_.data_ptr()), compute_stream());
    } else {
      for (int b = 0; b < nb; ++b) {
        if (work_[b]) {
          work_[b]->wait();
          work_[b].reset();
          if (bf16_) {
            if (rs_) chunk(shard_, b).copy_(chunk(comm_out_, b));
            else slice(grad_, b).copy_(slice(comm_, b));
          }
        }
      }
    }
    armed_ = false;
  }

  // Reduce every bucket now (graph mode: backward ran without hooks).
  void reduce_all() {
    arm(0);
    finalize();
  }

  // ---- the data plane's own collectives beyond the bucket reductions (direct mode) ----
  // Start-up bucket tuning on THIS communicator and comm stream (not the process group's, whose
  // pool stream lands on a compute-shared queue): mean ms of `iters` all-reduces of n floats.
  double time_allreduce(int64_t n, int64_t iters) {
    TORCH_CHECK(rcomm_ != nullptr && n > 0 && iters > 0, "time_allreduce: direct mode only");
    const c10::DeviceGuard guard(grad_.device());
    at::Tensor x = at::zeros({n}, grad_.options());
    hipEvent_t e0, e1;
    DPA_HIP_CHECK(hipEventCreate(&e0));
    DPA_HIP_CHECK(hipEventCreate(&e1));
    DPA_RCCL_CHECK(ncclAllReduce(x.data_ptr(), x.data_ptr(), (size_t)n, ncclFloat32, ncclSum, rcomm_, cs_));  // warm
    DPA_HIP_CHECK(hipEventRecord(e0, cs_));
    for (int64_t i = 0; i < iters; ++i)
      DPA_RCCL_CHECK(ncclAllReduce(x.data_ptr(), x.data_ptr(), (size_t)n, ncclFloat32, ncclSum, rcomm_, cs_));
    DPA_HIP_CHECK(hipEventRecord(e1, cs_));
    DPA_HIP_CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    DPA_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    last_coll_stream_ = cs_;
    return (double)ms / (double)iters;
  }

  // Re-plan the buckets (not while armed): the engine's measured plan replaces the provisional one
  // the communicator was created with.  All-reduce mode only (ZeRO-1's layout pads bucket ends).
  void set_buckets(std::vector<int64_t> bounds, std::vector<int64_t> param_bucket) {
    std::lock_guard<std::mutex> g(mu_);
    TORCH_CHECK(!armed_ && !rs_, "set_buckets: all-reduce mode, not armed");
    TORCH_CHECK(bounds.size() >= 2 && bounds.front() == 0 && bounds.back() <= grad_.numel() &&
                    param_bucket.size() == bucket_of_.size(), "set_buckets: bad plan");
    const int nb = (int)bounds.size() - 1;
    std::vector<int> size(nb, 0);
    for (int64_t b : param_bucket) {
      TORCH_CHECK(b >= 0 && b < nb, "param bucket index out of range");
      size[b] += 1;
    }
    for (int b = 0; b < nb; ++b) TORCH_CHECK(size[b] > 0, "empty bucket ", b);
    bounds_ = std::move(bounds);
    bucket_of_ = std::move(param_bucket);
    size_ = size;
    pending_ = size_;
    work_.assign(nb, {});
    launched_.assign(nb, false);
    for (hipEvent_t e : ready_) if (e) (void)hipEventDestroy(e);
    ready_.assign(nb, nullptr);
    if (cs_)
      for (auto& e : ready_) DPA_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }

  // ZeRO-1 parameter all-gather on the data plane's communicator and comm stream: for each bucket
  // in `order`, flat[bounds[b], bounds[b + 1]) is gathered in place from every rank's chunk
  // (chunk r of the bucket is rank r's).  flat: fp32 master or bf16 shadow, laid out like the
  // gradients.  Ordered after the current stream's work (an event); wait_gather() orders the
  // current stream after it.  Nothing blocks the host.
  void all_gather_buckets(at::Tensor flat, std::vector<int64_t> order) {
    TORCH_CHECK(rcomm_ != nullptr, "all_gather_buckets: direct mode only");
    TORCH_CHECK(flat.is_contiguous() && flat.dim() == 1 && flat.numel() >= bounds_.back() &&
                    (flat.scalar_type() == at::kFloat || flat.scalar_type() == at::kBFloat16),
                "all_gather_buckets: 1-D fp32 / bf16 flat buffer laid out like the gradients");
    const c10::DeviceGuard guard(grad_.device());
    const ncclDataType_t dt = flat.scalar_type() == at::kFloat ? ncclFloat32 : ncclBfloat16;
    const int64_t es = flat.element_size();
    char* base = static_cast<char*>(flat.data_ptr());
    if (!gather_ev_) DPA_HIP_CHECK(hipEventCreateWithFlags(&gather_ev_, hipEventDisableTiming));
    DPA_HIP_CHECK(hipEventRecord(gather_ev_, compute_stream()));
    DPA_HIP_CHECK(hipStreamWaitEvent(cs_, gather_ev_, 0));
    for (int64_t b : order) {
      TORCH_CHECK(b >= 0 && b + 1 < (int64_t)bounds_.size(), "bucket out of range");
      const int64_t n = bounds_[b + 1] - bounds_[b];
      TORCH_CHECK(n % world_ == 0, "bucket ", b, " is not divisible by the world size");
      const int64_t c = n / world_;
      char* whole = base + bounds_[b] * es;
      DPA_RCCL_CHECK(ncclAllGather(whole + (int64_t)rank_ * c * es, whole, (size_t)c, dt, rcomm_, cs_));
    }
    DPA_HIP_CHECK(hipEventRecord(gather_ev_, cs_));
    gather_pending_ = true;
    last_coll_stream_ = cs_;
  }
  void wait_gather() {
    if (!gather_pending_) return;
    DPA_HIP_CHECK(hipStreamWaitEvent(compute_stream(), gather_ev_, 0));
    gather_pending_ = false;
  }
  // stream of the last tuning / gather collective (tests: it is the comm stream)
  int64_t last_collective_stream() const { return (int64_t)reinterpret_cast<uintptr_t>(last_coll_stream_); }

  // ranks of the reducer-owned RCCL communicator (ncclCommCount), -1 without one
  int64_t comm_size() const {
    if (!rcomm_) return -1;
    int n = 0;
    DPA_RCCL_CHECK(ncclCommCount(rcomm_, &n));
    return n;
  }

  int64_t num_buckets() const { return (int64_t)launched_.size(); }
  int64_t next_bucket() const { return next_; }
  std::vector<int64_t> pending() const {
    return std::vector<int64_t>(pending_.begin(), pending_.end());
  }
  // buckets the last finalize() had to launch with parameters still pending
  std::vector<int64_t> late_buckets() const { return std::vector<int64_t>(late_.begin(), late_.end()); }
  // ---- opt-in direct xGMI all-reduce over IPC-mapped buffers (DPA_IPC_ALLREDUCE=1) ----
  // Phase 1: allocate this rank's staging buffer (two parity halves of the largest
  // bucket) and flag words with hipMalloc and export their IPC handles.
  pybind11::bytes ipc_export() {
    TORCH_CHECK(cs_ != nullptr, "the IPC data plane rides on the direct mode's comm stream (or init_ipc_only)");
    TORCH_CHECK(!rs_ && !bf16_, "IPC all-reduce: fp32 all-reduce buckets only");
    const c10::DeviceGuard guard(grad_.device());
    ipc_cap_ = 0;
    for (size_t b = 0; b + 1 < bounds_.size(); ++b) ipc_cap_ = std::max(ipc_cap_, bounds_[b + 1] - bounds_[b]);
    DPA_HIP_CHECK(hipMalloc(&ipc_stage_, 2 * ipc_cap_ * sizeof(float)));
    DPA_HIP_CHECK(hipMalloc(&ipc_flags_, IPC_FLAG_WORDS * sizeof(uint32_t)));
    DPA_HIP_CHECK(hipMemset(ipc_flags_, 0, IPC_FLAG_WORDS * sizeof(uint32_t)));
    ipc_err_t_ = at::zeros({1}, grad_.options().dtype(at::kInt));
    ipc_err_ = ipc_err_t_.data_ptr<int>();
    DPA_HIP_CHECK(hipDeviceSynchronize());
    hipIpcMemHandle_t h[2];
    DPA_HIP_CHECK(hipIpcGetMemHandle(&h[0], ipc_stage_));
    DPA_HIP_CHECK(hipIpcGetMemHandle(&h[1], ipc_flags_));
    return pybind11::bytes(reinterpret_cast<const char*>(h), sizeof(h));
  }

  // Phase 2: map every peer's buffers (handles gathered from all ranks, rank order).
  void ipc_open(std::vector<std::string> handles) {
    TORCH_CHECK((int)handles.size() == world_ && world_ <= IPC_MAXW, "one handle blob per rank, <= 8 ranks");
    const c10::DeviceGuard guard(grad_.device());
    for (int r = 0; r < world_; ++r) {
      if (r == rank_) {
        peers_.stage[r] = ipc_stage_;
        peers_.flags[r] = ipc_flags_;
        continue;
      }
      TORCH_CHECK(handles[r].size() == 2 * sizeof(hipIpcMemHandle_t), "bad IPC handle blob");
      hipIpcMemHandle_t h[2];
      std::memcpy(h, handles[r].data(), sizeof(h));
      void *st = nullptr, *fl = nullptr;
      DPA_HIP_CHECK(hipIpcOpenMemHandle(&st, h[0], hipIpcMemLazyEnablePeerAccess));
      DPA_HIP_CHECK(hipIpcOpenMemHandle(&fl, h[1], hipIpcMemLazyEnablePeerAccess));
      peers_.stage[r] = static_cast<float*>(st);
      peers_.flags[r] = static_cast<uint32_t*>(fl);
    }
    ipc_ready_ = true;
  }

  bool ipc_ready() const { return ipc_ready_; }
  // The kernels' error word as a device int32 [1] tensor (undefined without IPC): the
  // fused AdamW skips its update while it is non-zero, and the engine reads it back
  // asynchronously to raise (parallel/ddp.py).
  at::Tensor ipc_error_flag() const { return ipc_err_t_; }
  // the kernels' timeout word (host sync; debugging / tests only)
  int64_t ipc_error() const {
    if (!ipc_err_) return 0;
    int e = 0;
    DPA_HIP_CHECK(hipStreamSynchronize(cs_));
    DPA_HIP_CHECK(hipMemcpy(&e, ipc_err_, sizeof(int), hipMemcpyDeviceToHost));
    return e;
  }

  // priority of the reducer's comm stream (direct mode; lower = higher priority)
  // handle of the data plane's comm stream (0: none - not the direct mode)
  int64_t comm_stream() const { return (int64_t)reinterpret_cast<uintptr_t>(cs_); }

  int64_t stream_priority() const {
    int p = 0;
    if (cs_) (void)hipStreamGetPriority(cs_, &p);
    return p;
  }

 private:
  static hipStream_t compute_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }
  // the armed backward's stream (captured by arm(); the null stream included), else the current
  hipStream_t producer() const { return arm_c10_ ? arm_stream_ : compute_stream(); }
  static uint16_t* bf_ptr(const at::Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

  // The IPC data plane without an RCCL communicator: the comm stream and events of the direct
  // mode, every bucket through csrc/ipc_allreduce.hip (tests: two processes on one device over
  // gloo, where RCCL refuses two ranks per GPU - tests/test_ipc_reducer_gpu.py).
 public:
  void init_ipc_only(int64_t rank) {
    TORCH_CHECK(cs_ == nullptr, "the reducer already has a comm stream");
    TORCH_CHECK(grad_.is_cuda() && !rs_ && !bf16_, "IPC-only: fp32 all-reduce buckets of device gradients");
    TORCH_CHECK(world_ > 1 && world_ <= IPC_MAXW && rank >= 0 && rank < world_, "IPC-only: 2..8 ranks");
    const c10::DeviceGuard guard(grad_.device());
    rank_ = (int)rank;
    make_comm_stream(given_cs_);
  }

  // Simulated data plane (csrc/comm_sim.hip): a one-GPU PROJECTION of a world-`world` all-reduce.
  // Every bucket launches comm_sim_kernel on the comm stream instead of a collective: `cus`
  // workgroups that hold their CU slots for lat_us + 2 (W - 1) / W x bytes / busbw and move the
  // ring's local HBM bytes; the gradients stay this rank's (world-1 math).  Per-step timeline
  // sums accumulate on the device (sim_stats).
  // comm_stream: 0 = a new highest-priority stream (as the direct mode), else the handle of an
  // existing stream to run the stand-in kernels on (A/B of the stream's hardware queue)
  void init_sim(int64_t world, double busbw_gbps, int64_t cus, double lat_us, int64_t comm_stream) {
    TORCH_CHECK(cs_ == nullptr, "the reducer already has a comm stream");
    TORCH_CHECK(grad_.is_cuda() && !rs_, "sim data plane: all-reduce buckets of device gradients");
    const c10::DeviceGuard guard(grad_.device());
    sim_ = true;
    set_sim(world, busbw_gbps, cus, lat_us);
    const int nb = (int)launched_.size();
    sim_tl_ = at::empty({(int64_t)nb * 4 + 8}, grad_.options().dtype(at::kLong));
    DPA_HIP_CHECK(hipMemset(sim_tl_.data_ptr(), 0xff, sim_tl_.nbytes()));
    sim_acc_ = at::zeros({8}, grad_.options().dtype(at::kLong));
    make_comm_stream(reinterpret_cast<hipStream_t>(comm_stream));
  }
  void set_sim(int64_t world, double busbw_gbps, int64_t cus, double lat_us) {
    TORCH_CHECK(world >= 2 && busbw_gbps > 0 && cus >= 1 && cus <= 1024 && lat_us >= 0, "sim: bad parameters");
    sim_world_ = (int)world;
    sim_bw_ = busbw_gbps;
    sim_cus_ = (int)cus;
    sim_lat_ = lat_us;
  }
  bool sim() const { return sim_; }
  // {steps, exposed tail, ready->start delay, bucket busy time, comm span, last tail} in ms
  // (sums over the steps since the last reset; the device accumulates in 10 ns ticks)
  std::vector<double> sim_stats() {
    TORCH_CHECK(sim_, "not in sim mode");
    at::Tensor a = sim_acc_.cpu();
    const int64_t* v = a.data_ptr<int64_t>();
    std::vector<double> out{(double)v[0]};
    for (int i = 1; i < 6; ++i) out.push_back((double)v[i] * 1e-5);
    return out;
  }
  // the last step's per-bucket timeline [nb][3] = {grad ready, first start, last end} in ms after
  // the first grad-ready stamp, plus the backward's end as a last row (-1: not stamped)
  at::Tensor sim_timeline() {
    TORCH_CHECK(sim_, "not in sim mode");
    DPA_HIP_CHECK(hipStreamSynchronize(cs_));
    at::Tensor t = sim_tl_.cpu();
    const uint64_t* v = reinterpret_cast<const uint64_t*>(t.data_ptr<int64_t>());
    const int nb = (int)launched_.size();
    uint64_t t0 = ~0ull;
    for (int b = 0; b < nb; ++b) t0 = std::min(t0, v[b * 4 + 2]);
    at::Tensor out = at::full({nb + 1, 3}, -1.0, at::kDouble);
    double* o = out.data_ptr<double>();
    auto ms = [&](uint64_t x) { return (x == ~0ull || t0 == ~0ull) ? -1.0 : (double)(x - t0) * 1e-5; };
    for (int b = 0; b < nb; ++b) {
      o[b * 3] = ms(v[b * 4 + 2]);
      o[b * 3 + 1] = ms(v[b * 4]);
      o[b * 3 + 2] = v[b * 4 + 1] == ~0ull ? -1.0 : ms(~v[b * 4 + 1]);
    }
    o[nb * 3] = ms(v[(int64_t)nb * 4]);  // backward end
    return out;
  }
  void sim_reset() {
    TORCH_CHECK(sim_, "not in sim mode");
    sim_acc_.zero_();
  }
  // simulated duration of a bucket of `bytes` on the wire (ms)
  double sim_bucket_ms(int64_t bytes) const {
    return sim_lat_ * 1e-3 + 2.0 * (sim_world_ - 1) / sim_world_ * (double)bytes / (sim_bw_ * 1e9) * 1e3;
  }

 private:
  // words of bucket b: {0: first start, 1: ~last end, 2: grad ready, 3: unused}; after the
  // nb buckets: the backward's end
  unsigned long long* sim_slot(int b, int k) {
    return reinterpret_cast<unsigned long long*>(sim_tl_.data_ptr()) + (int64_t)b * 4 + k;
  }
  unsigned long long* sim_end_slot() { return sim_slot((int)launched_.size(), 0); }

  void launch_sim(int b, void* buf, int64_t bytes) {
    // grad-ready stamp on the producing stream (index 2 of the bucket's words), then the
    // collective's stand-in on the comm stream (words 0 / 1)
    const double ms = sim_bucket_ms(bytes);
    const uint64_t ticks = (uint64_t)(ms * 1e5);  // 100 MHz constant clock
    const int64_t touch = (int64_t)(2.0 * (sim_world_ - 1) / sim_world_ * (double)bytes);
    launch_comm_sim(buf, bytes, touch, ticks, sim_cus_, sim_slot(b, 0), cs_);
  }

  // The data plane's stream.  `given` (the stream plan's, runtime/streams.py): a stream on one of
  // the process's GPU_MAX_HW_QUEUES pooled queues.  Otherwise a new highest-priority stream - which
  // gets an HSA queue of its own, one more than the pooled four: with it present the overlapped
  // reference schedule ran 228.9 ms/step against 209.2 on a pooled normal-priority stream and 208.9
  // without any data plane (simulated comm, profiles/sim_comm_r6.json), so the engine passes the plan's.
  void make_comm_stream(hipStream_t given = nullptr) {
    if (given) {
      cs_ = given;
      own_cs_ = false;
    } else {
      int least = 0, greatest = 0;
      DPA_HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
      DPA_HIP_CHECK(hipStreamCreateWithPriority(&cs_, hipStreamNonBlocking, greatest));
    }
    ready_.assign(launched_.size(), nullptr);
    for (auto& e : ready_) DPA_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    DPA_HIP_CHECK(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
  }

  void init_direct(const std::string& uid, int rank, int world) {
    TORCH_CHECK(grad_.is_cuda(), "the direct RCCL data plane needs device gradients");
    TORCH_CHECK(uid.size() == NCCL_UNIQUE_ID_BYTES, "RCCL unique id must be ", NCCL_UNIQUE_ID_BYTES, " bytes");
    TORCH_CHECK(world == world_, "direct communicator size differs from the process group's");
    const c10::DeviceGuard guard(grad_.device());
    ncclUniqueId id;
    std::memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
    rank_ = rank;
    DPA_RCCL_CHECK(ncclCommInitRank(&rcomm_, world, id, rank));
    make_comm_stream(given_cs_);
  }

  at::Tensor slice(const at::Tensor& t, int b) const { return t.slice(0, bounds_[b], bounds_[b + 1]); }
  // this rank's reduce-scatter output for bucket b inside a compact shard buffer
  at::Tensor chunk(const at::Tensor& t, int b) const {
    return t.narrow(0, shard_off_[b], (bounds_[b + 1] - bounds_[b]) / world_);
  }

  void launch_ready_in_order() {
    const int nb = (int)launched_.size();
    while (next_ < nb && pending_[next_] == 0) launch(next_++);
  }

  void launch(int b) {
    if (launched_[b]) return;
    if (cs_) launch_direct(b);
    else launch_pg(b);
    launched_[b] = true;
  }

  void launch_direct(int b) {
    const int64_t n = bounds_[b + 1] - bounds_[b];
    // the grad-ready point: everything the backward's stream queued so far
    if (sim_) launch_time_marker(sim_slot(b, 2), producer());
    DPA_HIP_CHECK(hipEventRecord(ready_[b], producer()));
    DPA_HIP_CHECK(hipStreamWaitEvent(cs_, ready_[b], 0));
    float* g = grad_.data_ptr<float>() + bounds_[b];
    void* buf = g;
    ncclDataType_t dt = ncclFloat32;
    if (bf16_) {
      uint16_t* w = bf_ptr(comm_) + bounds_[b];
      launch_cast_bf16(g, w, n, cs_);
      buf = w;
      dt = ncclBfloat16;
    }
    if (sim_) {
      launch_sim(b, buf, n * (bf16_ ? 2 : 4));
      return;
    }
    if (ipc_ready_) {
      // one-shot below 256 KiB (latency), two-shot above (bandwidth: (W-1)/W n reads twice)
      IpcData d{};
      d.p[rank_] = g;
      // (a bucket the kernel cannot take - length % 4, 16-byte alignment - goes through
      // RCCL instead; the layout is identical on every rank, so all ranks agree)
      if (launch_ipc_allreduce(peers_, d, (int)world_, rank_, 1, n, ipc_cap_, ipc_epoch_ + 1,
                               n * 4 > (256 << 10), ipc_err_, cs_)) {
        ++ipc_epoch_;
        return;
      }
    }
    TORCH_CHECK(rcomm_ != nullptr, "IPC-only data plane: bucket ", b, " (", n,
                " floats) cannot take the IPC kernel and there is no RCCL communicator");
    if (rs_) {
      void* out = bf16_ ? (void*)(bf_ptr(comm_out_) + shard_off_[b]) : (void*)(shard_.data_ptr<float>() + shard_off_[b]);
      DPA_RCCL_CHECK(ncclReduceScatter(buf, out, (size_t)(n / world_), dt, ncclSum, rcomm_, cs_));
    } else {
      DPA_RCCL_CHECK(ncclAllReduce(buf, buf, (size_t)n, dt, ncclSum, rcomm_, cs_));
    }
  }

  void launch_pg(int b) {
    // the process group orders its collective (and the bf16 wire copy below) after the
    // CURRENT stream: make that the armed backward's stream, not whichever stream autograd
    // runs this parameter's hook on (in the overlapped schedule often the other one)
    c10::optional<c10::hip::HIPStreamGuardMasqueradingAsCUDA> guard;
    if (arm_c10_ && grad_.is_cuda()) guard.emplace(*arm_c10_);
    at::Tensor view = slice(grad_, b);
    if (bf16_) {
      at::Tensor wire = slice(comm_, b);
      wire.copy_(view);
      view = wire;
    }
    if (rs_) {
      at::Tensor out = chunk(bf16_ ? comm_out_ : shard_, b);
      work_[b] = pg_->_reduce_scatter_base(out, view);
    } else {
      std::vector<at::Tensor> ts{view};
      work_[b] = pg_->allreduce(ts);
    }
  }

  c10::intrusive_ptr<c10d::ProcessGroup> pg_;
  at::Tensor grad_, comm_, shard_, comm_out_;
  std::vector<int64_t> shard_off_;
  int64_t world_ = 1;
  bool rs_ = false;
  std::vector<int64_t> bounds_;
  std::vector<int64_t> bucket_of_;
  std::vector<int> size_, pending_;
  std::vector<c10::intrusive_ptr<c10d::Work>> work_;
  std::vector<bool> launched_;
  std::vector<int> late_;
  int next_ = 0;
  bool armed_ = false;
  bool bf16_;
  // direct data plane
  ncclComm_t rcomm_ = nullptr;
  int rank_ = 0;
  // IPC data plane
  bool ipc_ready_ = false;
  float* ipc_stage_ = nullptr;
  uint32_t* ipc_flags_ = nullptr;
  int* ipc_err_ = nullptr;
  at::Tensor ipc_err_t_;
  int64_t ipc_cap_ = 0;
  uint32_t ipc_epoch_ = 0;
  IpcPeers peers_{};
  hipEvent_t gather_ev_ = nullptr;
  bool gather_pending_ = false;
  hipStream_t last_coll_stream_ = nullptr;
  // simulated data plane
  bool sim_ = false;
  int sim_world_ = 2, sim_cus_ = 1;
  double sim_bw_ = 1.0, sim_lat_ = 0.0;
  at::Tensor sim_tl_, sim_acc_;
  hipStream_t given_cs_ = nullptr;  // the constructor's comm_stream (0: create one)
  hipStream_t cs_ = nullptr;
  bool own_cs_ = true;
  hipStream_t arm_stream_ = nullptr;  // the armed backward's stream (arm()); may be the null stream
  c10::optional<c10::hip::HIPStreamMasqueradingAsCUDA> arm_c10_;
  std::vector<hipEvent_t> ready_;
  hipEvent_t done_ = nullptr;
  std::mutex mu_;
};

void register_comm(pybind11::module& m) {
  m.def("rccl_unique_id", &rccl_unique_id, "new RCCL unique id (bytes) for the reducer's communicator");
  m.def("ipc_allreduce_sim", &ipc_allreduce_sim,
        "single-device test of the IPC all-reduce: the W tensors play W ranks -> error word");
  m.def("ipc_allreduce_sim_buckets", &ipc_allreduce_sim_buckets,
        "single-device test of the reducer's IPC issue pattern: buckets[b][rank], steps -> error word");
  pybind11::class_<BucketReducer>(m, "BucketReducer")
      .def(pybind11::init<c10::intrusive_ptr<c10d::ProcessGroup>, at::Tensor, std::vector<int64_t>,
                          std::vector<int64_t>, bool, c10::optional<at::Tensor>, std::vector<int64_t>,
                          std::string, int64_t, int64_t, int64_t>(),
           pybind11::arg("process_group"), pybind11::arg("grad_flat"), pybind11::arg("bounds"),
           pybind11::arg("param_bucket"), pybind11::arg("bf16_wire") = false,
           pybind11::arg("shard_out") = pybind11::none(),
           pybind11::arg("shard_offsets") = std::vector<int64_t>(),
           pybind11::arg("rccl_uid") = std::string(), pybind11::arg("rank") = 0, pybind11::arg("world") = 1,
           pybind11::arg("comm_stream") = 0)
      .def("arm", &BucketReducer::arm, pybind11::arg("stream") = 0)
      // disarm / mark_ready / finalize keep the GIL: they only enqueue work (microseconds), and a
      // release hands the GIL to another Python thread (the device prefetch thread) for up to its
      // 5 ms switch interval - 32 no_sync forwards per step of the reference 32 x 64 schedule each
      // called disarm and ran 55 ms/step slower (profiles/sim_comm_r6.json)
      .def("disarm", &BucketReducer::disarm)
      .def("armed", &BucketReducer::armed)
      .def("direct", &BucketReducer::direct)
      .def("stream_priority", &BucketReducer::stream_priority)
      .def("comm_stream", &BucketReducer::comm_stream)
      .def("init_ipc_only", &BucketReducer::init_ipc_only, pybind11::arg("rank"))
      .def_static("simulated",
                  [](at::Tensor grad_flat, std::vector<int64_t> bounds, std::vector<int64_t> param_bucket,
                     bool bf16_wire) {
                    return std::make_unique<BucketReducer>(c10::intrusive_ptr<c10d::ProcessGroup>(), grad_flat,
                                                           bounds, param_bucket, bf16_wire, c10::nullopt,
                                                           std::vector<int64_t>(), std::string(), 0, 1);
                  },
                  "a reducer without a process group, for the simulated data plane (then init_sim)")
      .def("init_sim", &BucketReducer::init_sim, pybind11::arg("world"), pybind11::arg("busbw_gbps"),
           pybind11::arg("cus"), pybind11::arg("lat_us"), pybind11::arg("comm_stream") = 0)
      .def("set_sim", &BucketReducer::set_sim, pybind11::arg("world"), pybind11::arg("busbw_gbps"),
           pybind11::arg("cus"), pybind11::arg("lat_us"))
      .def("sim", &BucketReducer::sim)
      .def("sim_stats", &BucketReducer::sim_stats)
      .def("sim_reset", &BucketReducer::sim_reset)
      .def("sim_timeline", &BucketReducer::sim_timeline)
      .def("time_allreduce", &BucketReducer::time_allreduce, pybind11::arg("n"), pybind11::arg("iters"),
           pybind11::call_guard<pybind11::gil_scoped_release>())
      .def("set_buckets", &BucketReducer::set_buckets)
      .def("all_gather_buckets", &BucketReducer::all_gather_buckets)
      .def("wait_gather", &BucketReducer::wait_gather)
      .def("last_collective_stream", &BucketReducer::last_collective_stream)
      .def("sim_bucket_ms", &BucketReducer::sim_bucket_ms)
      .def("ipc_export", &BucketReducer::ipc_export)
      .def("ipc_open", &BucketReducer::ipc_open)
      .def("ipc_ready", &BucketReducer::ipc_ready)
      .def("ipc_error", &BucketReducer::ipc_error)
      .def("ipc_error_flag", &BucketReducer::ipc_error_flag)
      .def("launched_count", &BucketReducer::launched_count)
      .def("late_buckets", &BucketReducer::late_buckets)
      .def("mark_ready", &BucketReducer::mark_ready)
      .def("finalize", &BucketReducer::finalize)
      .def("reduce_all", &BucketReducer::reduce_all, pybind11::call_guard<pybind11::gil_scoped_release>())
      .def("num_buckets", &BucketReducer::num_buckets)
      .def("comm_size", &BucketReducer::comm_size)
      .def("next_bucket", &BucketReducer::next_bucket)
      .def("pending", &BucketReducer::pending);
}

}  // namespace dpa
