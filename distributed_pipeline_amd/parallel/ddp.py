"""
Native data-parallel engine (SURVEY N-1/P-DP/P-GA): the MI355X replacement for
``torch.nn.parallel.DistributedDataParallel`` as used by the reference trainer
(reference: utils/trainer.py:115-128, 209-221).

Design (xGMI/RCCL-first rather than a translation of torch's C++ Reducer).  The
bucket bookkeeping and collective launches run in the native ``BucketReducer``
(``csrc/comm/reducer.cpp``) when the extension is present; the Python code here
implements the same protocol for the single-GPU multi-rank test transport.

* Gradients live in ONE flat fp32 buffer (:class:`FlatParamSpace`); buckets are
  contiguous slices of it, so a bucket all-reduce reads/writes the gradients
  in place - no copy-in/copy-out kernels.
* Bucket sizes are chosen for point-to-point xGMI rings, not NVSwitch: a small
  first bucket (default 4 MiB) so RCCL starts while backward is still deep in
  the network, then ~32 MiB buckets - large enough to saturate a ring's links,
  small enough to overlap.  (reference: ``bucket_cap_mb=128``.)  ``bucket_cap_mb <= 0``
  measures them instead (:func:`tune_bucket_sizes`: an all-reduce bandwidth sweep on the
  job's own process group at startup, the same decision on every rank).
* Readiness: a post-accumulate-grad hook per parameter decrements its bucket's
  pending counter (autograd runs it once per backward per leaf, after all uses,
  even when a fused wgrad GEMM accumulated the gradient in place and returned
  None); the bucket whose counter hits zero is all-reduced asynchronously.  On
  RCCL the C++ reducer owns its communicator and a highest-priority HIP stream:
  an event recorded at the grad-ready point on the stream the backward was ARMED on
  (not the hook's stream: autograd runs a leaf's hook on the stream of the forward
  that first used it) orders the bucket's all-reduce after its gradient kernels, and finalize() makes the
  compute stream wait on the comm stream (no host synchronisation).  Buckets are
  launched in order so every rank issues collectives in the same sequence.
* ``no_sync()`` has torch-DDP semantics: the decision is taken at *forward*
  time, so gradient accumulation over micro-batches issues exactly one
  reduction per optimizer step (SURVEY P-GA).
* The 1/world averaging is NOT applied here: the fused AdamW kernel folds it
  into its gradient scale (one fewer pass over 348 MiB per step).  Call
  :meth:`average_gradients` if a plain torch optimizer consumes the grads.
* Startup: one flat broadcast of all parameters from rank 0 plus a shape
  checksum all-reduce (replaces DDP's per-tensor broadcast, SURVEY X-4).
* Hook-free backward (e.g. a replayed HIP graph, where no Python hook fires):
  :meth:`reduce_all_now` launches every bucket after it.
* Unused parameters: a bucket whose hooks have not all fired by ``finalize()`` is
  launched there, after backward, without overlap (torch DDP raises instead).  The
  first armed step records which hooks fired and warns once, naming the unused
  parameters (``DPA_DDP_UNUSED=error`` raises instead).
* IPC data plane (``DPA_IPC_ALLREDUCE=1``): the kernels' bounded spin sets an error
  word on timeout instead of hanging; :meth:`step_skip_flag` hands it to the fused
  AdamW (the step is refused on the device, no host sync) and the engine reads it
  back asynchronously and raises at the next ``finalize()``.
* ZeRO-1 (``shard_optimizer=True``, parallel/zero.py): buckets are padded to a
  multiple of world x 16 elements and REDUCE-SCATTERED instead of all-reduced;
  rank r receives the summed r-th chunk of every bucket in a compact
  ``grad_shard`` buffer, the sharded optimizer updates only those elements (writing
  their bf16 compute shadow in the same kernel) and :meth:`gather_params` all-gathers
  the updated chunks of the bf16 SHADOW, half the bytes of the fp32 master, as async
  per-bucket collectives issued in the order the next forward needs them (the first
  layers' buckets first); the next forward waits for them.  The fp32 master is then
  stale outside this rank's chunks until :meth:`materialize_master` (checkpoint saves,
  replica checks) gathers it.  ``DPA_ZERO_GATHER=fp32`` gathers the fp32 master every
  step instead (and refreshes the shadow from it), as before.
"""
import contextlib
import os
import warnings

import torch
import torch.distributed as dist
from torch import nn

from ..ops._ext import get_ext
from .flat import ALIGN, FlatParamSpace, layout_order

_MiB = 1024 * 1024


def bucket_members(numels, cap_mb, first_mb):
    """Bucket membership (lists of layout indices) of parameters with these element
    counts, by the same rule as :func:`plan_buckets` - computable before the flat
    space exists (the sharded engine pads the space at these bucket ends)."""
    groups, cur, off, cur_start, limit = [], [], 0, 0, first_mb * _MiB
    for i, n in enumerate(numels):
        if cur and n * 4 > cap_mb * _MiB:
            # a parameter larger than a whole bucket (GPT-2's tied 50257 x 768 embedding,
            # 154 MB) gets a bucket of its own: the parameters before it are not held back
            # until its gradient - complete only after the embedding backward - is ready
            groups.append(cur)
            cur, cur_start, limit = [], off, cap_mb * _MiB
        cur.append(i)
        off = (off + n + ALIGN - 1) // ALIGN * ALIGN
        if (off - cur_start) * 4 >= limit or i == len(numels) - 1:
            groups.append(cur)
            cur, cur_start, limit = [], off, cap_mb * _MiB
    return groups


def plan_buckets(space, cap_mb, first_mb):
    """Split the flat layout into contiguous buckets at parameter boundaries."""
    layout = space.layout
    starts = [space.offsets[id(p)] for p in layout] + [space.numel]
    buckets = []
    cur_start, cur_params = 0, []
    limit = first_mb * _MiB
    for i, p in enumerate(layout):
        if cur_params and p.numel() * 4 > cap_mb * _MiB:  # own bucket (see bucket_members)
            buckets.append((cur_start, starts[i], cur_params))
            cur_start, cur_params = starts[i], []
            limit = cap_mb * _MiB
        cur_params.append(p)
        end = starts[i + 1]
        if (end - cur_start) * 4 >= limit or i == len(layout) - 1:
            buckets.append((cur_start, end if i < len(layout) - 1 else space.numel, cur_params))
            cur_start, cur_params = end, []
            limit = cap_mb * _MiB
    return buckets


def tune_bucket_sizes(numel, *, process_group=None, device=None, sizes_mb=(2, 4, 8, 16, 32, 64, 128),
                      min_buckets=4, frac=0.9, iters=5, timer=None):
    """Bucket sizes MEASURED on this job's links (``bucket_cap_mb <= 0``): the
    all-reduce bus bandwidth of the process group at each size in ``sizes_mb``, timed on every
    rank and MAX-reduced so all ranks take the same decision.  The cap is the smallest size
    within ``frac`` of the best bandwidth (a bigger bucket only delays the first launch and the
    overlap), at most 1/``min_buckets`` of the gradients (so the reduction still overlaps the
    backward); the first bucket is the smallest size within half the best bandwidth, at most
    the cap.  On point-to-point xGMI the knee sits where one ring step's payload stops being
    latency-bound, which depends on the ring count RCCL picks - hence measured, not assumed.
    ``timer(nfloats, iters) -> seconds`` times the all-reduce on the data plane that will carry
    the buckets (the C++ reducer's own RCCL communicator and high-priority comm stream,
    ``BucketReducer.time_allreduce``); without it the process group's ``dist.all_reduce`` is timed.
    Returns ``(cap_mb, first_mb, table)``; ``(32, 4, None)`` without a multi-rank group."""
    import time
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(process_group) < 2:
        return 32.0, 4.0, None
    world = dist.get_world_size(process_group)
    backend = dist.get_backend(process_group)
    dev = device if (backend == "nccl" and device is not None and device.type == "cuda") else torch.device("cpu")
    grad_mb = numel * 4 / _MiB
    sizes = [mb for mb in sizes_mb if mb <= max(sizes_mb[0], grad_mb)]
    times = []
    for mb in sizes:
        if timer is not None:
            times.append(timer(int(mb * _MiB) // 4, iters))
            continue
        x = torch.ones(int(mb * _MiB) // 4, dtype=torch.float32, device=dev)
        dist.all_reduce(x, group=process_group)  # warm: channel / buffer setup outside the timing
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(x, group=process_group)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        times.append((time.perf_counter() - t) / iters)
        del x
    tt = torch.tensor(times, dtype=torch.float64, device=dev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=process_group)
    times = tt.tolist()
    bw = [mb * _MiB * 2 * (world - 1) / world / t / 1e9 for mb, t in zip(sizes, times)]
    best = max(bw)
    limit = max(sizes[0], grad_mb / min_buckets)
    ok = [mb for mb, b in zip(sizes, bw) if b >= frac * best and mb <= limit]
    cap = float(ok[0] if ok else max([mb for mb in sizes if mb <= limit] or [sizes[0]]))
    half = [mb for mb, b in zip(sizes, bw) if b >= 0.5 * best and mb <= cap]
    first = float(half[0] if half else sizes[0])
    table = [{"mb": mb, "us": round(t * 1e6, 1), "busbw_GBps": round(b, 1)} for mb, t, b in zip(sizes, times, bw)]
    return cap, first, table


class _Bucket:
    __slots__ = ("index", "start", "end", "params", "pending", "work", "launched")

    def __init__(self, index, start, end, params):
        self.index, self.start, self.end, self.params = index, start, end, params
        self.pending = len(params)
        self.work = None
        self.launched = False


class DDPEngine(nn.Module):
    def __init__(self, module, *, device=None, bucket_cap_mb=32.0, first_bucket_mb=4.0,
                 shadow_dtype=None, process_group=None, reduce_dtype=torch.float32,
                 broadcast_from_rank0=True, space=None, shard_optimizer=False):
        super().__init__()
        self.module = module
        self.pg = process_group
        self.distributed = dist.is_available() and dist.is_initialized()
        self.sim_comm = None  # enable_sim_comm(): the simulated data plane's parameters
        self.bucket_tune = None
        # "auto" bucket sizes are measured on this job's links.  ZeRO-1 pads the flat space at
        # bucket ends, so its plan is measured up front on the process group; otherwise the plan
        # starts provisional (32 / 4 MiB) and is re-measured on the data plane itself once the
        # reducer's communicator exists (_tune_on_data_plane)
        self._tune_later = None
        if bucket_cap_mb is None or bucket_cap_mb <= 0:
            numel = sum(p.numel() for p in module.parameters() if p.requires_grad)
            auto_first = first_bucket_mb is None or first_bucket_mb <= 0
            if shard_optimizer and dist.is_available() and dist.is_initialized():
                dev = device if device is not None else next(module.parameters()).device
                bucket_cap_mb, tuned_first, self.bucket_tune = tune_bucket_sizes(
                    numel, process_group=process_group, device=torch.device(dev))
                if self.bucket_tune is not None:
                    self.bucket_tune = {"timed_on": "process group (ZeRO-1 layout is fixed before the reducer)",
                                        "sweep": self.bucket_tune}
                if auto_first:
                    first_bucket_mb = tuned_first
            else:
                self._tune_later = (numel, auto_first, device)
                bucket_cap_mb = 32.0
                if auto_first:
                    first_bucket_mb = 4.0
        elif first_bucket_mb is None or first_bucket_mb <= 0:
            # an explicit cap with the first bucket left at "auto": the fixed 4 MiB default (a
            # 0 MiB first bucket would close after one parameter)
            first_bucket_mb = 4.0
        first_bucket_mb = min(first_bucket_mb, bucket_cap_mb)
        self.world_size = dist.get_world_size(self.pg) if self.distributed else 1
        self.rank = dist.get_rank(self.pg) if self.distributed else 0
        # (world 1 keeps the sharded machinery - one shard - so it can be exercised alone)
        self.sharded = bool(shard_optimizer) and self.distributed
        # the flat layout follows the order gradients complete in the backward when the module
        # says it (grad_ready_order): buckets are launched in layout order, so one parameter
        # whose gradient completes late holds back every bucket after its own
        ready_order = module.grad_ready_order() if callable(getattr(module, "grad_ready_order", None)) else None
        if space is None:
            kw = {"order": ready_order}
            if self.sharded:
                # pad every bucket end so each bucket splits into world equal 16-aligned chunks
                layout = layout_order(module.parameters(), order=ready_order)
                groups = bucket_members([p.numel() for p in layout], bucket_cap_mb, first_bucket_mb)
                kw.update(break_after={g[-1] for g in groups}, break_align=self.world_size * ALIGN)
            space = FlatParamSpace(module.parameters(), device=device, shadow_dtype=shadow_dtype, **kw)
        self.space = space
        self.reduce_dtype = reduce_dtype
        self._sync_enabled = True
        self._armed = False
        self._arm_stream = None      # the armed backward's stream (see _arm)
        self._next_launch = 0
        self.bucket_cap_mb, self.first_bucket_mb = bucket_cap_mb, first_bucket_mb
        self._log_bucket_plan()
        self.buckets = [_Bucket(i, s, e, ps) for i, (s, e, ps) in
                        enumerate(plan_buckets(self.space, bucket_cap_mb, first_bucket_mb))]
        self._bucket_of = {}
        for b in self.buckets:
            for p in b.params:
                self._bucket_of[id(p)] = b
        self._hooks = []
        self._shadow_works = []      # ZeRO-1: outstanding async shadow all-gathers
        self._master_stale = False   # ZeRO-1: fp32 master valid only in this rank's chunks
        self._fired = set()          # layout indices whose hook fired (first armed step only)
        self._fire_seq = []          # ... in firing order
        self.bucket_order_report = None  # first armed step: do buckets complete in launch order?
        self._track_unused = True
        self._ipc_flag = None        # device int32 error word of the IPC all-reduce
        self._ipc_host = None
        self._ipc_event = None
        self._comm_buf = None
        self._comm_out = None
        self.grad_shard = None
        self.shard_chunks = []  # per bucket: (flat start of this rank's chunk, length, shard offset)
        if self.sharded:
            off = 0
            for b in self.buckets:
                n = b.end - b.start
                if n % (self.world_size * ALIGN):
                    raise RuntimeError(f"bucket {b.index} ({n} elements) is not world-divisible")
                c = n // self.world_size
                self.shard_chunks.append((b.start + self.rank * c, c, off))
                off += c
            self.grad_shard = torch.zeros(off, dtype=torch.float32, device=self.space.device)
        # gloo on device tensors is only a test transport (several ranks sharing one
        # GPU): stage each bucket through host memory synchronously so its ordering
        # w.r.t. the producing kernels is explicit.  RCCL ("nccl") orders via events.
        self._backend = dist.get_backend(self.pg) if self.distributed else None
        self._host_sync_before_comm = (self.distributed and self.space.device.type == "cuda"
                                       and self._backend == "gloo")
        # Native C++ bucket reducer (csrc/comm/reducer.cpp) for the real transports;
        # the Python implementation below stays as the reference / test transport.
        # The sharded (reduce-scatter) mode needs a backend with reduce_scatter: RCCL.
        self._native = None
        # opt-in direct xGMI all-reduce over IPC-mapped peer buffers (fp32 all-reduce buckets;
        # csrc/ipc_allreduce.hip) instead of RCCL rings.  Over gloo (several ranks on one device,
        # where RCCL refuses to run) the reducer takes it without a communicator: gloo only
        # exchanges the IPC handles and carries the control plane (tests/test_ipc_reducer_gpu.py)
        ipc_req = (self.distributed and os.environ.get("DPA_IPC_ALLREDUCE", "0") == "1" and not self.sharded
                   and self.reduce_dtype == torch.float32 and 1 < self.world_size <= 8
                   and self.space.device.type == "cuda")
        ipc_only = ipc_req and self._backend == "gloo"
        if (self.distributed and (not self._host_sync_before_comm or ipc_only)
                and (not self.sharded or self._backend == "nccl")
                and os.environ.get("DPA_NATIVE_REDUCER", "1") != "0"):
            ext = get_ext(required=False)
            if ext is not None and hasattr(ext, "BucketReducer"):
                pg = self.pg or dist.distributed_c10d._get_default_group()
                bounds = [b.start for b in self.buckets] + [self.buckets[-1].end]
                param_bucket = [self._bucket_of[id(p)].index for p in self.space.layout]
                # SURVEY N-2: on RCCL the reducer owns its communicator + a highest-
                # priority comm stream (DPA_REDUCER_COMM=pg: collectives through the c10d PG)
                uid = ""
                if (self._backend == "nccl" and self.space.device.type == "cuda"
                        and os.environ.get("DPA_REDUCER_COMM", "direct") == "direct"
                        and hasattr(ext, "rccl_unique_id")):
                    box = [ext.rccl_unique_id() if self.rank == 0 else None]
                    dist.broadcast_object_list(box, src=dist.get_global_rank(pg, 0), group=self.pg)
                    uid = box[0]
                self._native = ext.BucketReducer(pg, self.space.grad_flat, bounds, param_bucket,
                                                 self.reduce_dtype == torch.bfloat16,
                                                 self.grad_shard if self.sharded else None,
                                                 [c[2] for c in self.shard_chunks], uid, self.rank,
                                                 self.world_size, self._plan_comm_stream())
                if ipc_req and (uid or ipc_only):
                    if not uid:
                        self._native.init_ipc_only(self.rank)
                    blobs = [None] * self.world_size
                    dist.all_gather_object(blobs, self._native.ipc_export(), group=self.pg)
                    self._native.ipc_open(blobs)
                    self._ipc_flag = self._native.ipc_error_flag()
                    self._ipc_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
                    self._ipc_event = torch.cuda.Event()
        if self._tune_later is not None:
            self._tune_on_data_plane()
        if self.distributed and self.world_size > 1 and self.space.device.type == "cuda":
            # collectives share the CUs with the persistent GEMMs: let late-starting GEMM
            # workgroups take fewer tiles instead of finishing last (csrc/gemm256.hip)
            ext = get_ext(required=False)
            if ext is not None and hasattr(ext, "set_gemmp_dynamic"):
                ext.set_gemmp_dynamic(True)
        if self.distributed:
            self._verify_shapes()
            if broadcast_from_rank0:
                self.broadcast_parameters()
            self._install_hooks()

    # -- setup ---------------------------------------------------------------
    def _plan_comm_stream(self):
        """Handle of the stream plan's data-plane stream (runtime/streams.py role "comm": one of
        the pooled hardware queues); 0 (the reducer creates its own) off the GPU or without a plan."""
        if self.space.device.type != "cuda":
            return 0
        try:
            from ..runtime.streams import plan_stream
            s = plan_stream(self.space.device, "comm")
        except Exception:  # noqa: BLE001 - a plan is an optimisation, never a requirement
            return 0
        return int(s.cuda_stream) if s is not None else 0

    def _install_hooks(self):
        """One post-accumulate-grad hook per parameter.  It fires once per backward per leaf,
        also when a fused op wrote the gradient in place and returned None for it
        (AccumulateGrad still runs), so no op-side notification is needed.  Installed only
        while a backward can be armed: every micro-batch under ``no_sync`` runs without them
        (``forward`` removes them), because the reference 32 x 64 schedule would otherwise make
        161 x 31 Python hook calls per step that reduce nothing - measured on the simulated
        data plane as +43-63 ms/step of host time on a GPU-bound 210 ms step
        (profiles/sim_comm_r6.json)."""
        if self._hooks:
            return
        self._hooks = [p.register_post_accumulate_grad_hook(self._make_hook(p, i))
                       for i, p in enumerate(self.space.layout)]

    def _remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []

    def _log_bucket_plan(self):
        if self.bucket_tune is None or (self.distributed and dist.get_rank() != 0):
            return
        # measured sizes can differ run to run (and so can the bucket boundaries, hence the
        # order of the summation): say which were taken; pass them back as --ddp_bucket_cap_mb /
        # --ddp_first_bucket_mb to repeat the same bucket plan
        try:
            from basic_utils import logger
            logger.log(f"DDP buckets: cap {self.bucket_cap_mb} MiB, first {self.first_bucket_mb} MiB (measured on "
                       f"{self.bucket_tune.get('timed_on')}; set them explicitly to repeat this bucket plan)")
        except ImportError:  # pragma: no cover
            pass

    def _tune_on_data_plane(self):
        """Measure the bucket sizes on the data plane that carries them: the reducer's own RCCL
        communicator and comm stream when it has one (direct mode), else the process group;
        then re-plan the buckets (C++ reducer: ``set_buckets``)."""
        numel, auto_first, device = self._tune_later
        self._tune_later = None
        direct = self._native is not None and self._native.direct()
        timer = (lambda n, it: self._native.time_allreduce(n, it) / 1e3) if direct else None
        dev = device if device is not None else self.space.device
        cap, first, table = tune_bucket_sizes(numel, process_group=self.pg, device=torch.device(dev), timer=timer)
        if table is None:
            return
        self.bucket_tune = {"timed_on": ("reducer-owned RCCL communicator, comm stream" if direct
                                         else "process group"), "sweep": table}
        self.bucket_cap_mb = cap
        self.first_bucket_mb = min(first if auto_first else self.first_bucket_mb, cap)
        self.buckets = [_Bucket(i, s, e, ps) for i, (s, e, ps) in
                        enumerate(plan_buckets(self.space, self.bucket_cap_mb, self.first_bucket_mb))]
        self._bucket_of = {id(p): b for b in self.buckets for p in b.params}
        if self._native is not None:
            self._native.set_buckets([b.start for b in self.buckets] + [self.buckets[-1].end],
                                     [self._bucket_of[id(p)].index for p in self.space.layout])
        self._log_bucket_plan()

    def _coll_device(self):
        return self.space.device

    def _verify_shapes(self):
        sig = torch.tensor([self.space.numel, len(self.space.layout),
                            sum((i + 1) * p.numel() for i, p in enumerate(self.space.layout))],
                           dtype=torch.int64, device=self._coll_device())
        mx, mn = sig.clone(), sig.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=self.pg)
        dist.all_reduce(mn, op=dist.ReduceOp.MIN, group=self.pg)
        if not torch.equal(mx, mn):
            raise RuntimeError("DDPEngine: parameter shapes differ across ranks")

    def broadcast_parameters(self, src=0):
        if self.distributed:
            dist.broadcast(self.space.param_flat, src, group=self.pg)
            self.space.refresh_shadow()

    def broadcast_flat(self, flat, src=0):
        if self.distributed:
            dist.broadcast(flat, src, group=self.pg)

    @property
    def _reducing(self):
        """Gradients go through a data plane: a real process group, or the simulated one."""
        return self.distributed or self.sim_comm is not None

    # -- one-GPU projection of W > 1 ------------------------------
    def enable_sim_comm(self, world, busbw_gbps, cus=64, lat_us=10.0, bucket_cap_mb=None, first_bucket_mb=None,
                        comm_stream=None):
        """Run this world-1 engine's backward against a SIMULATED world-``world`` data plane
        (csrc/comm_sim.hip via the C++ reducer's sim mode): every bucket, when its gradients are
        ready, launches on the reducer's high-priority comm stream a kernel of ``cus`` workgroups
        that holds its CUs for ``lat_us + 2 (W - 1) / W x bytes / busbw`` and moves the ring's
        local HBM bytes; ``finalize()`` orders the optimizer after it, as after a real
        all-reduce.  The gradients stay this rank's (the step's math is world 1), the GEMMs take
        the dynamic tile schedule a W > 1 run uses, and the reducer accumulates per-step timeline
        sums on the device (:meth:`sim_stats`).  A projection, not a scaling measurement: the
        link model is the caller's (``busbw_gbps``), the overlap with this rank's compute is
        measured.  ``bucket_cap_mb`` / ``first_bucket_mb`` re-plan the buckets first (e.g. the
        reference's 128 / 1 MiB)."""
        if self.distributed:
            raise RuntimeError("enable_sim_comm: a world-1 engine only (the real data plane is active)")
        if self.space.device.type != "cuda":
            raise RuntimeError("enable_sim_comm: device gradients only")
        ext = get_ext(required=True)
        self.disable_sim_comm()
        if bucket_cap_mb is not None:
            first = first_bucket_mb if first_bucket_mb is not None else min(4.0, bucket_cap_mb)
            self.bucket_cap_mb, self.first_bucket_mb = bucket_cap_mb, min(first, bucket_cap_mb)
            self.buckets = [_Bucket(i, s, e, ps) for i, (s, e, ps) in
                            enumerate(plan_buckets(self.space, self.bucket_cap_mb, self.first_bucket_mb))]
            self._bucket_of = {id(p): b for b in self.buckets for p in b.params}
        bounds = [b.start for b in self.buckets] + [self.buckets[-1].end]
        param_bucket = [self._bucket_of[id(p)].index for p in self.space.layout]
        red = ext.BucketReducer.simulated(self.space.grad_flat, bounds, param_bucket,
                                          self.reduce_dtype == torch.bfloat16)
        # comm_stream: a torch stream for the stand-in kernels (A/B of the queue the data plane runs
        # on); None: the stream plan's comm stream, as the real data plane
        red.init_sim(int(world), float(busbw_gbps), int(cus), float(lat_us),
                     int(comm_stream.cuda_stream) if comm_stream is not None else self._plan_comm_stream())
        self._native = red
        self.sim_comm = {"world": int(world), "busbw_GBps": float(busbw_gbps), "cus": int(cus),
                         "lat_us": float(lat_us), "bucket_mb": self.bucket_sizes_mb(),
                         "wire": "bf16" if self.reduce_dtype == torch.bfloat16 else "fp32"}
        self._track_unused = True  # the first simulated step checks the bucket completion order
        self._install_hooks()
        if hasattr(ext, "set_gemmp_dynamic"):
            ext.set_gemmp_dynamic(True)  # as a W > 1 run (collectives share the CUs)
        return self.sim_comm

    def disable_sim_comm(self):
        if self.sim_comm is None:
            return
        self._remove_hooks()
        self._native = None
        self.sim_comm = None
        self._armed = False
        ext = get_ext(required=False)
        if ext is not None and hasattr(ext, "set_gemmp_dynamic"):
            ext.set_gemmp_dynamic(False)

    def sim_timeline(self):
        """The last step's per-bucket [grad ready, first start, last end] (ms after the first
        grad-ready stamp) and, as the last row, the backward's end (host sync; diagnostics)."""
        if self.sim_comm is None:
            return None
        return [[round(x, 3) for x in row] for row in self._native.sim_timeline().tolist()]

    def sim_stats(self, reset=False):
        """Simulated data plane, sums since the last reset (ms): steps, exposed tail (comm
        still running after the backward's last kernel), grad-ready -> first-workgroup delay
        summed over buckets, bucket busy time summed, comm-stream span; plus per-step means."""
        if self.sim_comm is None:
            return None
        v = self._native.sim_stats()
        n = max(1.0, v[0])
        out = {"steps": int(v[0]), "exposed_tail_ms": round(v[1] / n, 3), "ready_to_start_ms": round(v[2] / n, 3),
               "bucket_busy_ms": round(v[3] / n, 3), "comm_span_ms": round(v[4] / n, 3),
               "last_step_tail_ms": round(v[5], 3),
               "model_ms_per_step": round(sum(self._native.sim_bucket_ms(int((b.end - b.start) * (
                   2 if self.reduce_dtype == torch.bfloat16 else 4))) for b in self.buckets), 3),
               "last_bucket_model_ms": round(self._native.sim_bucket_ms(int((self.buckets[-1].end - self.buckets[-1].start) * (
                   2 if self.reduce_dtype == torch.bfloat16 else 4))), 3)}
        if reset:
            self._native.sim_reset()
        return out

    # -- forward ---------------------------------------------------------------
    def forward(self, *args, **kwargs):
        self.wait_shadow()
        if self._reducing and torch.is_grad_enabled() and self.training:
            self._armed = self._sync_enabled
            if self._armed:
                self._arm()
            else:
                if self._native is not None and self._native.armed():
                    self._native.disarm()
                self._remove_hooks()  # a no_sync backward reduces nothing: no hook calls
        return self.module(*args, **kwargs)

    def _arm(self):
        """Arm for a backward that produces its gradients on the CURRENT stream.  The
        bucket launches are ordered after that stream, not after whatever stream a hook
        happens to run on: autograd runs a leaf's AccumulateGrad (and its post-accumulate
        hook) on the stream of the forward that first used the leaf, which in the
        overlapped micro-batch schedule is often the other stream."""
        self._install_hooks()
        cuda = self.space.device.type == "cuda"
        self._arm_stream = torch.cuda.current_stream(self.space.device) if cuda else None
        if self._native is not None:
            self._native.arm(self._arm_stream.cuda_stream if cuda else 0)
            return
        for b in self.buckets:
            b.pending = len(b.params)
            b.work = None
            b.launched = False
        self._next_launch = 0

    def arm_for_backward(self):
        """Arm the reducer for the next backward regardless of how the forward ran: the
        overlapped micro-batch schedule (utils/trainer.py) runs every forward under
        ``no_sync`` - the last micro-batch's forward is issued while an earlier backward
        is still being issued - and arms right before the last backward."""
        if not self._reducing:
            return
        self._armed = True
        self._arm()

    def disarm(self):
        """Abandon a partially run backward (e.g. an out-of-memory retry): no bucket of
        it may be reduced, and the next forward re-arms."""
        if self._native is not None:
            self._native.disarm()
        self._armed = False

    @contextlib.contextmanager
    def no_sync(self):
        prev = self._sync_enabled
        self._sync_enabled = False
        try:
            yield
        finally:
            self._sync_enabled = prev

    # -- reduction ----------------------------------------------------------------
    def _make_hook(self, p, index):
        if self._native is not None:
            native = self._native

            def native_hook(_param):
                if self._track_unused and self._armed:
                    self._fired.add(index)
                    self._fire_seq.append(index)
                native.mark_ready(index)  # no-op unless armed
            return native_hook

        def hook(_param):
            if not self._armed:
                return
            if self._track_unused:
                self._fired.add(index)
                self._fire_seq.append(index)
            b = self._bucket_of[id(p)]
            b.pending -= 1
            if b.pending == 0:
                if self._arm_stream is not None:
                    with torch.cuda.stream(self._arm_stream):
                        self._launch_ready_in_order()
                else:
                    self._launch_ready_in_order()
        return hook

    def _launch_ready_in_order(self):
        while self._next_launch < len(self.buckets):
            b = self.buckets[self._next_launch]
            if b.pending > 0:
                return
            self._launch(b)
            self._next_launch += 1

    def _wire(self):
        if self._comm_buf is None:
            self._comm_buf = torch.empty(self.space.numel, dtype=self.reduce_dtype,
                                         device=self.space.device)
        return self._comm_buf

    def _launch_sharded(self, b, view):
        s, c, off = self.shard_chunks[b.index]
        out = self.grad_shard[off:off + c]
        if self._backend != "nccl":
            # gloo (CPU tests / host-staged transport) has no reduce_scatter: all-reduce
            # the bucket and keep this rank's chunk (same sums, twice the traffic)
            full = view.to("cpu") if view.is_cuda else view.clone()
            dist.all_reduce(full, group=self.pg)
            out.copy_(full[s - b.start:s - b.start + c])
            b.work = None
        elif self.reduce_dtype == torch.float32:
            b.work = dist.reduce_scatter_tensor(out, view, group=self.pg, async_op=True)
        else:
            wire = self._wire()[b.start:b.end]
            wire.copy_(view)
            if self._comm_out is None:
                self._comm_out = torch.empty_like(self.grad_shard, dtype=self.reduce_dtype)
            wout = self._comm_out[off:off + c]
            b.work = (dist.reduce_scatter_tensor(wout, wire, group=self.pg, async_op=True), wout, out)
        b.launched = True

    def _launch(self, b):
        if b.launched:
            return
        view = self.space.grad_flat[b.start:b.end]
        if self.sharded:
            self._launch_sharded(b, view)
            return
        if self._host_sync_before_comm:
            # test transport: stage through host memory synchronously (gloo's own
            # device-tensor path is not used)
            host = view.to("cpu")
            dist.all_reduce(host, group=self.pg)
            view.copy_(host)
            b.work = None
            b.launched = True
            return
        if self.reduce_dtype == torch.float32:
            b.work = dist.all_reduce(view, group=self.pg, async_op=True)
        else:  # narrow wire format: pack, reduce, unpack (fp32 accumulation of ranks in RCCL)
            if self._comm_buf is None:
                self._comm_buf = torch.empty(self.space.numel, dtype=self.reduce_dtype,
                                             device=self.space.device)
            buf = self._comm_buf[b.start:b.end]
            buf.copy_(view)
            b.work = (dist.all_reduce(buf, group=self.pg, async_op=True), buf, view)
        b.launched = True

    def finalize(self):
        """Wait for (and launch any not-yet-launched) bucket reductions."""
        if not self._reducing or not self._armed:
            return
        if self._native is not None:
            self._check_ipc_error()
            self._native.finalize()
            self._armed = False
            self._check_unused(self._native.late_buckets())
            if self._ipc_flag is not None:
                self._ipc_host.copy_(self._ipc_flag, non_blocking=True)
                self._ipc_event.record()
            return
        late = [b.index for b in self.buckets[self._next_launch:] if b.pending > 0]
        for b in self.buckets[self._next_launch:]:
            self._launch(b)
        self._next_launch = len(self.buckets)
        for b in self.buckets:
            w = b.work
            if isinstance(w, tuple):
                w[0].wait()
                w[2].copy_(w[1])
            elif w is not None:
                w.wait()
            b.work = None
        self._armed = False
        self._check_unused(late)

    def _check_unused(self, late_buckets):
        """First armed step: name the parameters whose grad-ready hook never fired (their
        buckets were reduced late, after backward); later steps are not tracked."""
        if not self._track_unused:
            return
        self._track_unused = False
        self._check_bucket_order()
        if not late_buckets:
            self._fired.clear()
            return
        idx = {id(p): i for i, p in enumerate(self.space.layout)}
        names = {id(p): n for n, p in self.module.named_parameters()}
        unused = [names.get(id(p), f"<param {idx[id(p)]}>") for b in late_buckets
                  for p in self.buckets[b].params if idx[id(p)] not in self._fired]
        self._fired.clear()
        msg = (f"DDPEngine: {len(unused)} parameter(s) received no gradient in this step "
               f"({', '.join(unused[:8])}{'...' if len(unused) > 8 else ''}); buckets {list(late_buckets)} "
               "were all-reduced after backward, so their communication no longer overlaps it. "
               "Remove the unused parameters from the model (DPA_DDP_UNUSED=error raises).")
        if os.environ.get("DPA_DDP_UNUSED", "warn") == "error":
            raise RuntimeError(msg)
        warnings.warn(msg, RuntimeWarning, stacklevel=3)

    ORDER_SLACK = 8  # hook firings (see _check_bucket_order)

    def _check_bucket_order(self):
        """First armed step: buckets are launched in layout order, so a bucket whose last
        gradient completes after a later bucket's holds that one back (no overlap for it).  Warn
        and name the parameter; the fix is a ``grad_ready_order()`` on the module."""
        seq, self._fire_seq = self._fire_seq, []
        if not seq:
            return
        pos = {i: k for k, i in enumerate(seq)}
        idx = {id(p): i for i, p in enumerate(self.space.layout)}
        done = []
        for b in self.buckets:
            ks = [pos.get(idx[id(p)], -1) for p in b.params]
            done.append(max(ks))
        # a later bucket completing a few hook firings earlier is one fused backward op returning
        # several parameters' gradients at once (their hooks fire back to back in an order autograd
        # picks): no real hold-back.  Only a completion more than ORDER_SLACK firings late is.
        held = [b for b in range(len(done) - 1) if done[b] > min(done[b + 1:]) + self.ORDER_SLACK]
        self.bucket_order_report = {"bucket_completion_rank": done, "held_back_by": held}
        if held:
            names = {id(p): n for n, p in self.module.named_parameters()}
            b = held[0]
            late = max(self.buckets[b].params, key=lambda p: pos.get(idx[id(p)], -1))
            warnings.warn(f"DDPEngine: bucket {b} completes after later buckets (its last gradient: "
                          f"{names.get(id(late), '?')}), so their all-reduces wait for it; give the module a "
                          f"grad_ready_order() (parallel/flat.py layout_order)", RuntimeWarning, stacklevel=3)

    def step_skip_flag(self):
        """Device int32 word that is non-zero when this step's gradient reduction failed
        (IPC all-reduce timeout); pass it to the fused optimizer's ``skip``.  None when no
        such failure mode is active."""
        return self._ipc_flag

    def _check_ipc_error(self):
        """Raise on a previous step's IPC all-reduce failure (read back asynchronously)."""
        if self._ipc_flag is None or not self._ipc_event.query():
            return
        if int(self._ipc_host[0]) != 0:
            raise RuntimeError("DDPEngine: the IPC all-reduce timed out waiting for a peer (its "
                               "gradients were not reduced; the optimizer step was refused). "
                               "Ranks drifted apart by more than the kernel's 20 s bound - "
                               "unset DPA_IPC_ALLREDUCE to use RCCL, which blocks instead.")

    def comm_ranks(self):
        """Ranks of the communicator the data plane reduces over: the reducer-owned RCCL
        communicator's ``ncclCommCount`` in direct mode, else the process group's size
        (1 when not distributed).  ``bench.py`` reports it as evidence that RCCL saw N ranks."""
        if not self.distributed:
            return 1
        if self._native is not None and self._native.direct():
            return int(self._native.comm_size())
        return dist.get_world_size(self.pg)

    def warmup_comm(self):
        """One reduction of every bucket (of zeroed gradients) on the data plane and one
        c10d all-reduce of the largest bucket's size, so that RCCL's lazily allocated
        channel buffers - of the reducer-owned communicator and of the process group's -
        exist before the trainer sizes its executed micro-batch against free HBM
        (``TrainLoop._settle_exec_microbatch``).  Leaves the gradients zero."""
        if not self.distributed:
            return
        self.zero_grad()
        self.reduce_all_now()
        dev = self.space.grad_flat.device
        if dist.get_backend(self.pg) != "nccl":
            dev = torch.device("cpu")
        big = max(b.end - b.start for b in self.buckets)
        dist.all_reduce(torch.zeros(big, dtype=torch.float32, device=dev), group=self.pg)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        self.zero_grad()

    def reduce_all_now(self):
        """Graph mode: backward ran without hooks; reduce every bucket now."""
        if not self._reducing:
            return
        if self._native is not None:
            self._native.reduce_all()
            return
        self._armed = True
        for b in self.buckets:
            b.launched = False
        self._next_launch = 0
        # no hook fired here by design: this is not the first-backward check of unused
        # parameters / bucket order (which would flag every parameter and then be spent)
        track, self._track_unused = self._track_unused, False
        try:
            self.finalize()
        finally:
            self._track_unused = track

    def average_gradients(self):
        if self.world_size > 1:
            (self.grad_shard if self.sharded else self.space.grad_flat).mul_(1.0 / self.world_size)

    # -- ZeRO-1 helpers -----------------------------------------------------------------
    def _gather_direct(self):
        """ZeRO-1 gathers go through the reducer's own communicator and comm stream (direct mode):
        never on the process group's pool stream, which shares a hardware queue with compute."""
        return self._native is not None and self._native.direct()

    def all_gather_chunks(self, full):
        """``full`` is a flat buffer laid out like the parameters whose per-bucket chunk
        ``shard_chunks[b]`` is valid on each owning rank: gather every bucket in place."""
        if self._gather_direct():
            self._native.all_gather_buckets(full, list(range(len(self.buckets))))
            self._native.wait_gather()
            return
        for b, (s, c, _off) in zip(self.buckets, self.shard_chunks):
            whole = full[b.start:b.end]
            mine = full[s:s + c]
            if self._host_sync_before_comm:  # gloo on device tensors: host-staged
                host = whole.to("cpu")
                dist.all_gather_into_tensor(host, host[s - b.start:s - b.start + c].clone(),
                                            group=self.pg)
                whole.copy_(host)
            elif self._backend == "nccl":
                dist.all_gather_into_tensor(whole, mine, group=self.pg)  # in place
            else:
                dist.all_gather_into_tensor(whole, mine.clone(), group=self.pg)

    def gather_params(self):
        """After the sharded optimizer step: every rank's updated chunks to every rank.
        With a bf16 compute shadow (the optimizer wrote this rank's shadow chunks) only
        the shadow is gathered - async, per bucket, first-needed first - and the fp32
        master is marked stale; otherwise the fp32 chunks are gathered and the shadow
        refreshed from them."""
        if not self.sharded:
            return
        sh = self.space.shadow_flat
        if sh is None or os.environ.get("DPA_ZERO_GATHER", "bf16") == "fp32":
            self.all_gather_chunks(self.space.param_flat)
            self.space.refresh_shadow()
            self._master_stale = False
            return
        if os.environ.get("DPA_ZERO_POISON") == "1":
            # test hook: NaN into the fp32 master outside this rank's chunks, so any read
            # of a stale master element (instead of the gathered shadow) shows up
            keep = torch.zeros(self.space.numel, dtype=torch.bool, device=self.space.param_flat.device)
            for s_, c, _ in self.shard_chunks:
                keep[s_:s_ + c] = True
            self.space.param_flat.masked_fill_(~keep, float("nan"))
        if self._gather_direct():
            # the layout runs from the last layers to the first: the buckets the next forward
            # needs first (the highest) go first, on the comm stream; wait_shadow() orders the
            # next forward after them
            self._native.all_gather_buckets(sh, list(reversed(range(len(self.buckets)))))
            self._shadow_works.append("native")
            self.space.shadow_written()
            self._master_stale = True
            return
        # bit copy as int32 pairs (gloo has no 16-bit all-gather; every bucket and chunk
        # boundary is a multiple of 16 elements)
        wire = sh.view(torch.int32)
        # the layout runs from the last layers to the first: issue the buckets the next
        # forward needs first (the highest) first
        for b, (s_, c, _off) in reversed(list(zip(self.buckets, self.shard_chunks))):
            whole = wire[b.start // 2:b.end // 2]
            mine = wire[s_ // 2:(s_ + c) // 2]
            if self._host_sync_before_comm:  # gloo on device tensors: host-staged, synchronous
                host = whole.to("cpu")
                lo = (s_ - b.start) // 2
                dist.all_gather_into_tensor(host, host[lo:lo + c // 2].clone(), group=self.pg)
                whole.copy_(host)
            elif self._backend == "nccl":
                self._shadow_works.append(dist.all_gather_into_tensor(whole, mine, group=self.pg,
                                                                      async_op=True))
            else:
                dist.all_gather_into_tensor(whole, mine.clone(), group=self.pg)
        self.space.shadow_written()
        self._master_stale = True

    def wait_shadow(self):
        """Order the outstanding shadow all-gathers before the current stream's next work
        (a stream-side wait on RCCL, no host block)."""
        works, self._shadow_works = self._shadow_works, []
        for w in works:
            if w == "native":
                self._native.wait_gather()
            else:
                w.wait()

    def materialize_master(self):
        """Collective (every rank): make the full fp32 master current after shadow-only
        gathers (before checkpointing or reading parameters outside the forward)."""
        if self.sharded and self._master_stale:
            self.wait_shadow()
            self.all_gather_chunks(self.space.param_flat)
            self._master_stale = False

    def all_reduce_sum_(self, t):
        """Small control-plane sum (e.g. the squared grad norm) on this engine's transport."""
        if not self.distributed:
            return t
        if self._host_sync_before_comm:
            host = t.to("cpu")
            dist.all_reduce(host, group=self.pg)
            t.copy_(host)
        else:
            dist.all_reduce(t, group=self.pg)
        return t

    def zero_grad(self, set_to_none=False):  # noqa: ARG002 - flat grads are never None
        self.space.zero_grad()

    # -- misc -----------------------------------------------------------------------
    def bucket_sizes_mb(self):
        return [round((b.end - b.start) * 4 / _MiB, 3) for b in self.buckets]

    def state_dict(self, *args, **kwargs):
        return self.module.state_dict(*args, **kwargs)

    def load_state_dict(self, *args, **kwargs):
        return self.module.load_state_dict(*args, **kwargs)
