"""Two ranks sharing one HIP device (gloo transport on device tensors): the native
engine's bucket hooks, comm ordering and no_sync on real GPU streams, with the
bf16 kernels in the loop.  (RCCL itself needs distinct GPUs; its path is the
same engine code with backend "nccl".)"""
import contextlib
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from basic_utils.dist_util import find_free_port

pytestmark = pytest.mark.gpu

CFG = dict(model="diffuseq", config_name="tiny", hidden_size=256, num_layers=2, num_heads=4,
           intermediate_size=1024, vocab_size=3000, seq_len=128, hidden_dim=128, hidden_t_dim=128,
           dropout=0.0, precision="bf16")


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from distributed_pipeline_amd.models import build_model, create_gaussian_diffusion
        from distributed_pipeline_amd.parallel.ddp import DDPEngine
        torch.manual_seed(1234 + rank)  # different init per rank -> engine broadcasts rank 0
        model = build_model(**CFG).cuda()
        eng = DDPEngine(model, shadow_dtype=torch.bfloat16, bucket_cap_mb=1.0, first_bucket_mb=0.25)
        diff = create_gaussian_diffusion(steps=100)
        g = torch.Generator().manual_seed(7)
        ids = torch.randint(1000, 3000, (world, 2, 4, 128), generator=g).cuda()
        mask = torch.ones_like(ids)
        mask[..., :32] = 0
        t = torch.randint(0, 100, (world, 2, 4), generator=g).cuda()
        eng.zero_grad()
        for mb in range(2):
            ctx = eng.no_sync() if mb == 0 else torch.enable_grad()
            torch.manual_seed(99 + mb * 10 + rank)
            with ctx:
                terms = diff.training_losses(eng, None, t[rank, mb],
                                             dict(input_ids=ids[rank, mb], input_mask=mask[rank, mb]))
            terms["loss"].mean().backward()
        eng.finalize()
        q.put((rank, eng.space.grad_flat.cpu().numpy().copy(), len(eng.buckets)))
    finally:
        dist.destroy_process_group()


def test_two_ranks_one_gpu_gradients_agree():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = find_free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, g0, nb), (_, g1, _) = res
    g0, g1 = torch.from_numpy(g0), torch.from_numpy(g1)
    assert nb > 3
    assert torch.isfinite(g0).all() and g0.abs().sum() > 0
    torch.testing.assert_close(g0, g1, rtol=0, atol=0)  # all-reduced sums identical on both ranks


def _rccl_worker(port, wire, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        from distributed_pipeline_amd.models import build_model, create_gaussian_diffusion
        from distributed_pipeline_amd.parallel.ddp import DDPEngine
        torch.manual_seed(1234)
        model = build_model(**CFG).cuda()
        rd = torch.bfloat16 if wire == "bf16" else torch.float32
        eng = DDPEngine(model, shadow_dtype=torch.bfloat16, bucket_cap_mb=1.0,
                        first_bucket_mb=0.25, reduce_dtype=rd)
        native = eng._native is not None
        diff = create_gaussian_diffusion(steps=100)
        g = torch.Generator().manual_seed(7)
        ids = torch.randint(1000, 3000, (4, 128), generator=g).cuda()
        mask = torch.ones_like(ids)
        mask[:, :32] = 0
        t = torch.randint(0, 100, (4,), generator=g).cuda()

        from distributed_pipeline_amd.ops.nn import RNG

        def run(sync):
            eng.zero_grad()
            torch.manual_seed(99)
            RNG.counter = 0  # same in-kernel noise / dropout streams in both runs
            with (torch.enable_grad() if sync else eng.no_sync()):
                terms = diff.training_losses(eng, None, t, dict(input_ids=ids, input_mask=mask))
            terms["loss"].mean().backward()
            launched = eng._native.next_bucket() if native else -1
            eng.finalize()
            return eng.space.grad_flat.clone(), launched

        local, _ = run(sync=False)   # no collective
        reduced, launched = run(sync=True)  # RCCL all-reduce of every bucket (world 1: identity)
        direct = bool(native and eng._native.direct())
        # the data plane runs on the stream plan's comm stream (a pooled hardware queue)
        from distributed_pipeline_amd.runtime.streams import plan_stream
        prio = int(native and eng._native.comm_stream() == plan_stream(torch.device("cuda", 0), "comm").cuda_stream)
        q.put((native, len(eng.buckets), local.cpu().numpy(), reduced.cpu().numpy(), launched, direct,
               prio))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_native_reducer_over_rccl_single_rank(wire):
    """The C++ BucketReducer with a real RCCL process group on HIP streams: every
    bucket is launched from the autograd hooks while backward is still running, so a
    pack/launch ordered before its gradient kernels would corrupt the result."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(find_free_port(), wire, q))
    p.start()
    native, nb, local, reduced, launched, direct, prio = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert native, "native BucketReducer not used with the RCCL process group"
    assert nb > 3
    # the reducer-owned RCCL communicator on the stream plan's comm stream (SURVEY N-2; a pooled
    # queue, not a fifth high-priority one: profiles/sim_comm_r6.json), every bucket launched from
    # the grad-ready hooks while backward ran (overlap)
    assert direct and prio == 1, (direct, prio)
    assert launched == nb, f"{launched}/{nb} buckets launched before finalize()"
    local, reduced = torch.from_numpy(local), torch.from_numpy(reduced)
    assert local.abs().sum() > 0
    # split-K wgrad accumulates with fp32 atomics, so two backwards differ in rounding
    # only; an ordering bug would give zeros / partial sums instead
    err = ((reduced - local).abs().max() / local.abs().max()).item()
    assert err < (1e-5 if wire == "fp32" else 8e-3), err
    # 99.9% of elements agree to bf16 rounding
    close = torch.isclose(reduced, local, rtol=1e-2, atol=1e-6 * local.abs().max().item())
    assert close.float().mean() > 0.999


def _zero_rccl_worker(port, wire, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        from distributed_pipeline_amd.parallel.ddp import DDPEngine
        from distributed_pipeline_amd.parallel.optimizer import FusedAdamW
        from distributed_pipeline_amd.parallel.zero import ZeroFusedAdamW
        rd = torch.bfloat16 if wire == "bf16" else torch.float32
        out = []
        for sharded in (False, True):
            torch.manual_seed(5)
            model = torch.nn.Sequential(*[torch.nn.Linear(256, 256) for _ in range(4)]).cuda()
            eng = DDPEngine(model, bucket_cap_mb=0.25, first_bucket_mb=0.1, shard_optimizer=sharded,
                            reduce_dtype=rd)
            assert eng.sharded == sharded
            kw = dict(lr=1e-2, weight_decay=0.01, ema_rates=[0.9])
            opt = ZeroFusedAdamW(eng, **kw) if sharded else FusedAdamW(eng.space, **kw)
            torch.manual_seed(6)
            for _ in range(3):
                eng.zero_grad()
                x = torch.randn(64, 256, device="cuda")
                eng(x).square().mean().backward()
                eng.finalize()
                opt.step()
                if sharded:
                    eng.gather_params()
            out.append(eng.space.param_flat.detach().cpu().numpy().copy())
            if sharded:
                # the parameter all-gathers ran on the reducer's own communicator and comm stream
                # (not the process group's pool stream), and so does the bucket-size timing
                nat = eng._native
                gather_on_comm = nat.direct() and nat.last_collective_stream() == nat.comm_stream() != 0
                ms = nat.time_allreduce(1 << 20, 3)
                tune_on_comm = nat.last_collective_stream() == nat.comm_stream() and ms > 0
        q.put((out, gather_on_comm, tune_on_comm))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_zero1_reduce_scatter_over_rccl_single_rank(wire):
    """ZeRO-1 on a real RCCL communicator: buckets REDUCE-SCATTERED by the reducer's
    own communicator into the shard buffer, sharded AdamW, all-gather of the updated
    chunks - must match the unsharded engine step for step (world 1)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_zero_rccl_worker, args=(find_free_port(), wire, q))
    p.start()
    (plain, sharded), gather_on_comm, tune_on_comm = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert gather_on_comm and tune_on_comm
    torch.testing.assert_close(torch.from_numpy(sharded), torch.from_numpy(plain), rtol=1e-6, atol=1e-7)


def _rccl_overlap_worker(port, comm, q):
    """W = 1 over RCCL, the trainer's overlapped 4 x 64 schedule with weight-gradient deferral
    and a bf16 wire: the buckets are packed / reduced from hooks that autograd runs on either of
    two streams while the deferred weight gradients join before the armed last backward."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DPA_REDUCER_COMM=comm)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        from basic_utils import logger
        from distributed_pipeline_amd.ops.nn import RNG
        from utils.initialization import create_diffusion_from_config, create_model_from_config
        from utils.trainer import DiffusionTrainLoop
        logger.configure(dir="/tmp/dpa_rccl_overlap", format_strs=[])
        torch.manual_seed(1234)
        model = create_model_from_config(model="diffuseq", precision="bf16", config_name="tiny",
                                         hidden_size=256, num_layers=2, num_heads=4, intermediate_size=1024,
                                         vocab_size=3000, seq_len=128, hidden_dim=128, hidden_t_dim=128,
                                         dropout=0.1).cuda()
        diffusion, sampler = create_diffusion_from_config(diffusion_steps=100)
        g = torch.Generator().manual_seed(7)
        B, L = 256, 128
        batch = {"input_ids": torch.randint(1000, 3000, (B, L), generator=g).cuda(),
                 "input_mask": torch.cat([torch.zeros(B, 32, dtype=torch.long),
                                          torch.ones(B, L - 32, dtype=torch.long)], 1).cuda()}
        loop = DiffusionTrainLoop(diffusion=diffusion, schedule_sampler=sampler, model=model, data=iter([batch]),
                                  batch_size=B, microbatch=64, lr=1e-4, ema_rate="0.9999", log_interval=1,
                                  save_interval=10 ** 9, resume_checkpoint="", learning_steps=1,
                                  checkpoint_path="/tmp/dpa_rccl_overlap", ddp_engine="native", precision="bf16",
                                  exec_microbatch=-1, overlap_microbatches=True, defer_wgrad=4,
                                  device_prefetch=False, bucket_cap_mb=1.0, first_bucket_mb=0.25,
                                  grad_reduce_dtype="bf16")
        eng = loop.ddp_model

        def run(reduce):
            eng.zero_grad()
            torch.manual_seed(99)
            RNG.counter = 0  # same noise / dropout / timesteps in both runs
            loop.use_ddp = reduce
            with (contextlib.nullcontext() if reduce else eng.no_sync()):
                loop.forward_backward(batch)
            launched = eng._native.next_bucket() if (reduce and eng._native is not None) else -1
            if reduce:
                eng.finalize()
            torch.cuda.synchronize()
            return eng.space.grad_flat.clone(), launched

        local, _ = run(False)       # nothing armed: the local sum of the 4 micro-batches
        reduced, launched = run(True)   # the armed last backward: every bucket over the bf16 wire
        q.put((eng._native is not None, eng._native.direct() if eng._native is not None else False,
               len(eng.buckets), launched, local.cpu().numpy(), reduced.cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("comm", ["direct", "pg"])
def test_native_reducer_overlapped_schedule_bf16_wire_single_rank(comm):
    """W = 1 RCCL, the overlapped micro-batch schedule, deferred weight gradients, bf16 wire:
    the reduced gradient equals the local no-reduction gradient to bf16 rounding.  The one
    single-rank configuration where a bucket packed before its last gradient contribution
    (a mis-ordered arm / hook stream) shows: that element would miss part of its
    sum.  ``pg``: collectives through the c10d process group, ordered on the armed stream."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_overlap_worker, args=(find_free_port(), comm, q))
    p.start()
    native, direct, nb, launched, local, reduced = q.get(timeout=300)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert native and direct == (comm == "direct"), (native, direct)
    assert nb > 3 and launched == nb, (launched, nb)
    local, reduced = torch.from_numpy(local), torch.from_numpy(reduced)
    assert local.abs().sum() > 0
    # the bf16 wire rounds every element once: within 2^-8 relative of the local sum
    # (plus the fp32 atomic-order noise of two backward runs)
    tol = 2.0 ** -8 * local.abs() + 1e-6 * local.abs().max()
    bad = ((reduced - local).abs() > tol).float().mean().item()
    assert bad < 1e-3, bad
