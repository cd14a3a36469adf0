"""Native DDP engine (flat buckets, no_sync, rank-0 broadcast) on CPU/gloo, world 2 and 4.

Equivalence criterion: averaged gradients of W ranks equal the
single-process gradient of the concatenated batch to fp32 round-off.
"""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from basic_utils.dist_util import find_free_port
from distributed_pipeline_amd.parallel.ddp import DDPEngine, plan_buckets
from distributed_pipeline_amd.parallel.flat import FlatParamSpace


class _InplaceWgrad(torch.autograd.Function):
    """Mimics the fused wgrad GEMM: dW/db accumulated straight into .grad, None returned."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.params = (w, b)
        return x @ w.t() + b

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        pw, pb = ctx.params
        pw.grad.add_(dy.t() @ x)
        pb.grad.add_(dy.sum(0))
        return dy @ w, None, None


class _FusedLinear(torch.nn.Linear):
    def forward(self, x):
        if self.weight.grad is None:  # reference model: plain autograd
            return super().forward(x)
        return _InplaceWgrad.apply(x, self.weight, self.bias)


def _model(seed, fused=False):
    torch.manual_seed(seed)
    lin = _FusedLinear if fused else torch.nn.Linear
    return torch.nn.Sequential(lin(16, 64), torch.nn.Tanh(), torch.nn.Linear(64, 64),
                               torch.nn.Tanh(), lin(64, 4))


def _worker(rank, world, port, q, fused=False, native="1", wire="fp32"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DPA_NATIVE_REDUCER=native)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model = _model(seed=100 + rank, fused=fused)  # different init per rank: engine broadcasts rank 0
        eng = DDPEngine(model, bucket_cap_mb=0.01, first_bucket_mb=0.002,
                        reduce_dtype=torch.bfloat16 if wire == "bf16" else torch.float32)
        if native == "1":
            assert eng._native is not None, "native C++ reducer expected"
        torch.manual_seed(0)
        xs = torch.randn(2, world * 8, 16)  # 2 micro-batches, full batch split over ranks
        ys = torch.randn(2, world * 8, 4)
        eng.zero_grad()
        for mb in range(2):
            x = xs[mb, rank * 8:(rank + 1) * 8]
            y = ys[mb, rank * 8:(rank + 1) * 8]
            ctx = eng.no_sync() if mb == 0 else torch.enable_grad()
            with ctx:
                loss = torch.nn.functional.mse_loss(eng(x), y)
            loss.backward()
        # overlap: every bucket was launched from the grad-ready hooks DURING backward,
        # none is left for finalize() (also for weights accumulated in place by a fused op)
        launched = eng._native.next_bucket() if eng._native is not None else eng._next_launch
        eng.finalize()
        eng.average_gradients()
        # numpy copies travel by value (tensor storages are shared via fds, which
        # races with the worker exiting)
        q.put((rank, eng.space.param_flat.numpy().copy(), eng.space.grad_flat.numpy().copy(),
               len(eng.buckets), launched))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,fused,native,wire", [(2, False, "1", "fp32"), (4, False, "1", "fp32"),
                                                     (2, True, "1", "fp32"), (2, False, "0", "fp32"),
                                                     (2, True, "0", "fp32"), (2, False, "1", "bf16"),
                                                     (2, False, "0", "bf16")])
def test_ddp_engine_matches_single_process(world, fused, native, wire):
    """fused=True: some layers accumulate their weight grads in place and return None
    (like the split-K wgrad GEMM); buckets must still wait for those gradients."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = find_free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, fused, native, wire))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # reference: rank-0 init, full batch per micro-batch, mean over ranks of per-rank means
    model = _model(seed=100)
    torch.manual_seed(0)
    xs = torch.randn(2, world * 8, 16)
    ys = torch.randn(2, world * 8, 4)
    for mb in range(2):
        for r in range(world):
            loss = torch.nn.functional.mse_loss(model(xs[mb, r * 8:(r + 1) * 8]),
                                                ys[mb, r * 8:(r + 1) * 8]) / world
            loss.backward()
    space = FlatParamSpace(model.parameters())
    ref_grad = space.grad_flat
    for rank, pflat, gflat, nb, launched in res:
        pflat, gflat = torch.from_numpy(pflat), torch.from_numpy(gflat)
        assert nb > 1, "test must exercise several buckets"
        assert launched == nb, f"rank {rank}: only {launched}/{nb} buckets launched before finalize()"
        torch.testing.assert_close(pflat, space.param_flat)            # broadcast from rank 0
        tol = dict(rtol=1e-5, atol=1e-6) if wire == "fp32" else dict(rtol=2e-2, atol=2e-3)
        torch.testing.assert_close(gflat, ref_grad, **tol)


def test_bucket_plan_covers_buffer_in_order():
    model = _model(0)
    space = FlatParamSpace(model.parameters())
    buckets = plan_buckets(space, cap_mb=0.01, first_mb=0.002)
    assert buckets[0][0] == 0 and buckets[-1][1] == space.numel
    for (s0, e0, _), (s1, e1, _) in zip(buckets, buckets[1:]):
        assert e0 == s1 and s0 < e0
    # reverse registration order: the last layer's params come first
    assert buckets[0][2][0] is list(model.parameters())[-1]
    assert sum(len(b[2]) for b in buckets) == len(list(model.parameters()))


def test_flat_space_views_and_alignment():
    model = _model(0)
    before = [p.detach().clone() for p in model.parameters()]
    space = FlatParamSpace(model.parameters())
    for p, b in zip(model.parameters(), before):
        assert torch.equal(p, b)
        assert p.data_ptr() % 64 == 0
        assert p.grad is not None and p.grad.data_ptr() >= space.grad_flat.data_ptr()
    assert space.numel % 64 == 0
