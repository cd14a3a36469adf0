"""ZeRO-1 sharded optimizer (parallel/zero.py) on CPU/gloo, world 2 and 4.

Three clipped AdamW steps with two EMA rates through the sharded engine must leave
parameters, AdamW moments (in torch.optim.AdamW state_dict format) and EMAs equal to
the unsharded engine's; the sharded state must round-trip through state_dict /
load_state_dict and hold 1/world of the optimizer state per rank."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from basic_utils.dist_util import find_free_port


def _model(seed):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.Tanh(), torch.nn.Linear(64, 64),
                               torch.nn.Tanh(), torch.nn.Linear(64, 4))


def _run(rank, world, sharded):
    from distributed_pipeline_amd.parallel.ddp import DDPEngine
    from distributed_pipeline_amd.parallel.optimizer import FusedAdamW
    from distributed_pipeline_amd.parallel.zero import ZeroFusedAdamW
    model = _model(100 + rank)  # different init per rank: the engine broadcasts rank 0
    eng = DDPEngine(model, bucket_cap_mb=0.01, first_bucket_mb=0.002, shard_optimizer=sharded)
    kw = dict(lr=1e-2, weight_decay=0.01, ema_rates=(0.9, 0.99))
    opt = ZeroFusedAdamW(eng, **kw) if sharded else FusedAdamW(eng.space, **kw)
    g = torch.Generator().manual_seed(0)
    for _ in range(3):
        x = torch.randn(world * 8, 16, generator=g)
        y = torch.randn(world * 8, 4, generator=g)
        eng.zero_grad()
        loss = torch.nn.functional.mse_loss(eng(x[rank * 8:(rank + 1) * 8]), y[rank * 8:(rank + 1) * 8])
        loss.backward()
        eng.finalize()
        norm = opt.compute_grad_norm(grad_scale=1.0 / world, max_norm=0.5)
        opt.step(grad_scale=1.0 / world, clip=norm)
    params = torch.cat([v.reshape(-1) for v in eng.space.views(eng.space.param_flat)])
    sd = opt.state_dict()
    moments = torch.cat([torch.cat([s["exp_avg"].reshape(-1), s["exp_avg_sq"].reshape(-1)])
                         for _, s in sorted(sd["state"].items())])
    emas = torch.cat([torch.cat([p.reshape(-1) for p in opt.ema_params(i)]) for i in range(2)])
    extra = {}
    if sharded:
        extra["state_numel"] = opt.exp_avg.numel()
        extra["full_numel"] = eng.space.numel
        opt2 = ZeroFusedAdamW(eng, **kw)
        opt2.load_state_dict(sd)
        extra["roundtrip"] = bool(torch.equal(opt2.exp_avg, opt.exp_avg)
                                  and torch.equal(opt2.exp_avg_sq, opt.exp_avg_sq)
                                  and opt2.step_count == opt.step_count)
        before = [e.clone() for e in opt.ema_flats]
        opt.load_ema(0, opt.ema_params(0), broadcast=eng.broadcast_flat)
        extra["ema_reload"] = bool(torch.equal(before[0], opt.ema_flats[0]))
    return params.numpy().copy(), moments.numpy().copy(), emas.numpy().copy(), float(norm[0]), extra


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, _run(rank, world, False), _run(rank, world, True)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_zero1_matches_unsharded_engine(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = find_free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref0 = None
    for rank, ref, zr in res:
        for a, b in zip(ref[:3], zr[:3]):
            torch.testing.assert_close(torch.from_numpy(b), torch.from_numpy(a), rtol=1e-5, atol=1e-6)
        assert abs(ref[3] - zr[3]) <= 1e-5 * max(1.0, abs(ref[3]))
        extra = zr[4]
        assert extra["roundtrip"] and extra["ema_reload"]
        assert extra["state_numel"] * world == extra["full_numel"]   # 1/world of the state
        if ref0 is None:
            ref0 = ref[0]
        torch.testing.assert_close(torch.from_numpy(ref[0]), torch.from_numpy(ref0))  # replicas agree


def _bf16_model(seed):
    from distributed_pipeline_amd.models.layers import Linear
    torch.manual_seed(seed)
    return torch.nn.Sequential(Linear(16, 64, act="tanh"), Linear(64, 64, act="tanh"), Linear(64, 4))


def _run_bf16(rank, world, sharded):
    """bf16 compute through the shadow: the sharded engine gathers only the bf16 shadow
    (the fp32 master outside this rank's chunks is poisoned with NaN and must never be
    read by the forward) and materialises the master on demand."""
    from distributed_pipeline_amd.parallel.ddp import DDPEngine
    from distributed_pipeline_amd.parallel.optimizer import FusedAdamW
    from distributed_pipeline_amd.parallel.zero import ZeroFusedAdamW
    os.environ["DPA_ZERO_POISON"] = "1" if sharded else "0"
    model = _bf16_model(100 + rank)
    eng = DDPEngine(model, bucket_cap_mb=0.004, first_bucket_mb=0.001, shard_optimizer=sharded,
                    shadow_dtype=torch.bfloat16)
    kw = dict(lr=1e-2, weight_decay=0.01, ema_rates=(0.9,))
    opt = ZeroFusedAdamW(eng, **kw) if sharded else FusedAdamW(eng.space, **kw)
    g = torch.Generator().manual_seed(0)
    losses = []
    for _ in range(3):
        x = torch.randn(world * 8, 16, generator=g).bfloat16()
        y = torch.randn(world * 8, 4, generator=g)
        eng.zero_grad()
        out = eng(x[rank * 8:(rank + 1) * 8]).float()
        loss = torch.nn.functional.mse_loss(out, y[rank * 8:(rank + 1) * 8])
        loss.backward()
        eng.finalize()
        norm = opt.compute_grad_norm(grad_scale=1.0 / world)
        opt.step(grad_scale=1.0 / world)  # the sharded optimizer ends with gather_params()
        losses.append(float(loss.detach()))
    stale = bool(torch.isnan(eng.space.param_flat).any()) if sharded else False
    eng.materialize_master()
    flat = lambda f: torch.cat([v.reshape(-1) for v in eng.space.views(f)]).float().numpy().copy()  # noqa: E731
    return flat(eng.space.param_flat), flat(eng.space.shadow_flat), losses, stale, float(norm[0])


def _worker_bf16(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, _run_bf16(rank, world, False), _run_bf16(rank, world, True)))
    finally:
        dist.destroy_process_group()


def test_zero1_bf16_shadow_gather_matches_unsharded():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = find_free_port()
    procs = [ctx.Process(target=_worker_bf16, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _rank, ref, shd in res:
        assert shd[3], "the poisoned stale master should still hold NaN before materialize"
        assert ref[2] == shd[2]                                # identical losses: forward read shadows only
        assert (ref[0] == shd[0]).all()                        # master after materialize_master
        assert (ref[1] == shd[1]).all()                        # gathered bf16 shadow
