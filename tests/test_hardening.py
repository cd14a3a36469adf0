"""Multi-rank hardening of the DDP engine and trainer (CPU / gloo, world 2).

* unused parameters: the first armed step names them (warning, or an error with
  DPA_DDP_UNUSED=error) instead of silently losing the backward overlap;
* rank-agreed executed micro-batch: an out-of-memory error on ONE rank during the
  auto-sized first step must not desynchronise the collectives - every rank settles
  on the MIN size through a collective-free probe, and the gradients still equal the
  reference's sum over micro-batches;
* the fused AdamW's device skip flag (set by a failed IPC all-reduce) refuses the step;
* in-process NUMA binding helpers (sysfs parsing, per-rank CPU split).
"""
import os
import warnings

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from basic_utils import dist_util
from basic_utils.dist_util import find_free_port


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)


class _Partly(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(8, 8)
        self.unused = torch.nn.Linear(8, 8)  # never called
        self.b = torch.nn.Linear(8, 2)

    def forward(self, x):
        return self.b(torch.tanh(self.a(x)))


def _unused_worker(rank, world, port, q, mode):
    _init(rank, world, port)
    os.environ["DPA_DDP_UNUSED"] = mode
    try:
        from distributed_pipeline_amd.parallel.ddp import DDPEngine
        torch.manual_seed(0)
        eng = DDPEngine(_Partly(), bucket_cap_mb=0.0005, first_bucket_mb=0.0002)
        msgs, err = [], None
        for step in range(2):
            eng.zero_grad()
            loss = eng(torch.randn(4, 8)).square().mean()
            loss.backward()
            with warnings.catch_warnings(record=True) as w:
                warnings.simplefilter("always")
                try:
                    eng.finalize()
                except RuntimeError as e:  # DPA_DDP_UNUSED=error
                    err = str(e)
                    break
            msgs += [str(x.message) for x in w if issubclass(x.category, RuntimeWarning)]
        q.put((rank, msgs, err))
    finally:
        dist.destroy_process_group()


def _run(fn, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = find_free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda t: t[0])


def test_unused_parameter_is_named_once():
    for rank, msgs, err in _run(_unused_worker, 2, "warn"):
        assert err is None
        assert len(msgs) == 1, msgs  # first armed step only
        assert "unused.weight" in msgs[0] and "unused.bias" in msgs[0]
        assert "a.weight" not in msgs[0]


def test_unused_parameter_error_mode():
    for rank, msgs, err in _run(_unused_worker, 2, "error"):
        assert err is not None and "unused.weight" in err


# --------------------------------------------------------------------------- #
# rank-agreed executed micro-batch


def _settle_worker(rank, world, port, q):
    _init(rank, world, port)
    try:
        from basic_utils import logger
        from utils.trainer import TrainLoop

        logger.configure(dir=None, format_strs=[])
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(6, 16), torch.nn.Tanh(), torch.nn.Linear(16, 1))
        limit = 4 if rank == 0 else 16  # rank 0 "runs out of memory" above 4 samples

        class Loop(TrainLoop):
            supports_microbatch_fusion = True

            def compute_losses(self, mb):
                n = mb["x"].shape[0]
                if n > limit and not self._exec_settled:
                    raise torch.cuda.OutOfMemoryError(f"fake OOM at {n} samples")
                if self._exec_settled:
                    self.chunks.append(n)
                out = self.ddp_model(mb["x"]).squeeze(-1)
                return {"loss": (out - mb["y"]) ** 2}

            def backward_from_losses(self, losses):
                (losses["loss"] * self.loss_scale).mean().backward()

        g = torch.Generator().manual_seed(1 + rank)
        batch = {"x": torch.randn(8, 6, generator=g), "y": torch.randn(8, generator=g)}
        loop = Loop(model=model, data=iter([batch] * 4), batch_size=8, microbatch=2, lr=1e-3,
                    ema_rate="0.9", log_interval=10, save_interval=10 ** 9, resume_checkpoint="",
                    learning_steps=0, checkpoint_path="", ddp_engine="native", precision="fp32",
                    exec_microbatch=0)
        loop.chunks = []
        loop.exec_microbatch = 8          # what auto mode picks on a GPU (the whole batch)
        loop.forward_backward(batch)
        loop.ddp_model.finalize()
        grads = loop.ddp_model.space.grad_flat.clone()
        # reference: 4 micro-batches of 2, summed, then the rank sum (no averaging yet)
        ref = torch.zeros_like(grads)
        for p in model.parameters():
            p.grad = None
        space = loop.ddp_model.space
        for i in range(0, 8, 2):
            out = model(batch["x"][i:i + 2]).squeeze(-1)
            ((out - batch["y"][i:i + 2]) ** 2).mean().backward()
        for p in model.parameters():
            o, e = space.range_of(p)
            ref[o:e] = p.grad.reshape(-1)
        dist.all_reduce(ref)
        q.put((rank, loop.exec_microbatch, list(loop.chunks), (grads - ref).abs().max().item()))
    finally:
        dist.destroy_process_group()


def test_exec_microbatch_rank_agreed_after_one_rank_ooms():
    res = _run(_settle_worker, 2)
    for rank, emb, chunks, err in res:
        assert emb == 4, (rank, emb)           # MIN over ranks of what fit
        assert chunks == [4, 4], chunks        # both ranks run the same schedule
        assert err < 1e-5, err                 # gradient = reference sum over micro-batches


# --------------------------------------------------------------------------- #


def test_adamw_skip_flag_refuses_step():
    from distributed_pipeline_amd.ops import optim as fused
    p = torch.randn(64)
    g = torch.randn(64)
    m, v = torch.zeros(64), torch.zeros(64)
    e = p.clone()
    p0 = p.clone()
    fused.adamw_ema_(p, g, m, v, lr=0.1, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, step=1,
                     emas=[e], ema_rates=[0.5], skip=torch.ones(1, dtype=torch.int32))
    assert torch.equal(p, p0) and torch.equal(m, torch.zeros(64)) and torch.equal(e, p0)
    fused.adamw_ema_(p, g, m, v, lr=0.1, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0, step=1,
                     emas=[e], ema_rates=[0.5], skip=torch.zeros(1, dtype=torch.int32))
    assert not torch.equal(p, p0)


def test_numa_helpers(tmp_path):
    assert dist_util._parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    dev = tmp_path / "bus/pci/devices/0000:72:00.0"
    dev.mkdir(parents=True)
    (dev / "numa_node").write_text("1\n")
    node = tmp_path / "devices/system/node/node1"
    node.mkdir(parents=True)
    (node / "cpulist").write_text("48-95,144-191\n")
    cpus = dist_util.gpu_numa_cpus("0000:72:00.0", str(tmp_path))
    assert cpus == set(range(48, 96)) | set(range(144, 192))
    assert dist_util.gpu_numa_cpus("0000:99:00.0", str(tmp_path)) == set()
    (dev / "numa_node").write_text("-1\n")
    assert dist_util.gpu_numa_cpus("0000:72:00.0", str(tmp_path)) == set()
    parts = [dist_util.split_cpus(set(range(10)), i, 4) for i in range(4)]
    assert sorted(len(x) for x in parts) == [2, 2, 3, 3]
    assert set().union(*parts) == set(range(10))
    assert dist_util.bind_cpus_to_gpu(0, mode="off") is None


def test_exec_microbatch_shrinks_for_hbm_headroom(tmp_path):
    """One rank, auto executed micro-batch: a step that fits but leaves less HBM than the
    reserve at its peak (``TrainLoop._hbm_headroom_ok``) is redone one chunk smaller - the
    gradient of the redone step equals the reference sum of micro-batch gradients (nothing of
    the first try remains) and the logged loss is that of the redone step only."""
    from basic_utils import logger
    from utils.trainer import TrainLoop

    logger.configure(dir=str(tmp_path), format_strs=[])
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(6, 16), torch.nn.Tanh(), torch.nn.Linear(16, 1))

    class Loop(TrainLoop):
        supports_microbatch_fusion = True

        def compute_losses(self, mb):
            self.chunks.append(mb["x"].shape[0])
            out = self.ddp_model(mb["x"]).squeeze(-1)
            return {"loss": (out - mb["y"]) ** 2}

        def backward_from_losses(self, losses):
            (losses["loss"] * self.loss_scale).mean().backward()

        def _hbm_headroom_ok(self):  # "too little left" above 4 samples per chunk
            return self.exec_microbatch <= 4

    g = torch.Generator().manual_seed(1)
    batch = {"x": torch.randn(8, 6, generator=g), "y": torch.randn(8, generator=g)}
    loop = Loop(model=model, data=iter([batch] * 4), batch_size=8, microbatch=2, lr=1e-3,
                ema_rate="0.9", log_interval=10, save_interval=10 ** 9, resume_checkpoint="",
                learning_steps=0, checkpoint_path="", ddp_engine="native", precision="fp32",
                exec_microbatch=0)
    loop.chunks = []
    loop.exec_microbatch = 8
    loop.forward_backward(batch)
    # 8 (one chunk) fits but is refused for headroom; the next size is two balanced chunks of 4
    assert loop._exec_settled and loop.exec_microbatch == 4
    assert loop.chunks[-2:] == [4, 4]
    grads = loop.ddp_model.space.grad_flat.clone()
    ref = torch.zeros_like(grads)
    for p in model.parameters():
        p.grad = None
    for i in range(0, 8, 2):
        out = model(batch["x"][i:i + 2]).squeeze(-1)
        ((out - batch["y"][i:i + 2]) ** 2).mean().backward()
    space = loop.ddp_model.space
    for p in model.parameters():
        o, e = space.range_of(p)
        ref[o:e] = p.grad.reshape(-1)
    torch.testing.assert_close(grads, ref, rtol=1e-5, atol=1e-6)
