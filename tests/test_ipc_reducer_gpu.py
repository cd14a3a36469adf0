"""The C++ BucketReducer's IPC data plane end to end: two processes sharing one HIP device
(gloo for the control plane and the handle exchange), ``DPA_IPC_ALLREDUCE=1``, so every
gradient bucket is all-reduced by csrc/ipc_allreduce.hip over the peer's IPC-mapped staging
buffer and flag words, launched from the autograd hooks on the reducer's comm stream while the
backward still runs (``BucketReducer::init_ipc_only``: the direct mode's stream and events
without an RCCL communicator, which refuses two ranks per GPU).  Over three steps the epochs
alternate the staging parity; the first bucket (output_down_proj's last Linear, first in the
model's gradient-ready layout: 0.13 MiB) takes the one-shot kernel and the 1 MiB buckets the
two-shot one.  The reduced gradient must equal the sum of both ranks' local
(no_sync) gradients.

Reference: /root/reference/utils/trainer.py:216-220 (DDP's bucketed all-reduce of the
backward's gradients)."""
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
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DPA_IPC_ALLREDUCE="1")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from distributed_pipeline_amd.models import build_model, create_gaussian_diffusion
        from distributed_pipeline_amd.ops.nn import RNG
        from distributed_pipeline_amd.parallel.ddp import DDPEngine
        torch.manual_seed(1234)
        model = build_model(**CFG).cuda()
        eng = DDPEngine(model, shadow_dtype=torch.bfloat16, bucket_cap_mb=1.0, first_bucket_mb=0.1)
        assert eng._native is not None and eng._native.ipc_ready(), "IPC data plane not set up"
        assert not eng._native.direct()  # no RCCL communicator: IPC only
        diff = create_gaussian_diffusion(steps=100)
        g = torch.Generator().manual_seed(7 + rank)  # different data per rank
        ids = torch.randint(1000, 3000, (3, 4, 128), generator=g).cuda()
        mask = torch.ones_like(ids)
        mask[..., :32] = 0
        t = torch.randint(0, 100, (3, 4), generator=g).cuda()

        def run(step, sync):
            eng.zero_grad()
            torch.manual_seed(99 + step)
            RNG.counter = 0
            with (torch.enable_grad() if sync else eng.no_sync()):
                terms = diff.training_losses(eng, None, t[step], dict(input_ids=ids[step], input_mask=mask[step]))
            terms["loss"].mean().backward()
            launched = eng._native.next_bucket()
            eng.finalize()
            return eng.space.grad_flat.clone(), launched

        out = []
        for step in range(3):
            local, _ = run(step, sync=False)
            reduced, launched = run(step, sync=True)
            torch.cuda.synchronize()
            out.append((local.cpu().numpy(), reduced.cpu().numpy(), launched))
        q.put((rank, out, len(eng.buckets), int(eng._native.ipc_error()),
               [b.end - b.start for b in eng.buckets]))
    finally:
        dist.destroy_process_group()


def test_bucket_reducer_ipc_plane_two_ranks_one_gpu():
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
    (_, out0, nb, err0, sizes), (_, out1, _, err1, _) = res
    assert err0 == 0 and err1 == 0, "IPC kernel timed out waiting for its peer"
    assert nb > 3
    assert min(sizes) * 4 <= 256 << 10 < max(sizes) * 4, sizes  # one-shot and two-shot buckets
    for step in range(3):
        l0, r0, launched = out0[step]
        l1, r1, _ = out1[step]
        l0, r0, l1, r1 = (torch.from_numpy(x) for x in (l0, r0, l1, r1))
        assert launched == nb, f"step {step}: {launched}/{nb} buckets launched from the hooks"
        assert l0.abs().sum() > 0 and not torch.equal(l0, l1)
        torch.testing.assert_close(r0, r1, rtol=0, atol=0)  # both ranks hold the same sum
        want = l0 + l1
        err = ((r0 - want).abs().max() / want.abs().max()).item()
        assert err < 1e-5, (step, err)
