"""The overlapped micro-batch schedule at world size 2 (two ranks on one HIP device, gloo
transport on device tensors).  ``_forward_backward_overlapped`` runs every forward under
``no_sync`` and arms the DDP engine right before the last backward
(``DDPEngine.arm_for_backward``); with weight-gradient deferral the held micro-batches'
GEMMs run on a third stream that the trainer joins before that backward.  At world 2 the
reduced gradient must equal the sum over ranks of each rank's purely local (never reduced)
sequential gradient, and the sequential DDP schedule must agree with both.

Reference schedule: /root/reference/utils/trainer.py:209-235 (``no_sync`` for every
micro-batch but the last, one all-reduce per optimizer step)."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from basic_utils.dist_util import find_free_port

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from basic_utils import logger
        from distributed_pipeline_amd.ops.nn import RNG, WGRAD_DEFER
        from utils.initialization import create_diffusion_from_config, create_model_from_config
        from utils.trainer import DiffusionTrainLoop

        logger.configure(dir=f"/tmp/dpa_overlap_w2_{rank}", format_strs=[])
        torch.manual_seed(0)
        model = create_model_from_config(model="diffuseq", precision="bf16", config_name="tiny",
                                         hidden_size=256, num_layers=2, num_heads=4, intermediate_size=1024,
                                         vocab_size=30522, seq_len=128, hidden_dim=128, hidden_t_dim=128,
                                         dropout=0.1).cuda()
        diffusion, sampler = create_diffusion_from_config(diffusion_steps=2000)
        g = torch.Generator().manual_seed(100 + rank)  # different data per rank
        B, L = 64, 128
        batch = {"input_ids": torch.randint(1000, 30522, (B, L), generator=g),
                 "input_mask": torch.cat([torch.zeros(B, 48, dtype=torch.long),
                                          torch.ones(B, L - 48, dtype=torch.long)], 1)}
        loop = DiffusionTrainLoop(diffusion=diffusion, schedule_sampler=sampler, model=model,
                                  data=iter([batch]), batch_size=B, microbatch=16, lr=1e-4,
                                  ema_rate="0.9999", log_interval=1, save_interval=10 ** 9,
                                  resume_checkpoint="", learning_steps=1,
                                  checkpoint_path=f"/tmp/dpa_overlap_w2_{rank}", ddp_engine="native",
                                  precision="bf16", exec_microbatch=-1, overlap_microbatches=True,
                                  device_prefetch=False, defer_wgrad=4)
        eng = loop.ddp_model
        assert loop.use_ddp and eng.world_size == world

        def run(overlap, defer, local):
            loop.overlap_microbatches = overlap
            loop.defer_wgrad = defer
            torch.manual_seed(7 + rank)
            RNG.counter = 0
            before = WGRAD_DEFER.stats["multi_launches"]
            if local:
                with eng.no_sync():  # nothing is reduced: this rank's own gradient
                    loop.forward_backward(batch)
                torch.cuda.synchronize()
                grad = eng.space.grad_flat.clone()
                dist.all_reduce(grad)  # the sum over ranks, taken by hand
            else:
                loop.forward_backward(batch)
                eng.finalize()
                torch.cuda.synchronize()
                grad = eng.space.grad_flat.clone()
            return grad, WGRAD_DEFER.stats["multi_launches"] - before

        ref, _ = run(False, 0, local=True)
        ref2, _ = run(False, 0, local=True)
        seq, _ = run(False, 0, local=False)
        ovl, nmulti = run(True, 4, local=False)
        q.put((rank, ref.cpu(), ref2.cpu(), seq.cpu(), ovl.cpu(), nmulti))
    finally:
        dist.destroy_process_group()


def test_overlapped_schedule_two_ranks_matches_local_sum():
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
    for rank, ref, ref2, seq, ovl, nmulti in res:
        assert nmulti > 0, "the deferred multi-segment weight gradients did not run"
        scale = ref.abs().max().item()
        assert scale > 0 and torch.isfinite(ovl).all()
        noise = (ref - ref2).abs().max().item()  # fp32 atomic column sums: run-to-run noise
        for name, g in (("sequential", seq), ("overlapped", ovl)):
            err = (g - ref).abs().max().item()
            # deferral changes the split-K summation order: fp32 rounding of the sum
            assert err <= max(4 * noise, 2e-5 * scale), (rank, name, err, noise, scale)
    # both ranks hold the same reduced gradient
    torch.testing.assert_close(res[0][4], res[1][4], rtol=0, atol=0)


def _graph_worker(rank, world, port, q):
    """Two ranks, HIP-graph mode: the captured step runs under ``no_sync`` and the engine
    reduces every bucket after each replay (``DDPEngine.reduce_all_now``)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from basic_utils import logger
        from distributed_pipeline_amd.ops.nn import RNG
        from utils.initialization import create_diffusion_from_config, create_model_from_config, seed_all
        from utils.trainer import DiffusionTrainLoop

        logger.configure(dir=f"/tmp/dpa_graph_w2_{rank}", format_strs=[])
        g = torch.Generator().manual_seed(200 + rank)  # different data per rank
        B, L, steps = 64, 128, 4
        batches = [{"input_ids": torch.randint(1000, 30522, (B, L), generator=g).cuda(),
                    "input_mask": torch.cat([torch.zeros(B, 48, dtype=torch.long),
                                             torch.ones(B, L - 48, dtype=torch.long)], 1).cuda()}
                   for _ in range(steps)]

        def run(graph):
            seed_all(0)
            RNG.counter = 0
            model = create_model_from_config(model="diffuseq", precision="bf16", config_name="tiny",
                                             hidden_size=256, num_layers=2, num_heads=4, intermediate_size=1024,
                                             vocab_size=30522, seq_len=128, hidden_dim=128, hidden_t_dim=128,
                                             dropout=0.1).cuda()
            diffusion, sampler = create_diffusion_from_config(diffusion_steps=2000)
            loop = DiffusionTrainLoop(diffusion=diffusion, schedule_sampler=sampler, model=model,
                                      data=iter(batches), batch_size=B, microbatch=16, lr=1e-4,
                                      ema_rate="0.9999", log_interval=1, save_interval=10 ** 9,
                                      resume_checkpoint="", learning_steps=steps,
                                      checkpoint_path=f"/tmp/dpa_graph_w2_{rank}", ddp_engine="native",
                                      precision="bf16", exec_microbatch=-1, overlap_microbatches=True,
                                      device_prefetch=False, defer_wgrad=4, cuda_graph=graph)
            assert loop.use_ddp
            torch.manual_seed(7 + rank)
            for b in batches:
                loop.run_step(b)
                logger.dumpkvs()
            torch.cuda.synchronize()
            return loop._graph is not None, loop.ddp_model.space.param_flat.clone().cpu()

        q.put((rank, run(False), run(False), run(True)))
    finally:
        dist.destroy_process_group()


def test_graph_mode_two_ranks_matches_eager():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = find_free_port()
    procs = [ctx.Process(target=_graph_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, (cap0, p0), (_, pa), (cap1, p1) in res:
        assert not cap0 and cap1, "graph mode did not capture"
        noise = (p0 - pa).abs().max().item()
        err = (p0 - p1).abs().max().item()
        assert err <= max(4 * noise, 2.5e-4), (rank, err, noise)
    # reduced gradients: every rank took the same optimizer steps
    torch.testing.assert_close(res[0][3][1], res[1][3][1], rtol=0, atol=0)
