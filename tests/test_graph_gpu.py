"""HIP-graph mode of the trainer (utils/trainer.py ``cuda_graph``): after two eager steps
the step's whole forward/backward - the overlapped 4-chunk reference schedule, three HIP
streams, weight-gradient deferral - is captured once and replayed.  The replays must draw
exactly the randomness the eager steps would have drawn (device-side Philox offset base +
torch's graph-safe generator), so the gradients, losses and parameters of replayed steps
equal an all-eager run's up to the fp32 atomic column-sum noise, and the logged losses come
from each replay's own outputs."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(graph, steps=4):
    from basic_utils import logger
    from distributed_pipeline_amd.ops.nn import RNG
    from utils.initialization import create_diffusion_from_config, create_model_from_config, seed_all
    from utils.trainer import DiffusionTrainLoop

    logger.configure(dir="/tmp/dpa_graph_test", format_strs=[])
    seed_all(0)
    RNG.counter = 0
    model = create_model_from_config(model="diffuseq", precision="bf16", config_name="tiny",
                                     hidden_size=256, num_layers=2, num_heads=4, intermediate_size=1024,
                                     vocab_size=30522, seq_len=128, hidden_dim=128, hidden_t_dim=128,
                                     dropout=0.1).cuda()
    diffusion, sampler = create_diffusion_from_config(diffusion_steps=2000)
    g = torch.Generator().manual_seed(3)
    B, L = 64, 128
    batches = [{"input_ids": torch.randint(1000, 30522, (B, L), generator=g).cuda(),
                "input_mask": torch.cat([torch.zeros(B, 48, dtype=torch.long),
                                         torch.ones(B, L - 48, dtype=torch.long)], 1).cuda()}
               for _ in range(steps)]
    loop = DiffusionTrainLoop(diffusion=diffusion, schedule_sampler=sampler, model=model,
                              data=iter(batches), batch_size=B, microbatch=16, lr=1e-4,
                              ema_rate="0.9999", log_interval=1, save_interval=10 ** 9, resume_checkpoint="",
                              learning_steps=steps, checkpoint_path="/tmp/dpa_graph_test", ddp_engine="native",
                              precision="bf16", exec_microbatch=-1, overlap_microbatches=True,
                              device_prefetch=False, defer_wgrad=4, cuda_graph=graph)
    torch.manual_seed(7)
    out = []
    for b in batches:
        loop.run_step(b)
        loss = logger.dumpkvs()["loss"]
        torch.cuda.synchronize()
        out.append((loop.ddp_model.space.grad_flat.clone(), loop.ddp_model.space.param_flat.clone(), loss))
    return loop, out


def test_graph_replay_matches_eager():
    from distributed_pipeline_amd.ops.nn import RNG
    _, ref = _run(False)
    _, ref2 = _run(False)
    loop, got = _run(True)
    assert loop._graph is not None, "the step was not captured"
    assert RNG._dev_base == 0  # reset after every replay
    for k, ((g0, p0, l0), (ga, pa, la), (g1, p1, l1)) in enumerate(zip(ref, ref2, got)):
        scale = g0.abs().max().item()
        noise = (g0 - ga).abs().max().item()
        err = (g0 - g1).abs().max().item()
        # deferral / column sums: fp32 atomic rounding between runs, nothing more
        assert err <= max(4 * noise, 2e-5 * scale), (k, err, noise, scale)
        assert (p0 - p1).abs().max().item() <= max(4 * (p0 - pa).abs().max().item(), 2.5e-4), k
        assert abs(l0 - l1) <= 1e-4 * abs(l0), (k, l0, l1)
    # the replayed steps drew new noise / dropout / timesteps: their losses differ per step
    assert got[2][2] != got[3][2]


def _run_base(graph, steps=5):
    """DiffuSeq-base widths (768 / 3072, 12 heads; 2 layers) with the 64-sample chunks of the
    reference schedule: the ffn-in forward has 384 output tiles against the overlap's 128-CU
    forward grid cap, so the persistent GEMMs claim tiles from the dynamic queues."""
    from basic_utils import logger
    from distributed_pipeline_amd.ops.nn import RNG
    from utils.initialization import create_diffusion_from_config, create_model_from_config, seed_all
    from utils.trainer import DiffusionTrainLoop

    logger.configure(dir="/tmp/dpa_graph_test_base", format_strs=[])
    seed_all(0)
    RNG.counter = 0
    model = create_model_from_config(model="diffuseq", precision="bf16", config_name="tiny",
                                     hidden_size=768, num_layers=2, num_heads=12, intermediate_size=3072,
                                     vocab_size=30522, seq_len=128, hidden_dim=128, hidden_t_dim=128,
                                     dropout=0.1).cuda()
    diffusion, sampler = create_diffusion_from_config(diffusion_steps=2000)
    g = torch.Generator().manual_seed(5)
    B, L = 256, 128
    batches = [{"input_ids": torch.randint(1000, 30522, (B, L), generator=g).cuda(),
                "input_mask": torch.cat([torch.zeros(B, 48, dtype=torch.long),
                                         torch.ones(B, L - 48, dtype=torch.long)], 1).cuda()}
               for _ in range(steps)]
    loop = DiffusionTrainLoop(diffusion=diffusion, schedule_sampler=sampler, model=model,
                              data=iter(batches), batch_size=B, microbatch=64, lr=1e-4,
                              ema_rate="0.9999", log_interval=1, save_interval=10 ** 9, resume_checkpoint="",
                              learning_steps=steps, checkpoint_path="/tmp/dpa_graph_test_base",
                              ddp_engine="native", precision="bf16", exec_microbatch=-1,
                              overlap_microbatches=True, device_prefetch=False, defer_wgrad=4, cuda_graph=graph)
    torch.manual_seed(7)
    out = []
    for b in batches:
        loop.run_step(b)
        logger.dumpkvs()
        torch.cuda.synchronize()
        out.append((loop.ddp_model.space.grad_flat.clone(), loop.ddp_model.space.param_flat.clone()))
    return loop, out


def test_graph_replay_with_dynamic_tile_queues_matches_eager():
    """The persistent GEMMs' per-XCD tile queues (on for world > 1) under HIP-graph replay:
    the counters' addresses are baked into the graph, so every launch must leave them zeroed
    (the kernel's last workgroup per queue resets them).  Stale counters would end workgroups
    early and leave output tiles unwritten: the replayed steps' gradients would be wrong."""
    from distributed_pipeline_amd.ops._ext import get_ext
    ext = get_ext(required=True)
    ext.set_gemmp_dynamic(True)
    try:
        _, ref = _run_base(False)
        _, ref2 = _run_base(False)
        loop, got = _run_base(True)
    finally:
        ext.set_gemmp_dynamic(False)
    assert loop._graph is not None, "the step was not captured"
    for k, ((g0, p0), (ga, pa), (g1, p1)) in enumerate(zip(ref, ref2, got)):
        scale = g0.abs().max().item()
        noise = (g0 - ga).abs().max().item()
        err = (g0 - g1).abs().max().item()
        assert err <= max(4 * noise, 2e-5 * scale), (k, err, noise, scale)
        assert (p0 - p1).abs().max().item() <= max(4 * (p0 - pa).abs().max().item(), 2.5e-4), k
