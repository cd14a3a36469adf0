"""Simulated W > 1 data plane (parallel/ddp.py ``enable_sim_comm``, csrc/comm_sim.hip, the C++
reducer's sim mode): a one-GPU projection of the bucket all-reduce overlap.

* It changes no value: the gradients and the updated weights of a step on the simulated data
  plane equal those of the plain world-1 step (the stand-in kernel writes back what it reads) up
  to the run-to-run order of the fp32 atomic bias-column sums (as tests/test_wt_shadow_gpu.py).
* The reducer's device-side timeline sees every bucket (ready -> start -> end) and the model
  time the link model gives them.
* The fused schedule hides everything but the last bucket: the exposed tail after the backward's
  last kernel is at most the last bucket's simulated time plus 1 ms."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _loop(B=64, layers=4):
    from basic_utils import logger
    from distributed_pipeline_amd.ops.nn import RNG
    from utils.initialization import create_diffusion_from_config, create_model_from_config, seed_all
    from utils.trainer import DiffusionTrainLoop

    logger.configure(dir="/tmp/dpa_sim_test", format_strs=[])
    seed_all(0)
    RNG.counter = 0
    model = create_model_from_config(model="diffuseq", precision="bf16", config_name="tiny",
                                     hidden_size=768, num_layers=layers, num_heads=12, intermediate_size=3072,
                                     vocab_size=30522, seq_len=128, hidden_dim=128, hidden_t_dim=128,
                                     dropout=0.1).cuda()
    diffusion, sampler = create_diffusion_from_config(diffusion_steps=2000)
    g = torch.Generator().manual_seed(1)
    L = 128
    batch = {"input_ids": torch.randint(1000, 30522, (B, L), generator=g),
             "input_mask": torch.cat([torch.zeros(B, 48, dtype=torch.long),
                                      torch.ones(B, L - 48, dtype=torch.long)], 1)}
    loop = DiffusionTrainLoop(diffusion=diffusion, schedule_sampler=sampler, model=model,
                              data=iter([batch] * 100), batch_size=B, microbatch=B, lr=1e-3,
                              ema_rate="0.9999", log_interval=10 ** 6, save_interval=10 ** 9, resume_checkpoint="",
                              learning_steps=100, checkpoint_path="/tmp/dpa_sim_test", ddp_engine="native",
                              precision="bf16", device_prefetch=False, bucket_cap_mb=8, first_bucket_mb=2)
    return loop, batch


def _step(loop, batch, seed):
    torch.manual_seed(seed)
    loop.run_step(batch)
    torch.cuda.synchronize()


def test_sim_comm_changes_no_value():
    loop, batch = _loop()
    _step(loop, batch, 5)
    p_plain = loop.ddp_model.space.param_flat.clone()
    g_plain = loop.ddp_model.space.grad_flat.clone()

    loop2, _ = _loop()
    eng = loop2.ddp_model
    info = eng.enable_sim_comm(8, 153.0, cus=32, lat_us=10.0)
    loop2.use_ddp = True
    assert info["world"] == 8 and len(info["bucket_mb"]) >= 3
    _step(loop2, batch, 5)
    st = eng.sim_stats()
    assert st["steps"] == 1
    # every bucket ran for at least its link-model time (the workgroups spin on the clock)
    assert st["bucket_busy_ms"] >= 0.95 * st["model_ms_per_step"] > 0
    g = eng.space.grad_flat
    scale = g_plain.abs().max().item()
    assert (g - g_plain).abs().max().item() <= 1e-5 * scale
    assert (eng.space.param_flat - p_plain).abs().max().item() <= 1e-5
    eng.disable_sim_comm()


def test_sim_comm_fused_tail_is_the_last_bucket():
    loop, batch = _loop(B=256, layers=6)
    eng = loop.ddp_model
    eng.enable_sim_comm(8, 153.0, cus=64, lat_us=10.0)
    loop.use_ddp = True
    for i in range(2):
        _step(loop, batch, 11 + i)
    eng.sim_stats(reset=True)
    for i in range(3):
        _step(loop, batch, 21 + i)
    st = eng.sim_stats()
    print(st)
    print("timeline [ready, start, end] ms; last row = backward end:", eng.sim_timeline())
    assert st["steps"] == 3
    assert st["exposed_tail_ms"] <= st["last_bucket_model_ms"] + 1.0, st
    # and the bucket stand-ins did not all wait for the end of the backward
    assert st["comm_span_ms"] > st["exposed_tail_ms"], st
    eng.disable_sim_comm()
