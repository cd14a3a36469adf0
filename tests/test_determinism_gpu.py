"""Bitwise-reproducible training steps: no reduction of the DiffuSeq step sums in arrival order.
The embedding gradient is a stable-sorted segment sum (csrc/sort.hip, csrc/diffusion.hip), the
tied head's weight gradient sums its token splits in order (csrc/xent.hip), the t == 0 samples'
embedding term rides on d x_start into that sorted sum, the LayerNorm / bias / attention-bias
column sums are two ordered passes (csrc/norm.hip, csrc/attention*.hip), the split-K weight
gradients merge through an ordered reduce (csrc/gemm256.hip) and the deferred ones run one writer
per tile (wgrad_group_kernel).  Two runs from the same seed must give the same bits - gradients,
parameters and logged losses - in the fused whole-batch step and in the overlapped micro-batch
schedule with weight-gradient deferral."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(exec_microbatch, overlap, defer, steps=2):
    from basic_utils import logger
    from distributed_pipeline_amd.ops.nn import RNG
    from utils.initialization import create_diffusion_from_config, create_model_from_config, seed_all
    from utils.trainer import DiffusionTrainLoop

    logger.configure(dir="/tmp/dpa_determinism_test", format_strs=[])
    seed_all(0)
    RNG.counter = 0
    model = create_model_from_config(model="diffuseq", precision="bf16", config_name="tiny",
                                     hidden_size=256, num_layers=2, num_heads=4, intermediate_size=1024,
                                     vocab_size=30522, seq_len=128, hidden_dim=128, hidden_t_dim=128,
                                     dropout=0.1).cuda()
    diffusion, sampler = create_diffusion_from_config(diffusion_steps=2000)
    g = torch.Generator().manual_seed(1)
    B, L = 256, 128
    ids = torch.randint(1000, 30522, (B, L), generator=g)
    ids[:, 100:] = 0  # padding: long runs of one id in the embedding gradient
    batch = {"input_ids": ids, "input_mask": torch.cat([torch.zeros(B, 48, dtype=torch.long),
                                                       torch.ones(B, L - 48, dtype=torch.long)], 1)}
    loop = DiffusionTrainLoop(diffusion=diffusion, schedule_sampler=sampler, model=model,
                              data=iter([batch] * (steps + 1)), batch_size=B, microbatch=64, lr=1e-4,
                              ema_rate="0.9999", log_interval=1, save_interval=10 ** 9, resume_checkpoint="",
                              learning_steps=steps, checkpoint_path="/tmp/dpa_determinism_test",
                              ddp_engine="native", precision="bf16", exec_microbatch=exec_microbatch,
                              overlap_microbatches=overlap, device_prefetch=False, defer_wgrad=defer)
    torch.manual_seed(7)
    losses = []
    for _ in range(steps):
        loop.run_step(batch)
        losses.append(logger.dumpkvs()["loss"])
    torch.cuda.synchronize()
    sp = loop.ddp_model.space
    return sp.grad_flat.clone(), sp.param_flat.clone(), losses, sp


def _first_diff(sp, a, b):
    """(layout index, shape) of every parameter whose slice differs - the failing reduction's site"""
    out = []
    for i, p in enumerate(sp.layout):
        off, n = sp.offsets[id(p)], p.numel()
        if not torch.equal(a[off:off + n], b[off:off + n]):
            out.append((i, tuple(p.shape)))
    return out


@pytest.mark.parametrize("exec_microbatch,overlap,defer", [(0, False, 0), (-1, True, 2)],
                         ids=["fused", "overlapped-deferred"])
def test_training_steps_bitwise_reproducible(exec_microbatch, overlap, defer):
    g0, p0, l0, sp = _run(exec_microbatch, overlap, defer)
    g1, p1, l1, _ = _run(exec_microbatch, overlap, defer)
    assert torch.equal(g0, g1), _first_diff(sp, g0, g1)
    assert torch.equal(p0, p1), _first_diff(sp, p0, p1)
    assert l0 == l1


def _run_gpt2(steps=2):
    from basic_utils import logger
    from distributed_pipeline_amd.ops.nn import RNG
    from utils.initialization import create_model_from_config, seed_all
    from utils.trainer import LMTrainLoop

    logger.configure(dir="/tmp/dpa_determinism_gpt2", format_strs=[])
    seed_all(0)
    RNG.counter = 0
    model = create_model_from_config(model="gpt2", precision="bf16", config_name="tiny", hidden_size=256,
                                     num_layers=2, num_heads=4, vocab_size=50257, seq_len=256,
                                     dropout=0.1).cuda()
    g = torch.Generator().manual_seed(2)
    ids = torch.randint(0, 50257, (16, 256), generator=g)
    batch = {"input_ids": ids, "labels": ids.clone()}
    loop = LMTrainLoop(model=model, data=iter([batch] * (steps + 1)), batch_size=16, microbatch=8, lr=1e-4,
                       ema_rate="0.9999", log_interval=1, save_interval=10 ** 9, resume_checkpoint="",
                       learning_steps=steps, checkpoint_path="/tmp/dpa_determinism_gpt2", ddp_engine="native",
                       precision="bf16", exec_microbatch=0, device_prefetch=False)
    torch.manual_seed(7)
    losses = []
    for _ in range(steps):
        loop.run_step(batch)
        losses.append(logger.dumpkvs()["loss"])
    torch.cuda.synchronize()
    sp = loop.ddp_model.space
    return sp.grad_flat.clone(), sp.param_flat.clone(), losses, sp


def test_gpt2_training_steps_bitwise_reproducible():
    """The causal-LM path too: general attention kernels (ordered qkv-bias sums), tied wte/LM head
    (sorted embedding gradient, split-K head weight gradient with an ordered merge)."""
    g0, p0, l0, sp = _run_gpt2()
    g1, p1, l1, _ = _run_gpt2()
    assert torch.equal(g0, g1), _first_diff(sp, g0, g1)
    assert torch.equal(p0, p1), _first_diff(sp, p0, p1)
    assert l0 == l1


def _resume_loop(ckdir, batch):
    from utils.initialization import create_diffusion_from_config, create_model_from_config, seed_all
    from utils.trainer import DiffusionTrainLoop
    seed_all(0)
    model = create_model_from_config(model="diffuseq", precision="bf16", config_name="tiny",
                                     hidden_size=256, num_layers=2, num_heads=4, intermediate_size=1024,
                                     vocab_size=30522, seq_len=128, hidden_dim=128, hidden_t_dim=128,
                                     dropout=0.1).cuda()
    diffusion, sampler = create_diffusion_from_config(diffusion_steps=2000)
    # learning_steps=0: constant lr (the anneal reads step + resume_step, which a resumed run
    # re-bases - reference semantics); every other piece of state must round-trip exactly
    return DiffusionTrainLoop(diffusion=diffusion, schedule_sampler=sampler, model=model,
                              data=iter([batch] * 8), batch_size=64, microbatch=64, lr=1e-3,
                              ema_rate="0.9,0.999", log_interval=1, save_interval=10 ** 9, resume_checkpoint="",
                              learning_steps=0, checkpoint_path=str(ckdir), ddp_engine="native",
                              precision="bf16", exec_microbatch=0, device_prefetch=False)


def test_checkpoint_resume_is_bitwise_equivalent(tmp_path):
    """Save after 3 steps, resume in a new loop, 2 more steps: parameters, EMAs and optimizer
    moments equal the uninterrupted run's bit for bit (model/opt/ema files + the RNG sidecar with
    the kernel RNG counter, trainer.py save / _load_rng)."""
    from basic_utils import logger
    from distributed_pipeline_amd.ops.nn import RNG
    # the reference finds the checkpoint to resume in the logger's directory (trainer.py
    # find_resume_checkpoint): log and checkpoints share it, as in run/train.py
    logger.configure(dir=str(tmp_path / "ck"), format_strs=[])
    g = torch.Generator().manual_seed(3)
    B, L = 64, 128
    batch = {"input_ids": torch.randint(1000, 30522, (B, L), generator=g),
             "input_mask": torch.cat([torch.zeros(B, 48, dtype=torch.long), torch.ones(B, L - 48, dtype=torch.long)], 1)}
    RNG.counter = 0
    torch.manual_seed(5)
    a = _resume_loop(tmp_path / "ck", batch)
    for _ in range(3):
        a.run_step(batch)
        a.step += 1
    a.save()
    for _ in range(2):
        a.run_step(batch)
        a.step += 1
    torch.cuda.synchronize()
    want_p = a.ddp_model.space.param_flat.clone()
    want_ema = [[t.detach().clone() for t in lst] for lst in a.ema_params]
    RNG.counter = 12345  # clobbered: the resumed loop must restore it from the sidecar
    torch.manual_seed(999)
    b = _resume_loop(tmp_path / "ck", batch)
    assert b.resume_step == 3
    for _ in range(2):
        b.run_step(batch)
        b.step += 1
    torch.cuda.synchronize()
    got_p = b.ddp_model.space.param_flat
    assert torch.equal(want_p, got_p), _first_diff(b.ddp_model.space, want_p, got_p)
    for wl, gl in zip(want_ema, b.ema_params):
        for x, y in zip(wl, gl):
            assert torch.equal(x, y.detach())
