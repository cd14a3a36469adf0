"""Full-size numerics on DiffuSeq-base (768 x 12,
V = 30522, L = 128):

* the bf16 native engine (hand-written kernels, fp32 master weights, fused AdamW/EMA,
  fused executed micro-batch) tracks the fp32 stock-PyTorch reference engine (torch
  DDP-equivalent, torch AdamW, one fwd/bwd per micro-batch) over 200 optimizer steps:
  late-window mean loss within 2%;
* at full shapes, one fused forward/backward over the whole batch gives the same
  gradient as the reference's accumulation over 64-sample micro-batches.

The per-step losses go to $DPA_CONVERGENCE_LOG when set (profiles/convergence_base_r2.log).
"""
import itertools
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

STEPS = 200
BASE = dict(model="diffuseq", config_name="bert-base-uncased", vocab_size=30522, seq_len=128,
            hidden_dim=128, hidden_t_dim=128)


def _data(B, L, n=4):
    g = torch.Generator().manual_seed(123)
    mask = torch.cat([torch.zeros(B, L // 2, dtype=torch.long), torch.ones(B, L - L // 2, dtype=torch.long)], 1)
    return [{"input_ids": torch.randint(1000, 30000, (B, L), generator=g), "input_mask": mask} for _ in range(n)]


def _train(precision, engine, tmp, B=128):
    from basic_utils import logger
    from utils.initialization import create_diffusion_from_config, create_model_from_config, seed_all
    from utils.trainer import DiffusionTrainLoop

    logger.configure(dir=os.path.join(tmp, f"{precision}_{engine}"), format_strs=[])
    seed_all(0)
    model = create_model_from_config(precision=precision, dropout=0.1, **BASE).cuda()
    diffusion, sampler = create_diffusion_from_config(diffusion_steps=2000)
    loop = DiffusionTrainLoop(diffusion=diffusion, schedule_sampler=sampler, model=model,
                              data=itertools.cycle(_data(B, 128)), batch_size=B, microbatch=64, lr=1e-4,
                              ema_rate="0.5,0.9,0.99", log_interval=10 ** 9, save_interval=10 ** 9,
                              resume_checkpoint="", learning_steps=0, checkpoint_path=tmp,
                              ddp_engine=engine, precision=precision,
                              exec_microbatch=-1 if engine == "torch" else 0)
    losses = []
    torch.manual_seed(7)
    for _ in range(STEPS):
        loop.run_step(next(loop.data))
        losses.append(float(logger.dumpkvs()["loss"]))
        loop.step += 1
    return torch.tensor(losses), loop.exec_microbatch


def test_base_bf16_native_tracks_fp32_reference_200_steps(tmp_path, monkeypatch):
    """Also the byte-cutting epilogues against the plain bf16 path: the default native run stores
    act' as u8 codes and folds residual + dropout into the N = 768 GEMMs (ops/nn.py _ACT_Q8,
    _RES_FUSE); a third run with both off must track the same curve (its dropout masks come from
    the Philox stream instead of the pair hash, so the trajectories differ by dropout noise only)."""
    from distributed_pipeline_amd.ops import nn as nn_ops
    ref, ex_r = _train("fp32", "torch", str(tmp_path))
    nat, ex_n = _train("bf16", "native", str(tmp_path))
    monkeypatch.setattr(nn_ops, "_ACT_Q8", False)
    monkeypatch.setattr(nn_ops, "_RES_FUSE", False)
    plain, _ = _train("bf16", "native", str(tmp_path))
    assert ex_r == 64 and ex_n == 128  # reference schedule vs the fused default
    assert torch.isfinite(nat).all() and torch.isfinite(ref).all() and torch.isfinite(plain).all()
    head_r, tail_r = ref[:20].mean().item(), ref[-50:].mean().item()
    head_n, tail_n = nat[:20].mean().item(), nat[-50:].mean().item()
    tail_p = plain[-50:].mean().item()
    path = os.environ.get("DPA_CONVERGENCE_LOG")
    if path:
        with open(path, "w") as f:
            f.write("# DiffuSeq-base 768x12 seq128, batch 128 (2 x 64), lr 1e-4, 200 steps, synthetic\n")
            f.write("# step fp32_torch_engine bf16_native_engine(u8 act', fused residual-dropout) "
                    "bf16_native_engine(bf16 act', unfused)\n")
            for i, (a, b, c) in enumerate(zip(ref.tolist(), nat.tolist(), plain.tolist())):
                f.write(f"{i} {a:.5f} {b:.5f} {c:.5f}\n")
            f.write(f"# head(20) fp32 {head_r:.5f} bf16 {head_n:.5f} | tail(50) fp32 {tail_r:.5f} "
                    f"bf16 {tail_n:.5f} bf16-plain {tail_p:.5f} | rel diff {abs(tail_n - tail_r) / tail_r:.4f} "
                    f"(plain {abs(tail_p - tail_r) / tail_r:.4f})\n")
    assert tail_r < head_r and tail_n < head_n, (head_r, tail_r, head_n, tail_n)
    assert abs(tail_n - tail_r) / tail_r < 0.02, (tail_n, tail_r)
    assert abs(tail_p - tail_r) / tail_r < 0.02, (tail_p, tail_r)


def test_fused_exec_microbatch_equals_accumulation_full_shapes(monkeypatch):
    """exec_microbatch = 256 (one fwd/bwd) vs 4 x 64 accumulated under no_sync, same
    noise and timesteps (explicit noise -> the PyTorch diffusion formulas; the x_start
    jitter zeroed), dropout 0."""
    monkeypatch.setattr(torch, "randn_like", lambda x: torch.zeros_like(x))
    from distributed_pipeline_amd.models import build_model, create_gaussian_diffusion
    from distributed_pipeline_amd.parallel.ddp import DDPEngine
    torch.manual_seed(0)
    model = build_model(precision="bf16", dropout=0.0, **BASE).cuda()
    eng = DDPEngine(model, shadow_dtype=torch.bfloat16)
    diff = create_gaussian_diffusion(steps=2000)
    B, mb = 256, 64
    d = _data(B, 128, 1)[0]
    ids, mask = d["input_ids"].cuda(), d["input_mask"].cuda()
    g = torch.Generator(device="cuda").manual_seed(3)
    t = torch.randint(0, 2000, (B,), device="cuda", generator=g)
    noise = torch.randn(B, 128, 128, device="cuda", generator=g)

    def loss_of(s, e):
        terms = diff.training_losses(eng, None, t[s:e], dict(input_ids=ids[s:e], input_mask=mask[s:e]),
                                     noise=noise[s:e])
        return terms["loss"]

    eng.zero_grad()
    (loss_of(0, B).mean() * (B / mb)).backward()
    fused = eng.space.grad_flat.clone()
    eng.zero_grad()
    for s in range(0, B, mb):
        loss_of(s, s + mb).mean().backward()
    acc = eng.space.grad_flat.clone()
    rel = ((fused - acc).norm() / acc.norm()).item()
    assert acc.abs().sum() > 0 and rel < 2e-2, rel
