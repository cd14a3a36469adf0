"""Numerics criterion of SURVEY 7.4 item 5: the bf16 native path (hand-written
kernels, flat fp32 master weights, fused AdamW/EMA) must track the fp32 stock-PyTorch
reference loss curve.  Tiny DiffuSeq, a fixed memorisable token set, same seeds and
batches on both paths; losses compared as averages over a window (the diffusion
loss is noisy per step: random t, and the fused path draws its noise in-kernel)."""
import itertools
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

STEPS = 160


def _train(precision, engine, tmp):
    from basic_utils import logger
    from utils.initialization import create_diffusion_from_config, create_model_from_config, seed_all
    from utils.trainer import DiffusionTrainLoop

    logger.configure(dir=os.path.join(tmp, f"{precision}_{engine}"), format_strs=[])
    seed_all(0)
    model = create_model_from_config(model="diffuseq", precision=precision, config_name="tiny",
                                     hidden_size=256, num_layers=2, num_heads=4, intermediate_size=1024,
                                     vocab_size=2048, seq_len=64, hidden_dim=128, hidden_t_dim=128,
                                     dropout=0.0).cuda()
    diffusion, sampler = create_diffusion_from_config(diffusion_steps=2000)
    g = torch.Generator().manual_seed(123)
    B, L = 32, 64
    data = [{"input_ids": torch.randint(100, 2048, (B, L), generator=g),
             "input_mask": torch.cat([torch.zeros(B, 24, dtype=torch.long),
                                      torch.ones(B, L - 24, dtype=torch.long)], 1)} for _ in range(2)]
    loop = DiffusionTrainLoop(diffusion=diffusion, schedule_sampler=sampler, model=model,
                              data=itertools.cycle(data), batch_size=B, microbatch=B, lr=1e-3,
                              ema_rate="0.9", log_interval=10 ** 9, save_interval=10 ** 9,
                              resume_checkpoint="", learning_steps=0, checkpoint_path=tmp,
                              ddp_engine=engine, precision=precision)
    losses = []
    torch.manual_seed(7)
    for _ in range(STEPS):
        loop.run_step(next(loop.data))
        losses.append(float(logger.dumpkvs()["loss"]))
        loop.step += 1
    return torch.tensor(losses)


def test_bf16_native_tracks_fp32_reference_loss_curve(tmp_path):
    ref = _train("fp32", "torch", str(tmp_path))
    nat = _train("bf16", "native", str(tmp_path))
    assert torch.isfinite(nat).all() and torch.isfinite(ref).all()
    head_r, tail_r = ref[:10].mean().item(), ref[-30:].mean().item()
    head_n, tail_n = nat[:10].mean().item(), nat[-30:].mean().item()
    assert tail_r < 0.5 * head_r, (head_r, tail_r)          # the reference actually learns
    assert tail_n < 0.5 * head_n, (head_n, tail_n)
    # the two curves agree to within a few percent over the late window
    assert abs(tail_n - tail_r) / tail_r < 0.08, (tail_n, tail_r)
    print(f"loss head fp32 {head_r:.4f} bf16 {head_n:.4f} | tail fp32 {tail_r:.4f} bf16 {tail_n:.4f}")
