"""Transposed weight shadows (ops/nn.py shadow_t) across optimizer steps: the data-gradient GEMMs
read W^T, rebuilt once per shadow version (parallel/flat.py).  Three training steps with them must
match three steps without them - a stale W^T (one step behind the weights) would not."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _train(monkeypatch, wt):
    from basic_utils import logger
    from distributed_pipeline_amd.ops import nn as nn_ops
    from distributed_pipeline_amd.ops.nn import RNG
    from utils.initialization import create_diffusion_from_config, create_model_from_config, seed_all
    from utils.trainer import DiffusionTrainLoop

    monkeypatch.setattr(nn_ops, "_WT_SHADOW", wt)
    logger.configure(dir="/tmp/dpa_wt_test", format_strs=[])
    seed_all(0)
    RNG.counter = 0
    model = create_model_from_config(model="diffuseq", precision="bf16", config_name="tiny",
                                     hidden_size=256, num_layers=2, num_heads=4, intermediate_size=1024,
                                     vocab_size=30522, seq_len=128, hidden_dim=128, hidden_t_dim=128,
                                     dropout=0.1).cuda()
    diffusion, sampler = create_diffusion_from_config(diffusion_steps=2000)
    g = torch.Generator().manual_seed(1)
    B, L = 32, 128
    batch = {"input_ids": torch.randint(1000, 30522, (B, L), generator=g),
             "input_mask": torch.cat([torch.zeros(B, 48, dtype=torch.long),
                                      torch.ones(B, L - 48, dtype=torch.long)], 1)}
    loop = DiffusionTrainLoop(diffusion=diffusion, schedule_sampler=sampler, model=model,
                              data=iter([batch] * 3), batch_size=B, microbatch=B, lr=1e-3,
                              ema_rate="0.9999", log_interval=1, save_interval=10 ** 9, resume_checkpoint="",
                              learning_steps=3, checkpoint_path="/tmp/dpa_wt_test", ddp_engine="native",
                              precision="bf16", device_prefetch=False)
    torch.manual_seed(7)
    before = dict(nn_ops.WT_STATS)
    for _ in range(3):
        loop.run_step(batch)
    torch.cuda.synchronize()
    used = nn_ops.WT_STATS["used"] - before["used"]
    copies = nn_ops.WT_STATS["copies"] - before["copies"]
    return loop.ddp_model.space.param_flat.clone(), used, copies


def test_wt_shadow_training_matches(monkeypatch):
    p0, used0, _ = _train(monkeypatch, False)
    p1, used1, copies1 = _train(monkeypatch, True)
    assert used0 == 0 and used1 > 0
    # one rebuild per weight per optimizer step (3 steps; the first forward's shadow is version 1)
    assert 0 < copies1 <= used1
    err = (p0 - p1).abs().max().item()
    # the same products in the same K order on both operand paths: the runs agree to the run-to-run
    # noise of the fp32 atomic column sums (3.6e-7 measured); a W^T one step stale would move the
    # weights by Adam's lr-sized (1e-3) steps
    assert err <= 1e-5, err


def test_transpose_bf16_batch_matches_torch():
    from distributed_pipeline_amd.ops._ext import get_ext
    ext = get_ext(required=True)
    torch.manual_seed(3)
    shapes = [(768, 2304), (2304, 768), (768, 768), (3072, 768), (768, 3072), (128, 768), (768, 128), (64, 64)]
    srcs = [torch.randn(r, c, device="cuda").bfloat16() for r, c in shapes * 13]  # 104: two launches
    dsts = [torch.empty(c, r, device="cuda", dtype=torch.bfloat16) for r, c in shapes * 13]
    assert ext.transpose_bf16_batch(srcs, dsts)
    for a, b in zip(srcs, dsts):
        assert torch.equal(b, a.t())
    assert not ext.transpose_bf16_batch([torch.zeros(96, 64, device="cuda", dtype=torch.bfloat16)],
                                        [torch.zeros(64, 96, device="cuda", dtype=torch.bfloat16)])
