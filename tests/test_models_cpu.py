"""Model / diffusion / data numerics on CPU (fp32 reference path)."""
import math

import numpy as np
import pytest
import torch

from data import load_data_from_args
from data.dataset import CLS_ID, SEP_ID, SyntheticSeq2SeqDataset
from distributed_pipeline_amd.models import (build_model, count_params, create_gaussian_diffusion,
                                             get_named_beta_schedule)
from distributed_pipeline_amd.models.layers import BertEncoder
from distributed_pipeline_amd.ops import nn as ops


def test_diffuseq_base_param_count():
    # 91,225,274 = SURVEY §2.4 probe of DiffuSeq-base
    assert count_params(build_model(model="diffuseq", precision="fp32")) == 91225274


def test_diffuseq_xl_size():
    n = count_params(build_model(model="diffuseq", config_name="diffuseq-xl", precision="fp32"))
    assert 1.25e9 < n < 1.4e9


def test_gpt2_small_size():
    n = count_params(build_model(model="gpt2", config_name="gpt2", precision="fp32", seq_len=1024))
    assert abs(n - 124.4e6) < 1e6  # GPT-2 small with tied lm_head


def test_sqrt_schedule_matches_closed_form():
    betas = get_named_beta_schedule("sqrt", 2000)
    ab = np.cumprod(1 - betas)
    t = np.array([0, 10, 1000, 1998])  # t = T-1 is clipped by max_beta
    target = 1 - np.sqrt((t + 1) / 2000 + 1e-4)
    np.testing.assert_allclose(ab[t], target / (1 - np.sqrt(1e-4)), rtol=1e-6)
    assert betas.max() <= 0.999


def test_q_sample_keeps_source_positions():
    d = create_gaussian_diffusion(steps=100)
    x0 = torch.randn(2, 5, 3)
    noise = torch.randn_like(x0)
    mask = torch.tensor([[0, 0, 1, 1, 1], [0, 1, 1, 1, 1]])
    t = torch.tensor([50, 99])
    xt = d.q_sample(x0, t, noise, mask)
    assert torch.equal(xt[0, :2], x0[0, :2]) and torch.equal(xt[1, :1], x0[1, :1])
    sa = math.sqrt(d.alphas_cumprod[50])
    torch.testing.assert_close(xt[0, 2:], sa * x0[0, 2:] + math.sqrt(1 - d.alphas_cumprod[50]) * noise[0, 2:])


def test_training_loss_terms_match_formula(monkeypatch):
    torch.manual_seed(0)
    model = build_model(model="diffuseq", config_name="tiny", precision="fp32", vocab_size=500,
                        dropout=0.0)
    d = create_gaussian_diffusion(steps=100)
    ids = torch.randint(0, 500, (3, 16))
    mask = torch.ones(3, 16, dtype=torch.long)
    mask[:, :5] = 0
    t = torch.tensor([0, 5, 99])
    zeros = lambda x: torch.zeros_like(x)  # noqa: E731
    monkeypatch.setattr(torch, "randn_like", zeros)
    terms = d.training_losses(model, None, t, dict(input_ids=ids, input_mask=mask))
    x0 = model.get_embeds(ids)
    out = model(d.q_sample(x0, t, torch.zeros_like(x0), mask), d.scale_timesteps(t))
    mse = ((x0 - out) ** 2).mean((1, 2))
    logits = model.get_logits(x0)
    dnll = torch.nn.functional.cross_entropy(logits.reshape(-1, 500), ids.reshape(-1),
                                             reduction="none").view(3, 16).mean(-1)
    tT = ((math.sqrt(d.alphas_cumprod[-1]) * x0) ** 2).mean((1, 2))
    torch.testing.assert_close(terms["mse"], mse, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(terms["decoder_nll"], dnll, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(terms["loss"], mse + dnll + tT, rtol=1e-5, atol=1e-5)


def test_encoder_matches_hf_bert():
    """Golden model: HF BertEncoder (transformers) with mapped weights, dropout off."""
    transformers = pytest.importorskip("transformers")
    from transformers.models.bert.modeling_bert import BertEncoder as HFEncoder
    cfg = transformers.BertConfig(hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                                  intermediate_size=256, hidden_dropout_prob=0.0,
                                  attention_probs_dropout_prob=0.0, layer_norm_eps=1e-12)
    torch.manual_seed(0)
    hf = HFEncoder(cfg).eval()
    ours = BertEncoder(128, 2, 2, 256, 0.0).eval()
    with torch.no_grad():
        for lo, lh in zip(ours.layer, hf.layer):
            a = lh.attention
            lo.attn.qkv.weight.copy_(torch.cat([a.self.query.weight, a.self.key.weight, a.self.value.weight]))
            lo.attn.qkv.bias.copy_(torch.cat([a.self.query.bias, a.self.key.bias, a.self.value.bias]))
            lo.attn_out.weight.copy_(a.output.dense.weight)
            lo.attn_out.bias.copy_(a.output.dense.bias)
            lo.attn_ln.weight.copy_(a.output.LayerNorm.weight)
            lo.attn_ln.bias.copy_(a.output.LayerNorm.bias)
            lo.ffn_in.weight.copy_(lh.intermediate.dense.weight)
            lo.ffn_in.bias.copy_(lh.intermediate.dense.bias)
            lo.ffn_out.weight.copy_(lh.output.dense.weight)
            lo.ffn_out.bias.copy_(lh.output.dense.bias)
            lo.ffn_ln.weight.copy_(lh.output.LayerNorm.weight)
            lo.ffn_ln.bias.copy_(lh.output.LayerNorm.bias)
    x = torch.randn(2, 10, 128)
    ref = hf(x)[0]
    torch.testing.assert_close(ours(x), ref, rtol=1e-4, atol=1e-4)


def test_bf16_cpu_path_runs_and_grads_fp32():
    model = build_model(model="diffuseq", config_name="tiny", precision="bf16", vocab_size=300)
    x = torch.randn(2, 8, 128)
    out = model(x, torch.tensor([1.0, 2.0]))
    out.float().sum().backward()
    for p in model.parameters():
        if p.grad is not None:
            assert p.grad.dtype == torch.float32


def test_synthetic_seq2seq_layout_and_determinism():
    ds = SyntheticSeq2SeqDataset(100, 32, 30522, seed=1)
    a, b = ds.__getitems__([3, 7]), ds.__getitems__([3, 7])
    assert torch.equal(a["input_ids"], b["input_ids"])
    ids, m = a["input_ids"][0], a["input_mask"][0]
    assert ids[0] == CLS_ID and (ids == SEP_ID).sum() == 2
    first_sep = int((ids == SEP_ID).nonzero()[0])
    assert m[:first_sep + 1].sum() == 0 and m[first_sep + 1:].all()


def test_sharded_loader_disjoint():
    it0 = load_data_from_args("train", "x", 4, deterministic=True, loop=False, num_loader_proc=0,
                              dataset="synthetic", seq_len=8, vocab_size=5000, shard=True, rank=0,
                              world_size=2, pin_memory=False)
    it1 = load_data_from_args("train", "x", 4, deterministic=True, loop=False, num_loader_proc=0,
                              dataset="synthetic", seq_len=8, vocab_size=5000, shard=True, rank=1,
                              world_size=2, pin_memory=False)
    b0, b1 = next(iter(it0)), next(iter(it1))
    assert not torch.equal(b0["input_ids"], b1["input_ids"])


def test_linear_cross_entropy_reference_path():
    x = torch.randn(6, 16)
    w = torch.nn.Parameter(torch.randn(40, 16))
    b = torch.nn.Parameter(torch.randn(40))
    tgt = torch.randint(0, 40, (6,))
    loss = ops.linear_cross_entropy(x, w, b, tgt)
    ref = torch.nn.functional.cross_entropy(x @ w.t() + b, tgt, reduction="none")
    torch.testing.assert_close(loss, ref)
