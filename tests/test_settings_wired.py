"""Every TrainSettings field is read by code (no dead CLI settings),
and the model/diffusion settings that used to be inert now act: use_plm_init,
emb_scale_factor, sigma_small, rescale_learned_sigmas, use_hip_kernels."""
import inspect
import os

import pytest
import torch

from config.train import TrainSettings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONSUMERS = ["run/train.py", "utils/initialization.py", "utils/trainer.py", "data/__init__.py",
             "data/dataset.py", "distributed_pipeline_amd/models/__init__.py",
             "distributed_pipeline_amd/models/gaussian_diffusion.py"]


def test_every_setting_is_consumed():
    src = "\n".join(open(os.path.join(ROOT, p)).read() for p in CONSUMERS)
    fields = TrainSettings.model_fields if hasattr(TrainSettings, "model_fields") else TrainSettings.__fields__
    dead = [f for f in fields if f not in src]
    assert not dead, f"settings nobody reads: {dead}"


def _tiny_bert_dir(tmp_path):
    transformers = pytest.importorskip("transformers")
    cfg = transformers.BertConfig(hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
                                  intermediate_size=128, vocab_size=100, max_position_embeddings=64)
    torch.manual_seed(0)
    bert = transformers.BertModel(cfg)
    path = str(tmp_path / "bert")
    bert.save_pretrained(path)
    return path, bert


def test_use_plm_init_bert_copies_encoder(tmp_path):
    from distributed_pipeline_amd.models import build_model
    path, bert = _tiny_bert_dir(tmp_path)
    m = build_model(model="diffuseq", config_name=path, precision="fp32", vocab_size=100, seq_len=32,
                    use_plm_init="bert")
    lo, lr = m.input_transformers.layer[1], bert.encoder.layer[1]
    q = lr.attention.self.query.weight
    torch.testing.assert_close(m.input_transformers.layer[1].attn.qkv.weight[:64], q)
    torch.testing.assert_close(lo.ffn_out.weight, lr.output.dense.weight)
    torch.testing.assert_close(m.position_embeddings.weight, bert.embeddings.position_embeddings.weight)
    torch.testing.assert_close(m.LayerNorm.weight, bert.embeddings.LayerNorm.weight)


def test_emb_scale_factor_scales_diffusion_space():
    from distributed_pipeline_amd.models import build_model
    torch.manual_seed(0)
    a = build_model(model="diffuseq", config_name="tiny", precision="fp32", vocab_size=100)
    b = build_model(model="diffuseq", config_name="tiny", precision="fp32", vocab_size=100,
                    emb_scale_factor=2.5)
    b.load_state_dict(a.state_dict())
    ids = torch.randint(0, 100, (2, 8))
    torch.testing.assert_close(b.get_embeds(ids), 2.5 * a.get_embeds(ids))


def test_sigma_small_selects_reverse_variance_and_sampling_runs():
    from utils.initialization import create_diffusion_from_config
    from distributed_pipeline_amd.models import build_model
    d_small, _ = create_diffusion_from_config(diffusion_steps=8, sigma_small=True)
    d_large, _ = create_diffusion_from_config(diffusion_steps=8, sigma_small=False)
    assert d_small.model_var_type == "fixed_small" and d_large.model_var_type == "fixed_large"
    torch.manual_seed(0)
    m = build_model(model="diffuseq", config_name="tiny", precision="fp32", vocab_size=100, seq_len=16).eval()
    ids = torch.randint(0, 100, (2, 16))
    x0 = m.get_embeds(ids)
    mask = torch.zeros(2, 16, dtype=torch.long)
    mask[:, 8:] = 1
    out = d_small.p_sample_loop(m, x0.shape, mask=mask, x_start=x0)
    assert out.shape == x0.shape and torch.isfinite(out).all()
    torch.testing.assert_close(out[:, :8], x0[:, :8])  # source positions are never noised
    t = torch.full((2,), 5)
    _, lv_s, _ = d_small.p_mean_variance(m, out, t)
    _, lv_l, _ = d_large.p_mean_variance(m, out, t)
    assert (lv_s < lv_l).all()  # posterior variance < beta_t


def test_rescale_learned_sigmas_requires_learned_sigma():
    from utils.initialization import create_diffusion_from_config
    with pytest.raises(ValueError):
        create_diffusion_from_config(diffusion_steps=8, rescale_learned_sigmas=True)


def test_use_hip_kernels_false_disables_native_ops():
    from distributed_pipeline_amd.models import build_model
    from distributed_pipeline_amd.ops import _ext
    try:
        build_model(model="mlp_diffusion", precision="fp32", vocab_size=64, hidden_dim=16, hidden_t_dim=16,
                    hidden_size=32, use_hip_kernels=False)
        assert _ext._NATIVE_ENABLED is False and _ext.get_ext() is None
    finally:
        _ext.set_native_enabled(True)
