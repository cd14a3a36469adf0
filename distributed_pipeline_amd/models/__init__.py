"""Model zoo: DiffuSeq transformer (base / XL), tiny MLP diffusion, GPT-2 small."""
import torch

from .diffuseq import TransformerNetModel, count_params
from .gaussian_diffusion import GaussianDiffusion, create_gaussian_diffusion, get_named_beta_schedule
from .gpt2 import GPT2LMModel
from .mlp_diffusion import MLPDiffusionModel
from .resample import create_named_schedule_sampler


def compute_dtype_for(precision):
    return torch.bfloat16 if precision == "bf16" else torch.float32


def build_model(*, model="diffuseq", precision="bf16", vocab_size=30522, hidden_dim=128,
                hidden_t_dim=128, seq_len=128, config_name="bert-base-uncased", hidden_size=0,
                num_layers=0, num_heads=0, intermediate_size=0, dropout=0.1, use_hip_kernels=True,
                use_plm_init="no", emb_scale_factor=1.0, **_):
    from ..ops import _ext
    _ext.set_native_enabled(use_hip_kernels)
    dt = compute_dtype_for(precision)
    if model == "diffuseq":
        m = TransformerNetModel(vocab_size=vocab_size, input_dims=hidden_dim,
                                hidden_t_dim=hidden_t_dim, seq_len=seq_len,
                                config_name=config_name, hidden_size=hidden_size,
                                num_layers=num_layers, num_heads=num_heads,
                                intermediate_size=intermediate_size, dropout=dropout,
                                compute_dtype=dt, emb_scale_factor=emb_scale_factor)
        if use_plm_init == "bert":
            from .plm_init import load_bert_init
            load_bert_init(m, config_name)
        return m
    if use_plm_init != "no":
        raise ValueError(f"use_plm_init={use_plm_init!r} is only defined for the diffuseq model")
    if model == "mlp_diffusion":
        return MLPDiffusionModel(vocab_size=vocab_size, input_dims=hidden_dim,
                                 hidden_t_dim=hidden_t_dim, hidden_size=hidden_size, compute_dtype=dt)
    if model == "gpt2":
        name = config_name if config_name in ("gpt2", "tiny") else "gpt2"
        return GPT2LMModel(config_name=name, vocab_size=vocab_size if vocab_size != 30522 else 0,
                           seq_len=seq_len, hidden_size=hidden_size, num_layers=num_layers,
                           num_heads=num_heads, dropout=dropout, compute_dtype=dt)
    raise ValueError(f"unknown model {model!r}")


__all__ = ["TransformerNetModel", "MLPDiffusionModel", "GPT2LMModel", "GaussianDiffusion",
           "create_gaussian_diffusion", "get_named_beta_schedule", "create_named_schedule_sampler",
           "build_model", "count_params", "compute_dtype_for"]
