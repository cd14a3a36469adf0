"""Tiny MLP diffusion denoiser (BASELINE config #1: CPU/gloo plumbing model).

Same interface as :class:`TransformerNetModel` (``get_embeds``, ``token_nll``,
``get_logits``, ``forward(x_t, t)``) so it trains through the same
``GaussianDiffusion`` loss and DiffuSeq train loop, but the denoiser is a
2-hidden-layer per-token MLP conditioned on the timestep embedding.
"""
import torch
from torch import nn

from ..ops import nn as ops
from .layers import Embedding, Linear


class MLPDiffusionModel(nn.Module):
    def __init__(self, *, vocab_size=30522, input_dims=16, hidden_t_dim=16, hidden_size=0,
                 compute_dtype=torch.float32, **_):
        super().__init__()
        H = hidden_size or 64
        self.input_dims, self.hidden_t_dim = input_dims, hidden_t_dim
        self.compute_dtype = compute_dtype
        self.word_embedding = Embedding(vocab_size, input_dims)
        self.lm_head = Linear(input_dims, vocab_size)
        with torch.no_grad():
            self.lm_head.weight = self.word_embedding.weight
        self.time_embed = Linear(hidden_t_dim, H, act="silu")
        self.inp = Linear(input_dims, H, act="silu")
        self.hidden = Linear(H, H, act="silu")
        self.out = Linear(H, input_dims)

    def get_embeds(self, input_ids):
        return ops.embedding(input_ids, self.word_embedding.weight, torch.float32)

    def get_logits(self, x):
        return ops.linear(x.float(), self.lm_head.weight, self.lm_head.bias)

    def token_nll(self, x, ids):
        return ops.linear_cross_entropy(x.to(self.compute_dtype), self.lm_head.weight,
                                        self.lm_head.bias, ids)

    def forward(self, x, timesteps):
        dt = self.compute_dtype
        temb = self.time_embed(ops.timestep_embedding(timesteps, self.hidden_t_dim).to(dt))
        h = self.inp(x.to(dt)) + temb.unsqueeze(1)
        h = self.hidden(h)
        return self.out(h)
