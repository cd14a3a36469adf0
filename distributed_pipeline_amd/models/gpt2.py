"""GPT-2 small causal LM (BASELINE config #4: the generic-model path).

Trained through the *generic* ``TrainLoop`` hooks (``compute_losses`` /
``backward_from_losses``) rather than the diffusion loop.  Weight tying
``lm_head.weight is wte.weight``; the LM loss uses the fused
linear-cross-entropy op so the [tokens, 50257] logits never exist in memory.
"""
import torch
from torch import nn

from ..ops import nn as ops
from . import presets
from .layers import Embedding, GPT2Block, LayerNorm


class GPT2LMModel(nn.Module):
    def __init__(self, *, config_name="gpt2", vocab_size=0, seq_len=1024, hidden_size=0,
                 num_layers=0, num_heads=0, dropout=0.1, compute_dtype=torch.bfloat16, **_):
        super().__init__()
        cfg = presets.resolve(config_name, hidden_size=hidden_size, num_layers=num_layers,
                              num_heads=num_heads, vocab_size=vocab_size)
        H = cfg["hidden_size"]
        self.cfg, self.compute_dtype, self.dropout = cfg, compute_dtype, dropout
        assert seq_len <= cfg["max_position_embeddings"]
        self.wte = Embedding(cfg["vocab_size"], H, init_std=0.02)
        self.wpe = Embedding(cfg["max_position_embeddings"], H, init_std=0.01)
        self.h = nn.ModuleList(GPT2Block(H, cfg["num_heads"], dropout, eps=cfg["layer_norm_eps"],
                                         n_layers=cfg["num_layers"]) for _ in range(cfg["num_layers"]))
        self.ln_f = LayerNorm(H, eps=cfg["layer_norm_eps"])
        self.register_buffer("position_ids", torch.arange(cfg["max_position_embeddings"]).unsqueeze(0),
                             persistent=False)

    def hidden_states(self, input_ids):
        dt = self.compute_dtype
        B, L = input_ids.shape
        # every residual add (and the embedding sum + dropout) runs fused with the
        # LayerNorm that reads it: x = x + dropout(branch), a = LN_next(x) in one kernel
        lns = [blk.ln_1 for blk in self.h] + [self.ln_f]
        x, a = ops.residual_layernorm(self.wte(input_ids, dt), None, lns[0].weight, lns[0].bias,
                                      self.dropout, lns[0].eps, self.training,
                                      pos=self.wpe(self.position_ids[:, :L], dt))
        for i, blk in enumerate(self.h):
            x, h = blk(x, a)
            x, a = ops.residual_layernorm(h, x, lns[i + 1].weight, lns[i + 1].bias, self.dropout,
                                          lns[i + 1].eps, self.training)
        return a

    def forward(self, input_ids, labels=None):
        """Returns per-token CE [B, L-1] when ``labels`` (shifted internally) are given."""
        h = self.hidden_states(input_ids)
        if labels is None:
            return ops.linear(h, self.wte.weight)
        B, L, H = h.shape
        x = h[:, :-1].reshape(-1, H)
        tgt = labels[:, 1:].reshape(-1)
        return ops.linear_cross_entropy(x, self.wte.weight, None, tgt).view(B, L - 1)


def _gpt2_train_flops_per_sample(self, seq_len):
    """6*P_lin + causal attention (~6*L*H per layer, half of the full 12*L*H) per
    token, plus the tied LM head (6*H*V), times seq_len."""
    cfg = self.cfg
    H, V, n = cfg["hidden_size"], cfg["vocab_size"], cfg["num_layers"]
    F_ = cfg.get("intermediate_size") or 4 * H
    per_tok = 6 * n * (4 * H * H + 2 * H * F_) + 6 * seq_len * H * n + 6 * H * V
    return per_tok * seq_len


GPT2LMModel.train_flops_per_sample = _gpt2_train_flops_per_sample

