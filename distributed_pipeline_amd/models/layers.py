"""
Transformer building blocks on top of ``distributed_pipeline_amd.ops.nn``.

Parameters are plain fp32 ``nn.Parameter``s (the master copy; the DDP engine
re-homes them into one flat buffer and attaches bf16 shadows).  Activations
run in the module's compute dtype (bf16 on MI355X, fp32 for the
reference-equivalent baseline).

The BERT encoder follows the post-LN layout of HF ``BertEncoder``
(bert-base-uncased: 12 x [self-attention, out-proj + residual + LN,
FFN(GELU) + residual + LN], LN eps 1e-12), with Q/K/V packed into one
[3H, H] projection so the forward is a single GEMM.
"""
import math

import torch
from torch import nn

from ..ops import nn as ops


class Linear(nn.Module):
    """``nn.Linear``-compatible parameters (``weight`` [out, in], ``bias`` [out])."""

    def __init__(self, in_features, out_features, bias=True, act="none", init_std=None):
        super().__init__()
        self.in_features, self.out_features, self.act = in_features, out_features, act
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        self.bias = nn.Parameter(torch.empty(out_features)) if bias else None
        self.reset_parameters(init_std)

    def reset_parameters(self, init_std=None):
        if init_std is None:  # torch nn.Linear default
            nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
            if self.bias is not None:
                bound = 1.0 / math.sqrt(self.in_features) if self.in_features > 0 else 0
                nn.init.uniform_(self.bias, -bound, bound)
        else:  # BERT/GPT-2 style
            nn.init.normal_(self.weight, std=init_std)
            if self.bias is not None:
                nn.init.zeros_(self.bias)

    def forward(self, x):
        return ops.linear(x, self.weight, self.bias, self.act)

    def extra_repr(self):
        return f"in={self.in_features}, out={self.out_features}, act={self.act}"


class MLP(nn.Sequential):
    """Linear(act) -> Identity -> Linear with DiffuSeq's Sequential parameter names
    (``0.*``, ``2.*``); runs as one fused op (see ``ops.mlp``)."""

    def __init__(self, d_in, d_hidden, d_out, act, init_std=None):
        super().__init__(Linear(d_in, d_hidden, act=act, init_std=init_std), nn.Identity(),
                         Linear(d_hidden, d_out, init_std=init_std))

    def forward(self, x):
        return ops.mlp(x, self[0], self[2])


class LayerNorm(nn.Module):
    def __init__(self, dim, eps=1e-12):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))
        self.bias = nn.Parameter(torch.zeros(dim))

    def forward(self, x, residual=None, dropout=0.0):
        """LN(dropout(x) + residual)."""
        return ops.add_dropout_layernorm(x, residual, self.weight, self.bias, dropout, self.eps,
                                         self.training)


class Embedding(nn.Module):
    def __init__(self, num, dim, init_std=None):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(num, dim))
        if init_std is None:
            nn.init.normal_(self.weight)
        else:
            nn.init.normal_(self.weight, std=init_std)

    def forward(self, ids, dtype):
        return ops.embedding(ids, self.weight, dtype)


class SelfAttention(nn.Module):
    def __init__(self, hidden, heads, dropout, causal=False, init_std=0.02):
        super().__init__()
        assert hidden % heads == 0
        self.heads, self.dropout, self.causal = heads, dropout, causal
        self.qkv = Linear(hidden, 3 * hidden, init_std=init_std)

    def forward(self, x):
        qkv = self.qkv(x)
        return ops.attention(qkv, self.heads, self.dropout, self.causal, self.training)


class BertLayer(nn.Module):
    """Post-LN transformer layer (HF BertLayer semantics, packed QKV)."""

    def __init__(self, hidden, heads, ffn, dropout, eps=1e-12, init_std=0.02):
        super().__init__()
        self.dropout = dropout
        self.attn = SelfAttention(hidden, heads, dropout, init_std=init_std)
        self.attn_out = Linear(hidden, hidden, init_std=init_std)
        self.attn_ln = LayerNorm(hidden, eps)
        self.ffn_in = Linear(hidden, ffn, act="gelu", init_std=init_std)
        self.ffn_out = Linear(ffn, hidden, init_std=init_std)
        self.ffn_ln = LayerNorm(hidden, eps)

    def forward(self, x):
        # each post-LN sublayer runs as one fused op on the HIP path (the op owns
        # both uses of its input, so the residual-branch gradient is accumulated
        # by the dgrad GEMM); the composed ops otherwise
        h = ops.attn_add_ln(x, self.attn.qkv, self.attn_out, self.attn_ln, self.attn.heads,
                            self.attn.dropout, self.dropout, self.training)
        return ops.mlp_add_ln(h, self.ffn_in, self.ffn_out, self.ffn_ln, self.dropout, self.training)


class BertEncoder(nn.Module):
    def __init__(self, hidden, layers, heads, ffn, dropout, eps=1e-12, init_std=0.02):
        super().__init__()
        self.layer = nn.ModuleList(BertLayer(hidden, heads, ffn, dropout, eps, init_std)
                                   for _ in range(layers))

    def forward(self, x):
        for lyr in self.layer:
            x = lyr(x)
        return x


class GPT2Block(nn.Module):
    """Pre-LN causal block (GPT-2)."""

    def __init__(self, hidden, heads, dropout, eps=1e-5, init_std=0.02, n_layers=12):
        super().__init__()
        self.dropout = dropout
        self.ln_1 = LayerNorm(hidden, eps)
        self.attn = SelfAttention(hidden, heads, dropout, causal=True, init_std=init_std)
        self.attn_proj = Linear(hidden, hidden, init_std=init_std / math.sqrt(2 * n_layers))
        self.ln_2 = LayerNorm(hidden, eps)
        self.mlp_fc = Linear(hidden, 4 * hidden, act="gelu", init_std=init_std)
        self.mlp_proj = Linear(4 * hidden, hidden, init_std=init_std / math.sqrt(2 * n_layers))

    def forward(self, x, a):
        """x: residual stream, a = ln_1(x) (produced by the previous fused residual
        step) -> (x + dropout(attn), MLP branch output); the caller adds that branch
        fused with the next LayerNorm (ops.residual_layernorm)."""
        h = self.attn_proj(self.attn(a))
        x, a = ops.residual_layernorm(h, x, self.ln_2.weight, self.ln_2.bias, self.dropout,
                                      self.ln_2.eps, self.training)
        return x, ops.mlp(a, self.mlp_fc, self.mlp_proj)
