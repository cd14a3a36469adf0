"""
DiffuSeq ``TransformerNetModel`` (the workload the reference
template's trainer was adapted for, reference utils/trainer.py:1-4).

    word_embedding: Embedding(V, E)           lm_head: Linear(E, V), weight tied
    time_embed:     Linear(E_t, 4E_t) -> SiLU -> Linear(4E_t, H)
    input_up_proj:  Linear(E, H) -> Tanh -> Linear(H, H)
    h = Dropout(LN(pos_emb + up(x_t) + time_emb[:, None]))
    h = BertEncoder(h)                        (post-LN, 12 x 768 for DiffuSeq-base)
    out = output_down_proj(h):  Linear(H, H) -> Tanh -> Linear(H, E)

Parameter names follow DiffuSeq where the structure is the same
(``word_embedding``, ``lm_head``, ``time_embed.{0,2}``, ``input_up_proj.{0,2}``,
``position_embeddings``, ``LayerNorm``, ``output_down_proj.{0,2}``); the
encoder packs Q/K/V into ``input_transformers.layer.N.attn.qkv``.
"""
import torch
from torch import nn

from ..ops import nn as ops
from . import presets
from .layers import MLP, BertEncoder, Embedding, LayerNorm, Linear


class TransformerNetModel(nn.Module):
    def __init__(self, *, vocab_size=30522, input_dims=128, hidden_t_dim=128, seq_len=128,
                 config_name="bert-base-uncased", hidden_size=0, num_layers=0, num_heads=0,
                 intermediate_size=0, dropout=0.1, compute_dtype=torch.bfloat16, emb_scale_factor=1.0,
                 **_):
        super().__init__()
        cfg = presets.resolve(config_name, hidden_size=hidden_size, num_layers=num_layers,
                              num_heads=num_heads, intermediate_size=intermediate_size,
                              vocab_size=vocab_size)
        H = cfg["hidden_size"]
        self.cfg = cfg
        self.input_dims, self.hidden_t_dim, self.hidden_size = input_dims, hidden_t_dim, H
        self.dropout = dropout
        self.compute_dtype = compute_dtype
        self.seq_len = seq_len
        # DiffuSeq's --emb_scale_factor: the diffusion space is the word embedding times
        # this factor (1.0 = DiffuSeq default; != 1 takes the PyTorch diffusion path)
        self.emb_scale_factor = float(emb_scale_factor)
        assert seq_len <= cfg["max_position_embeddings"]

        self.word_embedding = Embedding(cfg["vocab_size"], input_dims)
        self.lm_head = Linear(input_dims, cfg["vocab_size"])
        with torch.no_grad():
            self.lm_head.weight = self.word_embedding.weight  # tied rounding head

        t4 = hidden_t_dim * 4
        self.time_embed = MLP(hidden_t_dim, t4, H, act="silu")
        self.input_up_proj = MLP(input_dims, H, H, act="tanh")
        self.input_transformers = BertEncoder(H, cfg["num_layers"], cfg["num_heads"],
                                              cfg["intermediate_size"], dropout,
                                              eps=cfg["layer_norm_eps"], init_std=0.02)
        self.register_buffer("position_ids", torch.arange(cfg["max_position_embeddings"]).unsqueeze(0),
                             persistent=False)
        self.position_embeddings = Embedding(cfg["max_position_embeddings"], H, init_std=0.02)
        self.LayerNorm = LayerNorm(H, eps=cfg["layer_norm_eps"])
        self.output_down_proj = MLP(H, H, input_dims, act="tanh")

    def grad_ready_order(self):
        """Parameters in the order their gradients complete in the backward (the DDP engine's flat
        layout, parallel/ddp.py: buckets are all-reduced front to back as they complete).  The
        reverse of the registration order - DiffuSeq's, kept for checkpoint parity - would put
        ``position_embeddings`` and ``LayerNorm`` (registered after the encoder, used at its input)
        into the first bucket, which then completes only at the end of the backward and holds every
        later bucket's all-reduce with it (measured: profiles/sim_comm_r6.txt)."""
        rev = list(reversed(list(self.parameters())))
        first = {id(p) for m in (self.output_down_proj, self.input_transformers) for p in m.parameters()}
        return [p for p in rev if id(p) in first] + [p for p in rev if id(p) not in first]

    # -- DiffuSeq API -------------------------------------------------------
    def get_embeds(self, input_ids):
        """Word embeddings in fp32 (diffusion space stays fp32), times emb_scale_factor."""
        e = ops.embedding(input_ids, self.word_embedding.weight, torch.float32)
        return e if self.emb_scale_factor == 1.0 else e * self.emb_scale_factor

    def get_logits(self, hidden_repr):
        """Materialised rounding logits (API parity; training uses :meth:`token_nll`)."""
        return ops.linear(hidden_repr.float(), self.lm_head.weight, self.lm_head.bias)

    def token_nll(self, x, ids):
        """Per-token CE of the tied rounding head, fused (x: [N, E], ids: [N])."""
        dt = self.compute_dtype
        return ops.linear_cross_entropy(x.to(dt), self.lm_head.weight, self.lm_head.bias, ids)

    # -- forward ------------------------------------------------------------
    def forward(self, x, timesteps):
        dt = self.compute_dtype
        B, L, _ = x.shape
        temb = ops.timestep_embedding(timesteps, self.hidden_t_dim, dtype=dt)
        emb_t = self.time_embed(temb)                                        # [B, H]
        emb_x = self.input_up_proj(x.to(dt))                                 # [B, L, H]
        pos = self.position_embeddings(self.position_ids[:, :L], dt)         # [1, L, H]
        # Dropout(LayerNorm(emb_x + pos + emb_t)) as one kernel (ops.embed_layernorm)
        h = ops.embed_layernorm(emb_x, pos, emb_t, self.LayerNorm.weight, self.LayerNorm.bias,
                                self.dropout, self.LayerNorm.eps, self.training)
        h = self.input_transformers(h)
        return self.output_down_proj(h)


def _train_flops_per_sample(self, seq_len):
    """Matmul FLOPs of one training sample (forward + backward = 3x forward for
    trained weights): encoder Linears 6*P_lin per token, attention 12*L*H per
    token per layer, the up/down projections, and the tied rounding head: the
    decoder_nll CE (6*E*V per token) plus the forward-only logged nll (2*E*V)."""
    cfg, H, E, L = self.cfg, self.hidden_size, self.input_dims, seq_len
    F_ = cfg["intermediate_size"]
    p_lin = cfg["num_layers"] * (4 * H * H + 2 * H * F_) + (E * H + H * H) * 2
    per_tok = 6 * p_lin + 12 * L * H * cfg["num_layers"] + 8 * E * cfg["vocab_size"]
    return per_tok * L


TransformerNetModel.train_flops_per_sample = _train_flops_per_sample


def count_params(model):
    return sum(p.numel() for p in model.parameters())
