"""Encoder-stack golden test: our post-LN ``BertEncoder``
(models/layers.py, the DiffuSeq ``input_transformers``) against the transformers
library's ``BertEncoder`` with identical weights, fp32 on CPU."""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from distributed_pipeline_amd.models.layers import BertEncoder  # noqa: E402


def _copy_weights(ours, ref, H):
    with torch.no_grad():
        for lo, lr in zip(ours.layer, ref.layer):
            wq, wk, wv = lo.attn.qkv.weight.split(H, 0)
            bq, bk, bv = lo.attn.qkv.bias.split(H, 0)
            for lin, w, b in ((lr.attention.self.query, wq, bq), (lr.attention.self.key, wk, bk),
                              (lr.attention.self.value, wv, bv)):
                lin.weight.copy_(w)
                lin.bias.copy_(b)
            pairs = ((lr.attention.output.dense, lo.attn_out), (lr.attention.output.LayerNorm, lo.attn_ln),
                     (lr.intermediate.dense, lo.ffn_in), (lr.output.dense, lo.ffn_out),
                     (lr.output.LayerNorm, lo.ffn_ln))
            for r, o in pairs:
                r.weight.copy_(o.weight)
                r.bias.copy_(o.bias)


@pytest.mark.parametrize("L", [16, 128])
def test_encoder_matches_transformers_bert(L):
    torch.manual_seed(0)
    H, layers, heads, ffn = 64, 2, 4, 256
    ours = BertEncoder(H, layers, heads, ffn, 0.0, 1e-12, 0.02).eval()
    for p in ours.parameters():   # non-trivial LN affine params too
        if p.dim() == 1:
            torch.nn.init.normal_(p, 0.0, 0.1)
    cfg = transformers.BertConfig(hidden_size=H, num_hidden_layers=layers, num_attention_heads=heads,
                                  intermediate_size=ffn, hidden_act="gelu", hidden_dropout_prob=0.0,
                                  attention_probs_dropout_prob=0.0, layer_norm_eps=1e-12)
    cfg._attn_implementation = "eager"
    ref = transformers.models.bert.modeling_bert.BertEncoder(cfg).eval()
    _copy_weights(ours, ref, H)
    x = torch.randn(3, L, H)
    with torch.no_grad():
        y = ours(x)
        r = ref(x)[0]
    torch.testing.assert_close(y, r, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_native_bf16_encoder_matches_transformers_bert_fp32():
    """Same golden check through the hand-written kernels (bf16 activations, fused
    attention/LN sublayers, fp32 master weights) on the DiffuSeq-base head shape."""
    from distributed_pipeline_amd.ops import nn as opsnn
    torch.manual_seed(0)
    H, layers, heads, ffn, L = 256, 2, 4, 1024, 128
    ours = BertEncoder(H, layers, heads, ffn, 0.0, 1e-12, 0.02).cuda().eval()
    cfg = transformers.BertConfig(hidden_size=H, num_hidden_layers=layers, num_attention_heads=heads,
                                  intermediate_size=ffn, hidden_act="gelu", hidden_dropout_prob=0.0,
                                  attention_probs_dropout_prob=0.0, layer_norm_eps=1e-12)
    cfg._attn_implementation = "eager"
    ref = transformers.models.bert.modeling_bert.BertEncoder(cfg).cuda().eval()
    _copy_weights(ours, ref, H)
    x = torch.randn(4, L, H, device="cuda")
    n0 = opsnn.DB_HANDOFF_STATS["fused_sublayers"]
    with torch.no_grad():
        y = ours(x.bfloat16())
        r = ref(x)[0]
    assert y.dtype == torch.bfloat16
    assert opsnn.DB_HANDOFF_STATS["fused_sublayers"] - n0 == 2 * layers   # native fused path ran
    torch.testing.assert_close(y.float(), r, rtol=3e-2, atol=3e-2)
