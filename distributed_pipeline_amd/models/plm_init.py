"""``use_plm_init=bert``: initialise the DiffuSeq encoder from a pretrained BERT
(DiffuSeq ``TransformerNetModel`` with ``init_pretrained='bert'``).

Offline by construction: ``config_name`` must name a local transformers checkpoint
directory (or a model already in the local HF cache); nothing is downloaded.  The
HF encoder's separate Q/K/V projections are packed into this model's fused
``qkv`` Linear (rows [Q; K; V]); the position embeddings and the embedding
LayerNorm are copied too, as DiffuSeq does.
"""
import torch


def load_bert_init(model, name_or_path):
    try:
        from transformers import BertModel
    except ImportError as exc:  # pragma: no cover - transformers is installed here
        raise RuntimeError("use_plm_init=bert needs the transformers package") from exc
    bert = BertModel.from_pretrained(name_or_path, local_files_only=True)
    H = model.hidden_size
    if bert.config.hidden_size != H or bert.config.num_hidden_layers != len(model.input_transformers.layer):
        raise ValueError(f"pretrained {name_or_path!r} ({bert.config.hidden_size} x "
                         f"{bert.config.num_hidden_layers}) does not match the model ({H} x "
                         f"{len(model.input_transformers.layer)})")
    with torch.no_grad():
        for lo, lr in zip(model.input_transformers.layer, bert.encoder.layer):
            sa = lr.attention.self
            lo.attn.qkv.weight.copy_(torch.cat([sa.query.weight, sa.key.weight, sa.value.weight], 0))
            lo.attn.qkv.bias.copy_(torch.cat([sa.query.bias, sa.key.bias, sa.value.bias], 0))
            for ours, ref in ((lo.attn_out, lr.attention.output.dense), (lo.attn_ln, lr.attention.output.LayerNorm),
                              (lo.ffn_in, lr.intermediate.dense), (lo.ffn_out, lr.output.dense),
                              (lo.ffn_ln, lr.output.LayerNorm)):
                ours.weight.copy_(ref.weight)
                ours.bias.copy_(ref.bias)
        pe = bert.embeddings.position_embeddings.weight
        n = min(pe.shape[0], model.position_embeddings.weight.shape[0])
        model.position_embeddings.weight[:n].copy_(pe[:n])
        model.LayerNorm.weight.copy_(bert.embeddings.LayerNorm.weight)
        model.LayerNorm.bias.copy_(bert.embeddings.LayerNorm.bias)
    return model
