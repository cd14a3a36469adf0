"""Architecture presets selected by the ``config_name`` setting.

``bert-base-uncased`` is the DiffuSeq-base encoder;
``diffuseq-xl`` the ~1.3B configuration of BASELINE config #5
(26 x 2048 x 16 heads x 8192 FFN); ``gpt2`` GPT-2 small; ``tiny`` is for tests.
"""

PRESETS = {
    "bert-base-uncased": dict(hidden_size=768, num_layers=12, num_heads=12, intermediate_size=3072,
                              max_position_embeddings=512, vocab_size=30522, layer_norm_eps=1e-12),
    "bert-large-uncased": dict(hidden_size=1024, num_layers=24, num_heads=16, intermediate_size=4096,
                               max_position_embeddings=512, vocab_size=30522, layer_norm_eps=1e-12),
    "diffuseq-xl": dict(hidden_size=2048, num_layers=26, num_heads=16, intermediate_size=8192,
                        max_position_embeddings=512, vocab_size=30522, layer_norm_eps=1e-12),
    "gpt2": dict(hidden_size=768, num_layers=12, num_heads=12, intermediate_size=3072,
                 max_position_embeddings=1024, vocab_size=50257, layer_norm_eps=1e-5),
    "tiny": dict(hidden_size=64, num_layers=2, num_heads=2, intermediate_size=128,
                 max_position_embeddings=512, vocab_size=30522, layer_norm_eps=1e-12),
}


def _from_hf_dir(path):
    """Architecture of a local transformers BERT/GPT-2 checkpoint directory (config.json)."""
    import json
    import os
    with open(os.path.join(path, "config.json")) as f:
        c = json.load(f)
    H = c.get("hidden_size", c.get("n_embd"))
    return dict(hidden_size=H, num_layers=c.get("num_hidden_layers", c.get("n_layer")),
                num_heads=c.get("num_attention_heads", c.get("n_head")),
                intermediate_size=c.get("intermediate_size") or c.get("n_inner") or 4 * H,
                max_position_embeddings=c.get("max_position_embeddings", c.get("n_positions", 512)),
                vocab_size=c.get("vocab_size", 30522),
                layer_norm_eps=c.get("layer_norm_eps", c.get("layer_norm_epsilon", 1e-12)))


def resolve(config_name, **overrides):
    """Preset (or a local transformers checkpoint directory, e.g. for use_plm_init) merged
    with non-zero overrides (0 means "take the preset")."""
    import os
    if config_name in PRESETS:
        cfg = dict(PRESETS[config_name])
    elif os.path.isfile(os.path.join(str(config_name), "config.json")):
        cfg = _from_hf_dir(config_name)
    else:
        raise ValueError(f"unknown config_name {config_name!r}; known: {sorted(PRESETS)} "
                         "or a local checkpoint directory")
    for k, v in overrides.items():
        if v:
            cfg[k] = v
    if not overrides.get("intermediate_size") and overrides.get("hidden_size"):
        cfg["intermediate_size"] = 4 * cfg["hidden_size"]
    return cfg
