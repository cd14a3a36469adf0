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


def resolve(config_name, **overrides):
    """Preset merged with non-zero overrides (0 means "take the preset")."""
    if config_name not in PRESETS:
        raise ValueError(f"unknown config_name {config_name!r}; known: {sorted(PRESETS)}")
    cfg = dict(PRESETS[config_name])
    for k, v in overrides.items():
        if v:
            cfg[k] = v
    if not overrides.get("intermediate_size") and overrides.get("hidden_size"):
        cfg["intermediate_size"] = 4 * cfg["hidden_size"]
    return cfg
