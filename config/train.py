"""
Training settings (L4).  Field names, defaults and JSON key order of
``GeneralSettings`` / ``DataSettings`` match the reference
(reference: config/train.py:6-46), so reference ``train_config.json`` files load
unchanged.  ``YourSettings`` is filled with the workload groups the reference
left as a TODO: model, diffusion and MI355X performance settings.

``--config_json`` semantics (reference config/train.py:57-77): the JSON file is
loaded first; unlike the reference, individual flags are no longer mutually
exclusive and any flag given explicitly on the command line is applied on top
of the JSON (the reference silently ignored them).
"""
import json
import sys
from typing import final
from argparse import ArgumentParser as Ap, ArgumentDefaultsHelpFormatter as Df

from .base import S, Choice, Item as _


class GeneralSettings(S):
    lr: float \
        = _(1e-4, "Learning Rate")
    batch_size: int \
        = _(2048, "Batch size of running step and optimizing")
    microbatch: int \
        = _(64, "Batch size for forward and backward")
    learning_steps: int \
        = _(320000, "Steps for whole iteration")
    log_interval: int \
        = _(20, "Steps per log")
    save_interval: int \
        = _(2000, "Steps per save")
    eval_interval: int \
        = _(1000, "Steps per eval")
    ema_rate: str \
        = _("0.5,0.9,0.99", "EMA rate. separate rates by comma(',').")
    seed: int \
        = _(102, "Seed for train or test.")
    resume_checkpoint: str \
        = _("", "Checkpoint path(.pt) to resume training")
    checkpoint_path: str \
        = _("", "! This will be automatically updated while training !")
    gradient_clipping: float \
        = _(0., "Gradient clipping (>0), default: 0 (no clipping). ")
    weight_decay: float \
        = _(0., "Weight decay.")


class DataSettings(S):
    dataset: str \
        = _("dataset", "Name of dataset ('synthetic' = random tokens; otherwise {data_dir}/{split}.jsonl).")
    data_dir: str \
        = _("datasets/dataset", "Path for dataset to be saved.")
    data_loader_workers: int \
        = _(2, "num_workers for DataLoader.")


class ModelSettings(S):
    model: Choice("diffuseq", "mlp_diffusion", "gpt2") \
        = _("diffuseq", "Model family built by create_model_from_config.")
    config_name: str \
        = _("bert-base-uncased", "Encoder preset: bert-base-uncased | diffuseq-xl | gpt2 | tiny (see models/presets).")
    vocab_size: int \
        = _(30522, "Vocabulary size.")
    seq_len: int \
        = _(128, "Sequence length.")
    hidden_t_dim: int \
        = _(128, "Timestep-embedding dim.")
    hidden_dim: int \
        = _(128, "Word-embedding (diffusion space) dim.")
    hidden_size: int \
        = _(0, "Transformer width (0 = from config_name).")
    num_layers: int \
        = _(0, "Transformer depth (0 = from config_name).")
    num_heads: int \
        = _(0, "Attention heads (0 = from config_name).")
    intermediate_size: int \
        = _(0, "FFN width (0 = 4*hidden_size / from config_name).")
    dropout: float \
        = _(0.1, "Dropout probability (hidden and attention).")
    use_plm_init: Choice("no", "bert") \
        = _("no", "Initialise the encoder from a pretrained LM (offline: must be on disk).")


class DiffusionSettings(S):
    diffusion_steps: int \
        = _(2000, "Number of diffusion steps T.")
    noise_schedule: Choice("sqrt", "linear", "cosine", "trunc_cos", "trunc_lin", "pw_lin") \
        = _("sqrt", "Noise schedule.")
    schedule_sampler: Choice("uniform", "lossaware", "fixstep") \
        = _("uniform", "Timestep sampler.")
    predict_xstart: bool \
        = _(True, "Model predicts x0 (DiffuSeq default).")
    rescale_timesteps: bool \
        = _(True, "Feed t*1000/T to the model.")
    learn_sigma: bool \
        = _(False, "Learn the variance (unsupported, must be false).")
    rescale_learned_sigmas: bool \
        = _(False, "Unused unless learn_sigma.")
    sigma_small: bool \
        = _(False, "Use the small posterior variance.")
    emb_scale_factor: float \
        = _(1.0, "Scale applied to word embeddings.")


class PerfSettings(S):
    precision: Choice("bf16", "fp32") \
        = _("bf16", "Compute precision (fp32 master weights, AdamW and EMA always).")
    ddp_engine: Choice("native", "torch") \
        = _("native", "native = flat-bucket RCCL engine (+fused optimizer); torch = torch DDP + torch AdamW (reference-equivalent).")
    ddp_bucket_cap_mb: float \
        = _(0.0, "All-reduce bucket size (MiB) for the native engine; 0 (default) = measured at startup on the job's process group (all-reduce bandwidth sweep; 32 at world 1).")
    ddp_first_bucket_mb: float \
        = _(0.0, "First (last-layer) bucket size (MiB) so communication starts early; 0 (default) = measured (4 at world 1).")
    grad_reduce_dtype: Choice("fp32", "bf16") \
        = _("fp32", "Dtype on the wire for the gradient all-reduce.")
    shard_optimizer: bool \
        = _(False, "ZeRO-1: reduce-scatter gradients and shard AdamW moments + EMAs over the data-parallel ranks.")
    use_hip_kernels: bool \
        = _(True, "Use the hand-written gfx950 kernels (required on GPU).")
    exec_microbatch: int \
        = _(0, "Samples per executed forward/backward, a multiple of microbatch: 0 = auto (the whole "
               "per-rank batch, halved on out-of-memory), -1 = microbatch (the reference schedule). "
               "Gradients equal the reference's sum over micro-batches.")
    overlap_microbatches: bool \
        = _(True, "With several executed micro-batches per step (e.g. exec_microbatch=-1), run micro-batch "
                  "k+1's forward on a second HIP stream while k's backward runs (bitwise-identical gradients).")
    defer_wgrad: int \
        = _(8, "With several executed micro-batches per step: hold each Linear's weight-gradient operands for "
               "this many micro-batches and run them as one multi-segment split-K GEMM (same fp32 sum; "
               "0/1 = off, at most 8).")
    shard_data: bool \
        = _(False, "Give each rank a disjoint shard of the data (DistributedSampler-style).")
    log_cross_rank_mean: bool \
        = _(False, "Average logged metrics over ranks at dump time.")


class RuntimeSettings(S):
    """Observability, debugging and failure handling."""
    nan_guard: Choice("off", "skip", "abort") \
        = _("off", "Non-finite gradient norm: off | skip the optimizer step | abort.")
    debug_anomaly: bool \
        = _(False, "torch.autograd.set_detect_anomaly(True).")
    consistency_check_interval: int \
        = _(0, "Every N steps verify parameters are identical on all ranks (0 = off).")
    profile_steps: str \
        = _("", "torch.profiler window 'start:stop' (chrome trace in the run dir); empty = off.")
    roctx: bool \
        = _(False, "Emit roctx ranges (fwd/bwd/optimize/allreduce) for rocprofv3 --marker-trace.")
    save_rng_state: bool \
        = _(True, "Write rng_{step}_rank{r}.pt next to each checkpoint and restore it on resume.")
    tensorboard: bool \
        = _(False, "Also log scalars to TensorBoard event files (run_dir/tb).")


class YourSettings(RuntimeSettings, PerfSettings, DiffusionSettings, ModelSettings):
    """Workload-specific settings (the reference's TODO mixin)."""


@final
class TrainSettings(
        YourSettings,
        DataSettings,
        GeneralSettings
):

    @classmethod
    def to_argparse(cls, parser_or_group=None, add_json=False):
        if not add_json:
            return super(TrainSettings, cls).to_argparse(parser_or_group)
        if parser_or_group is None:
            parser_or_group = Ap(formatter_class=Df)
        setting_group = parser_or_group.add_argument_group(title="settings")
        setting_group.add_argument(
            "--config_json", type=str, required=False,
            help="Load all settings from this JSON file; flags given explicitly override it.")
        super(TrainSettings, cls).to_argparse(setting_group, _suppress_defaults=True)
        return parser_or_group

    @classmethod
    def from_argparse(cls, namespace, _top=True):
        ns = dict(vars(namespace)) if not isinstance(namespace, dict) else dict(namespace)
        cfg = ns.pop("config_json", None)
        overrides = {k: v for k, v in ns.items() if k in cls.model_fields}
        unknown = set(ns) - set(overrides)
        assert not (_top and unknown), str(unknown)
        if cfg:
            with open(cfg, "r") as f:
                data = json.load(f)
            if overrides:
                print(f"<INFO> --config_json {cfg}: overriding {sorted(overrides)} from the command line",
                      file=sys.stderr)
            data.update(overrides)
            return cls(**data)
        return cls(**overrides)


__all__ = ('TrainSettings', 'GeneralSettings', 'DataSettings', 'ModelSettings',
           'DiffusionSettings', 'PerfSettings', 'RuntimeSettings', 'YourSettings')
