"""
Seeding and model construction (L6), API-compatible with the reference
``utils/initialization.py`` (reference: utils/initialization.py:1-27).

``create_model_from_config(**settings)`` receives the whole ``TrainSettings``
dict (reference run/train.py:71 passes ``**args.dict()``) and ignores keys it
does not use; it dispatches on the ``model`` setting.
"""


def seed_all(seed, deterministic=False):
    import random

    import numpy as np
    import torch

    from basic_utils.dist_util import get_rank
    if deterministic:
        seed = int(seed)
        torch.backends.cudnn.deterministic = True  # noqa
        torch.backends.cudnn.benchmark = False  # noqa
    else:
        seed = int(seed) + get_rank()  # per-rank streams
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)  # also seeds every HIP device generator
    from distributed_pipeline_amd.ops.nn import RNG
    RNG.seed = seed & 0x7FFFFFFF  # in-kernel Philox streams (dropout)
    RNG.counter = 0


def create_model_from_config(*, model="diffuseq", **settings):
    """Build the model named by ``settings['model']`` (diffuseq | mlp_diffusion | gpt2)."""
    from distributed_pipeline_amd.models import build_model
    return build_model(model=model, **settings)


def create_diffusion_from_config(*, diffusion_steps=2000, noise_schedule="sqrt", predict_xstart=True,
                                 rescale_timesteps=True, learn_sigma=False, schedule_sampler="uniform",
                                 sigma_small=False, rescale_learned_sigmas=False, **_):
    from distributed_pipeline_amd.models import create_gaussian_diffusion, create_named_schedule_sampler
    diffusion = create_gaussian_diffusion(steps=diffusion_steps, noise_schedule=noise_schedule,
                                          predict_xstart=predict_xstart,
                                          rescale_timesteps=rescale_timesteps, learn_sigma=learn_sigma,
                                          sigma_small=sigma_small,
                                          rescale_learned_sigmas=rescale_learned_sigmas)
    return diffusion, create_named_schedule_sampler(schedule_sampler, diffusion)
