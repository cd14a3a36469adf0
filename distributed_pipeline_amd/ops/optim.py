"""Flat-buffer optimizer ops: grad L2 norm / clip coefficient, fused AdamW+EMA.

GPU tensors run the gfx950 kernels of ``csrc/optim.hip``; CPU tensors use the
PyTorch reference math below (identical formulas, used by the CPU tests and as
the numerics oracle for the GPU tests).
"""
import math

import torch

from ._ext import get_ext, use_native


def grad_norm_(grad_flat, out, partial=None, scale=1.0, max_norm=0.0):
    """Write [norm, clip_coef, norm_after_clip] of ``grad_flat*scale`` into ``out`` (3 floats)."""
    if use_native(grad_flat):
        if partial is None:
            partial = torch.empty(1024, dtype=torch.float32, device=grad_flat.device)
        get_ext().sqnorm(grad_flat, partial, out, float(scale), float(max_norm))
        return out
    norm = grad_flat.detach().double().pow(2).sum().sqrt().float() * scale
    coef = torch.ones((), dtype=torch.float32, device=grad_flat.device)
    if max_norm > 0:
        coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
    out[0] = norm
    out[1] = coef
    out[2] = norm * coef
    return out


def adamw_ema_(param, grad, exp_avg, exp_avg_sq, *, lr, beta1, beta2, eps, weight_decay, step,
               grad_scale=1.0, clip=None, shadow_bf16=None, emas=(), ema_rates=(), skip=None):
    """One fused AdamW step (torch.optim.AdamW math) + EMA + bf16 shadow refresh, in place.
    ``skip``: optional int32 device flag; while it is non-zero the step changes nothing (the
    kernel reads it, so a flag set by an earlier kernel on the stream needs no host sync)."""
    if use_native(param):
        get_ext().adamw_ema(param, grad, exp_avg, exp_avg_sq, shadow_bf16, list(emas),
                            [float(r) for r in ema_rates], float(lr), float(beta1), float(beta2),
                            float(eps), float(weight_decay), int(step), float(grad_scale), clip, skip)
        return
    if skip is not None and int(skip.reshape(-1)[0]) != 0:
        return
    g = grad.float() * grad_scale
    if clip is not None:
        g = g * clip[1]
    param.mul_(1.0 - lr * weight_decay)
    exp_avg.lerp_(g, 1.0 - beta1)
    exp_avg_sq.mul_(beta2).addcmul_(g, g, value=1.0 - beta2)
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    denom = (exp_avg_sq.sqrt() / math.sqrt(bc2)).add_(eps)
    param.addcdiv_(exp_avg, denom, value=-lr / bc1)
    if shadow_bf16 is not None:
        shadow_bf16.copy_(param)
    for e, r in zip(emas, ema_rates):
        e.mul_(r).add_(param, alpha=1.0 - r)


def ema_(ema, param, rate):
    if use_native(param):
        get_ext().ema_update(ema, param, float(rate))
    else:
        ema.mul_(rate).add_(param, alpha=1.0 - rate)


def cast_bf16_(src, dst):
    if use_native(src):
        get_ext().cast_bf16(src, dst)
    else:
        dst.copy_(src)
