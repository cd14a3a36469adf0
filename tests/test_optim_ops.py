"""Numerics of the fused optimizer kernels vs torch.optim.AdamW / fp32 references."""
import math

import pytest
import torch

from distributed_pipeline_amd.ops import optim as O


def _ref_adamw(p, grads, lr, wd, steps, betas=(0.9, 0.999), eps=1e-8):
    p = p.clone().requires_grad_(True)
    opt = torch.optim.AdamW([p], lr=lr, weight_decay=wd, betas=betas, eps=eps)
    for g in grads:
        p.grad = g.clone()
        opt.step()
    return p.detach(), opt.state[p]


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("gdtype", [torch.float32, torch.bfloat16])
def test_fused_adamw_matches_torch(device, gdtype):
    torch.manual_seed(0)
    n = 4096 + 64
    p0 = torch.randn(n)
    grads = [torch.randn(n).to(gdtype).float() for _ in range(3)]
    ref_p, ref_state = _ref_adamw(p0, grads, lr=1e-3, wd=0.01, steps=3)

    p = p0.clone().to(device)
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    shadow = torch.empty(n, dtype=torch.bfloat16, device=device)
    ema = [torch.zeros_like(p), p.clone()]
    ema_ref = [torch.zeros(n), p0.clone()]
    rates = [0.5, 0.99]
    for step, g in enumerate(grads, 1):
        O.adamw_ema_(p, g.to(device=device, dtype=gdtype), m, v, lr=1e-3, beta1=0.9, beta2=0.999,
                     eps=1e-8, weight_decay=0.01, step=step, shadow_bf16=shadow,
                     emas=ema, ema_rates=rates)
    # EMA reference from the torch trajectory
    pr = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([pr], lr=1e-3, weight_decay=0.01)
    for g in grads:
        pr.grad = g.clone()
        opt.step()
        for e, r in zip(ema_ref, rates):
            e.mul_(r).add_(pr.detach(), alpha=1 - r)
    torch.testing.assert_close(p.cpu(), ref_p, rtol=1e-5, atol=5e-5)
    torch.testing.assert_close(m.cpu(), ref_state["exp_avg"], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(v.cpu(), ref_state["exp_avg_sq"], rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(shadow.float().cpu(), p.cpu().bfloat16().float(), rtol=0, atol=0)
    for e, er in zip(ema, ema_ref):
        torch.testing.assert_close(e.cpu(), er, rtol=1e-5, atol=5e-5)


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_grad_norm_and_clip(device):
    torch.manual_seed(1)
    g = torch.randn(1 << 16).to(device)
    out = torch.zeros(3, device=device)
    O.grad_norm_(g, out, scale=0.5, max_norm=10.0)
    ref = (g.double() * 0.5).norm().item()
    assert math.isclose(out[0].item(), ref, rel_tol=1e-5)
    coef = min(1.0, 10.0 / (ref + 1e-6))
    assert math.isclose(out[1].item(), coef, rel_tol=1e-5)
    assert math.isclose(out[2].item(), ref * coef, rel_tol=1e-5)


@pytest.mark.gpu
def test_native_extension_loaded_on_gpu():
    from distributed_pipeline_amd.ops._ext import get_ext
    assert get_ext(required=True) is not None
