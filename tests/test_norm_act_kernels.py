"""Fused dropout+residual+LayerNorm and bias+activation HIP kernels vs PyTorch fp32."""
import pytest
import torch

from distributed_pipeline_amd.ops import nn as ops

pytestmark = pytest.mark.gpu


def _ext():
    from distributed_pipeline_amd.ops._ext import get_ext
    return get_ext(required=True)


@pytest.mark.parametrize("R,D,res", [(1000, 768, True), (37, 128, False), (4096, 2048, True), (64, 64, True)])
def test_add_ln_no_dropout(R, D, res):
    torch.manual_seed(0)
    y = torch.randn(R, D, device="cuda").bfloat16()
    r = torch.randn(R, D, device="cuda").bfloat16() if res else None
    g = (1 + 0.1 * torch.randn(D, device="cuda")).bfloat16()
    b = (0.1 * torch.randn(D, device="cuda")).bfloat16()
    out, hs, mean, rstd = _ext().add_ln_fwd(y, r, g, b, 0.0, 1e-12, 1, 0)
    h = y.float() + (r.float() if res else 0)
    h = h.bfloat16().float().requires_grad_(True)
    gf = g.float().requires_grad_(True)
    bf = b.float().requires_grad_(True)
    ref = torch.nn.functional.layer_norm(h, (D,), gf, bf, 1e-12)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)
    dout = torch.randn(R, D, device="cuda").bfloat16()
    ref.backward(dout.float())
    dres, dy, dg, db, dyb = _ext().add_ln_bwd(dout, hs, mean, rstd, g, 0.0, 1, 0, res, True, True)
    torch.testing.assert_close(dy.float(), h.grad, rtol=2e-2, atol=2e-2)
    ref_dyb = dy.float().sum(0)  # column sums of the emitted bf16 dy (next layer's bias grad)
    torch.testing.assert_close(dyb, ref_dyb, rtol=1e-3, atol=1e-3 * ref_dyb.abs().max().item())
    if res:
        torch.testing.assert_close(dres.float(), h.grad, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(dg, gf.grad, rtol=1e-2, atol=1e-2 * gf.grad.abs().max().item())
    torch.testing.assert_close(db, bf.grad, rtol=1e-2, atol=1e-2 * bf.grad.abs().max().item())


def test_add_ln_dropout_statistics_and_consistency():
    torch.manual_seed(0)
    R, D, p = 2048, 768, 0.1
    y = torch.ones(R, D, device="cuda").bfloat16()
    g = torch.ones(D, device="cuda").bfloat16()
    b = torch.zeros(D, device="cuda").bfloat16()
    out, hs, mean, rstd = _ext().add_ln_fwd(y, None, g, b, p, 1e-5, 7, 3)
    kept = (hs.float() != 0).float().mean().item()
    assert abs(kept - (1 - p)) < 0.01
    # same seed/offset -> same mask; different offset -> different mask
    _, hs2, _, _ = _ext().add_ln_fwd(y, None, g, b, p, 1e-5, 7, 3)
    _, hs3, _, _ = _ext().add_ln_fwd(y, None, g, b, p, 1e-5, 7, 4)
    assert torch.equal(hs, hs2) and not torch.equal(hs, hs3)
    # backward regenerates the same mask: dy is zero exactly where dropped
    dout = torch.randn(R, D, device="cuda").bfloat16()
    _, dy, _, _, dyb = _ext().add_ln_bwd(dout, hs, mean, rstd, g, p, 7, 3, False, True, True)
    assert torch.equal(dy == 0, hs == 0)
    torch.testing.assert_close(dyb, dy.float().sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("act", ["none", "gelu", "tanh", "silu"])
def test_linear_bias_act_autograd(act):
    torch.manual_seed(0)
    x = torch.randn(333, 256, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = torch.nn.Parameter(torch.randn(512, 256, device="cuda") * 0.05)
    b = torch.nn.Parameter(torch.randn(512, device="cuda") * 0.1)
    y = ops.linear(x, w, b, act)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().bfloat16().float().requires_grad_(True)
    br = b.detach().bfloat16().float().requires_grad_(True)
    z = xr @ wr.t() + br
    yr = {"none": z, "gelu": torch.nn.functional.gelu(z), "tanh": torch.tanh(z),
          "silu": torch.nn.functional.silu(z)}[act]
    yr.backward(dy.float())
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=3e-2, atol=3e-2 * xr.grad.abs().max().item())
    torch.testing.assert_close(w.grad, wr.grad, rtol=3e-2, atol=3e-2 * wr.grad.abs().max().item())
    torch.testing.assert_close(b.grad, br.grad, rtol=3e-2, atol=3e-2 * br.grad.abs().max().item())
