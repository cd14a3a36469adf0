"""The byte-cutting GEMM epilogues (csrc/gemm256.hip):

* EPI 8 / act code 5: the ffn-in forward stores act'(z) as 8-bit codes (two linear segments,
  bf16's own grid on [0.5, 1.13]) and the ffn-out data-gradient epilogue decodes them;
* EPI 7: the post-LN branch output's residual + dropout in the producing GEMM's epilogue
  (pair-hash bits), with the LayerNorm backward regenerating the same bits.

References are plain fp32 PyTorch of the same formulas; the dropout mask comes from the host
mirror of the hash (distributed_pipeline_amd/ops/dropout_ref.py)."""
import math

import pytest
import torch

from distributed_pipeline_amd.ops import nn as opsnn
from distributed_pipeline_amd.ops.dropout_ref import pair_keep_mask
from distributed_pipeline_amd.ops._ext import get_ext

pytestmark = pytest.mark.gpu


def _dact_ref(a, act):
    if act == 1:
        return 0.5 * (1 + torch.erf(a / 2 ** 0.5)) + a * torch.exp(-0.5 * a * a) / (2 * math.pi) ** 0.5
    s = torch.sigmoid(a)
    return s * (1 + a * (1 - s))


def _bf16_half_ulp(v):
    """half a bf16 ulp at |v| (fp32 tensor)"""
    e = torch.floor(torch.log2(v.abs().clamp_min(2.0 ** -126)))
    return 2.0 ** (e - 8)


@pytest.mark.parametrize("act", [1, 3])
def test_act_q8_codes_over_the_bf16_range(act):
    """Every bf16 pre-activation in [-8, 8] (and the extremes) through the forward epilogue:
    the decoded act' is within 0.0035 of fp32 act'(z) everywhere and within bf16's own rounding
    of act' wherever |act'| >= 0.5 (where the code grid is bf16's grid); 0 and 1 exact."""
    ext = get_ext(required=True)
    # all bf16 values in [-8, 8] plus large magnitudes, laid out as x[t, k]
    bits = torch.arange(0, 1 << 16, dtype=torch.int32).to(torch.int16)
    vals = bits.view(torch.bfloat16).float()
    vals = vals[torch.isfinite(vals) & ((vals.abs() <= 8) | (vals.abs() >= 1e3))]
    K = 128
    T = -(-vals.numel() // K)
    T = -(-T // 256) * 256
    xs = torch.zeros(T * K)
    xs[:vals.numel()] = vals
    x = xs.view(T, K).bfloat16().cuda()
    N = 256
    W = torch.zeros(N, K)
    W[torch.arange(N), torch.arange(N) % K] = 1.0   # z[t, n] = x[t, n % 128] exactly
    W = W.bfloat16().cuda()
    y, z8, mode = ext.gemm_nt(x, W, None, act, 2)
    assert mode == 2 and z8.dtype == torch.uint8 and z8.numel() == T * N
    zr = x.float()[:, torch.arange(N) % K]
    d = opsnn.act_q8_decode(z8, T, N)
    ref = _dact_ref(zr.double(), act).float()
    err = (d - ref).abs()
    assert err.max().item() <= 0.0035, err.max().item()
    big = ref.abs() >= 0.5
    assert bool((err[big] <= _bf16_half_ulp(ref[big]) + 5e-7).all()), (err[big] - _bf16_half_ulp(ref[big])).max()
    sat_hi, sat_lo = zr > (6 if act == 1 else 30), zr < -30
    assert bool((d[sat_hi] == 1.0).all()) and bool((d[sat_lo] == 0.0).all())
    # y is the same as the bf16-act' forward's
    y1, _, mode1 = ext.gemm_nt(x, W, None, act, 1)
    assert mode1 == 1 and torch.equal(y, y1)


@pytest.mark.parametrize("T,K,N", [(32768, 768, 3072), (16384, 1024, 4096)])
def test_act_q8_dact_gemm_matches_reference(T, K, N):
    """ffn-in forward with u8 act' -> ffn-out data gradient with act code 5 (and its bias
    column sums) against fp32 math on the decoded codes."""
    ext = get_ext(required=True)
    torch.manual_seed(7)
    x = torch.randn(T, K, device="cuda").bfloat16()
    W1 = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    b1 = torch.randn(N, device="cuda").bfloat16()
    y, z8, mode = ext.gemm_nt(x, W1, b1, 1, 2)
    assert mode == 2
    zr = (x.float() @ W1.float().t() + b1.float()).bfloat16().float()
    assert (opsnn.act_q8_decode(z8, T, N) - _dact_ref(zr, 1)).abs().max().item() < 0.02
    dy = torch.randn(T, K, device="cuda").bfloat16()
    W2 = (torch.randn(K, N, device="cuda") * 0.05).bfloat16()
    dz, db = ext.gemm_nn_dact(dy, W2, z8, 5, True)
    ref = (dy.float() @ W2.float()).bfloat16().float() * opsnn.act_q8_decode(z8, T, N)
    err = (dz.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item(), err
    torch.testing.assert_close(db, dz.float().sum(0), rtol=1e-2, atol=1e-2 * db.abs().max().item())
    # without the bias sums (EPI 3) the same values
    dz3, _ = ext.gemm_nn_dact(dy, W2, z8, 5, False)
    assert torch.equal(dz3, dz)


@pytest.mark.parametrize("T,K,N,p", [(16384, 768, 768, 0.1), (8192, 3072, 768, 0.1), (4096, 2048, 2048, 0.0),
                                     (4096, 768, 768, 0.3)])
def test_residual_dropout_epilogue_mask_and_values(T, K, N, p):
    ext = get_ext(required=True)
    torch.manual_seed(11)
    x = torch.randn(T, K, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    b = torch.randn(N, device="cuda").bfloat16()
    res = torch.randn(T, N, device="cuda").bfloat16()
    seed, off = 1234, 77
    h = ext.gemm_nt_res(x, W, b, res, p, seed, off)
    assert h is not None
    keep = pair_keep_mask(seed, off, T, N, p).cuda()
    if p > 0:
        assert abs(keep.float().mean().item() - (1 - p)) < 0.01
    y = (x.float() @ W.float().t() + b.float()).bfloat16().float()
    ref = res.float() + torch.where(keep, y / (1 - p), torch.zeros_like(y))
    # dropped elements are the residual exactly
    assert torch.equal(h[~keep], res[~keep])
    err = (h.float() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item(), err
    # the plain forward GEMM gives y
    y0, _, _ = ext.gemm_nt(x, W, b, 0)
    assert (y0.float() - y).abs().max().item() <= 1e-2 * y.abs().max().item()


def test_ln_backward_pair_hash_regenerates_the_epilogue_mask():
    """h = res + dropout(x W^T + b) (GEMM epilogue) -> LN forward -> LN backward in pair-hash
    mode: dy is zero exactly where the epilogue dropped, and (dres, dy) match torch autograd
    through the same mask."""
    ext = get_ext(required=True)
    torch.manual_seed(12)
    T, K, N, p, eps = 8192, 768, 768, 0.1, 1e-12
    x = torch.randn(T, K, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    b = torch.randn(N, device="cuda").bfloat16()
    res = torch.randn(T, N, device="cuda").bfloat16()
    g = (1 + 0.1 * torch.randn(N, device="cuda")).bfloat16()
    be = (0.1 * torch.randn(N, device="cuda")).bfloat16()
    seed, off = 99, 5
    h = ext.gemm_nt_res(x, W, b, res, p, seed, off)
    out, hs, mean, rstd = ext.add_ln_fwd(h, None, g, be, 0.0, eps, 0, 0, save_h=False)
    assert hs is None
    dout = torch.randn(T, N, device="cuda").bfloat16()
    dres, dy, dg, db, dyb = ext.add_ln_bwd(dout, h, mean, rstd, g, p, seed, off, True, True, True,
                                           pair_hash=True)
    keep = pair_keep_mask(seed, off, T, N, p).cuda()
    assert bool((dy[~keep] == 0).all())
    # torch reference through the same mask
    yb = (x.float() @ W.float().t() + b.float()).bfloat16().float().requires_grad_(True)
    rr = res.float().requires_grad_(True)
    hh = rr + torch.where(keep, yb / (1 - p), torch.zeros_like(yb))
    o = torch.nn.functional.layer_norm(hh, (N,), g.float(), be.float(), eps)
    torch.testing.assert_close(out.float(), o.detach(), rtol=3e-2, atol=3e-2)
    o.backward(dout.float())
    for a, r in ((dres, rr.grad), (dy, yb.grad)):
        e = (a.float() - r).abs().max().item()
        assert e <= 2e-2 * r.abs().max().item(), e
    torch.testing.assert_close(dyb, yb.grad.sum(0), rtol=2e-2, atol=2e-2 * yb.grad.sum(0).abs().max().item())


def test_fused_sublayers_res_gemm_match_composed_no_dropout(monkeypatch):
    """The one-op post-LN sublayers with the residual in the GEMM epilogue against the same
    layer built from the separate ops (dropout off: no mask to match), forward and backward."""
    from distributed_pipeline_amd.models.layers import BertLayer
    torch.manual_seed(0)
    lyr = BertLayer(256, 4, 1024, 0.0).cuda().train()
    x = torch.randn(4, 128, 256, device="cuda").bfloat16()
    dout = torch.randn(4, 128, 256, device="cuda").bfloat16()

    def run():
        lyr.zero_grad(set_to_none=True)
        xi = x.clone().requires_grad_(True)
        out = lyr(xi)
        out.backward(dout)
        return out.float(), xi.grad.float(), {n: q.grad.clone() for n, q in lyr.named_parameters()}

    assert opsnn._RES_FUSE
    o_f, dx_f, g_f = run()
    monkeypatch.setattr(opsnn, "_ln_block_ok", lambda *a, **k: False)
    o_c, dx_c, g_c = run()
    torch.testing.assert_close(o_f, o_c, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(dx_f, dx_c, rtol=3e-2, atol=3e-2 * dx_c.abs().max().item())
    for n in g_c:
        scale = g_c[n].abs().max().item() + 1e-6
        assert (g_f[n] - g_c[n]).abs().max().item() / scale < 3e-2, n


def test_q8_mlp_backward_survives_a_gemm256_toggle(monkeypatch):
    """a forward that stored u8 act' codes ("deriv8") and a backward whose fused dact
    GEMM declines (here: the persistent kernels switched off between the two, as the A/B tools
    do) must decode the codes and take the plain dgrad + activation-backward path, not fail."""
    from distributed_pipeline_amd.models.layers import Linear
    torch.manual_seed(0)
    fc1 = Linear(256, 1024, act="gelu").cuda()
    fc2 = Linear(1024, 256).cuda()
    x = torch.randn(512, 256, device="cuda").bfloat16()
    dy = torch.randn(512, 256, device="cuda").bfloat16()
    params = (*fc1.parameters(), *fc2.parameters())
    decodes = []
    real_decode = opsnn.act_q8_decode
    monkeypatch.setattr(opsnn, "act_q8_decode", lambda *a: decodes.append(1) or real_decode(*a))

    def run(toggle):
        for q in params:
            q.grad = None
        xi = x.clone().requires_grad_(True)
        y = opsnn.mlp(xi, fc1, fc2)
        if toggle:
            get_ext().set_gemm256(False)
        try:
            y.backward(dy)
        finally:
            get_ext().set_gemm256(True)
        return y.float(), xi.grad.float(), [q.grad.float().clone() for q in params]

    assert opsnn._ACT_Q8
    y0, dx0, g0 = run(False)
    assert not decodes  # the fused dact GEMM consumed the codes
    y1, dx1, g1 = run(True)
    assert decodes  # the fallback decoded them
    assert torch.equal(y0, y1)
    torch.testing.assert_close(dx1, dx0, rtol=3e-2, atol=3e-2 * dx0.abs().max().item())
    for a, b in zip(g1, g0):
        assert (a - b).abs().max().item() <= 3e-2 * (b.abs().max().item() + 1e-6)
