"""Fused linear + cross-entropy HIP kernels vs a PyTorch fp32 reference."""
import pytest
import torch

from distributed_pipeline_amd.ops import nn as ops

pytestmark = pytest.mark.gpu


def _ref(x, W, b, tgt):
    x = x.float().detach().requires_grad_(True)
    Wf = W.float().detach().requires_grad_(True)
    bf = b.float().detach().requires_grad_(True) if b is not None else None
    logits = x @ Wf.t() + (bf if bf is not None else 0)
    loss = torch.nn.functional.cross_entropy(logits, tgt, reduction="none")
    return loss, x, Wf, bf


# N < 98304: lxent_fwd_dx splits the vocabulary over blocks and merges (m, l, u) partials;
# 131072 tokens: one block per 128 tokens sweeps the whole vocabulary
@pytest.mark.parametrize("N,V,E,with_bias", [(300, 1000, 128, True), (4096, 30522, 128, True),
                                               (130, 517, 256, False), (70000, 2000, 128, True),
                                               (131072, 1000, 128, True)])
def test_lxent_fwd_bwd(N, V, E, with_bias):
    torch.manual_seed(0)
    dev = "cuda"
    x = (torch.randn(N, E, device=dev) * 0.5).bfloat16()
    W = (torch.randn(V, E, device=dev) * 0.5).bfloat16()
    b = (torch.randn(V, device=dev) * 0.1).bfloat16() if with_bias else None
    tgt = torch.randint(0, V, (N,), device=dev)
    tgt[::7] = -100 if N > 10 else tgt[::7]  # ignored tokens
    from distributed_pipeline_amd.ops._ext import get_ext
    ext = get_ext(required=True)
    loss, lse = ext.lxent_fwd(x, W, b, tgt)
    ref_loss, xr, Wr, br = _ref(x, W, b, tgt.clamp_min(0))
    ref_loss = torch.where(tgt < 0, torch.zeros_like(ref_loss), ref_loss)
    torch.testing.assert_close(loss, ref_loss, rtol=2e-3, atol=2e-3)
    g = torch.randn(N, device=dev)
    ref_loss.backward(g)
    dx, dW, db = ext.lxent_bwd(g, x, W, b, tgt, lse, True, True, with_bias)
    torch.testing.assert_close(dx.float(), xr.grad, rtol=2e-2, atol=2e-2 * xr.grad.abs().max().item())
    # fused forward + unscaled input gradient (training path): same loss / lse, and
    # g * dxu is the input gradient
    loss2, lse2, dxu = ext.lxent_fwd_dx(x, W, b, tgt)
    torch.testing.assert_close(loss2, ref_loss, rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(lse2, lse, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dxu * g[:, None], xr.grad, rtol=2e-2, atol=2e-2 * xr.grad.abs().max().item())
    torch.testing.assert_close(dW, Wr.grad, rtol=2e-2, atol=1e-2 * Wr.grad.abs().max().item())
    if with_bias:
        torch.testing.assert_close(db, br.grad, rtol=2e-2, atol=1e-2 * br.grad.abs().max().item())
    # the opt-in form: softmax-only weight-gradient kernel + sorted one-hot scatter
    _, dW2, db2 = ext.lxent_bwd(g, x, W, b, tgt, lse, False, True, with_bias, onehot_scatter=True)
    torch.testing.assert_close(dW2, Wr.grad, rtol=2e-2, atol=1e-2 * Wr.grad.abs().max().item())
    if with_bias:
        torch.testing.assert_close(db2, br.grad, rtol=2e-2, atol=1e-2 * br.grad.abs().max().item())


def test_linear_cross_entropy_autograd_matches_torch():
    torch.manual_seed(1)
    N, V, E = 512, 3000, 128
    x = torch.randn(N, E, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    W = torch.nn.Parameter(torch.randn(V, E, device="cuda") * 0.3)
    b = torch.nn.Parameter(torch.randn(V, device="cuda") * 0.1)
    tgt = torch.randint(0, V, (N,), device="cuda")
    loss = ops.linear_cross_entropy(x, W, b, tgt)
    loss.mean().backward()
    xr = x.detach().float().requires_grad_(True)
    Wr = W.detach().bfloat16().float().requires_grad_(True)
    br = b.detach().bfloat16().float().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(xr @ Wr.t() + br, tgt, reduction="none")
    ref.mean().backward()
    torch.testing.assert_close(loss, ref, rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(W.grad, Wr.grad, rtol=2e-2, atol=2e-2 * Wr.grad.abs().max().item())
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2e-2, atol=2e-2 * xr.grad.abs().max().item())


@pytest.mark.parametrize("N,V,E,with_bias,chunk_mb,keep", [(1000, 50257, 768, False, 16, True),
                                                           (1000, 50257, 768, False, 16, False),
                                                           (300, 1000, 512, True, 1, True),
                                                           # N % 128 == 0: one wgrad GEMM over all kept chunks
                                                           (1024, 50257, 768, False, 16, True),
                                                           (1024, 1000, 512, True, 1, True)])
def test_chunked_linear_cross_entropy_wide_E(N, V, E, with_bias, chunk_mb, keep, monkeypatch):
    """Wide-E path (GPT-2 LM head): hipBLASLt chunk logits + csrc/xent_rows.hip row
    kernels, several chunks (incl. a ragged last one), ignored targets, padding columns;
    logits kept from the forward (keep) or recomputed in the backward."""
    monkeypatch.setattr(ops, "_XENT_CHUNK_BYTES", chunk_mb << 20)
    if not keep:
        monkeypatch.setattr(ops, "_XENT_KEEP_BYTES", 0)
    torch.manual_seed(2)
    x = (torch.randn(N, E, device="cuda") * 0.05).bfloat16().requires_grad_(True)
    W = torch.nn.Parameter(torch.randn(V, E, device="cuda") * 0.5)
    b = torch.nn.Parameter(torch.randn(V, device="cuda") * 0.1) if with_bias else None
    tgt = torch.randint(0, V, (N,), device="cuda")
    tgt[::11] = -100
    loss = ops.linear_cross_entropy(x, W, b, tgt)
    g = torch.rand(N, device="cuda")
    (loss * g).sum().backward()
    xr = x.detach().float().requires_grad_(True)
    Wr = W.detach().bfloat16().float().requires_grad_(True)
    br = b.detach().bfloat16().float().requires_grad_(True) if with_bias else None
    logits = xr @ Wr.t() + (br if with_bias else 0)
    ref = torch.nn.functional.cross_entropy(logits, tgt.clamp_min(0), reduction="none")
    ref = torch.where(tgt < 0, torch.zeros_like(ref), ref)
    (ref * g).sum().backward()
    torch.testing.assert_close(loss, ref, rtol=1e-2, atol=3e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=3e-2, atol=3e-2 * xr.grad.abs().max().item())
    torch.testing.assert_close(W.grad, Wr.grad, rtol=3e-2, atol=2e-2 * Wr.grad.abs().max().item())
    if with_bias:
        torch.testing.assert_close(b.grad, br.grad, rtol=3e-2, atol=2e-2 * br.grad.abs().max().item())


def test_lxent_weight_gradient_bitwise_reproducible():
    """The head weight / bias gradient of the tied embedding is split over tokens; the splits'
    partials are summed in split order (no fp32 atomics), so two runs - accumulated onto a
    non-zero gradient, as into the flat .grad - give the same bits."""
    torch.manual_seed(4)
    dev = "cuda"
    N, V, E = 65536, 30522, 128
    x = (torch.randn(N, E, device=dev) * 0.5).bfloat16()
    W = (torch.randn(V, E, device=dev) * 0.5).bfloat16()
    b = (torch.randn(V, device=dev) * 0.1).bfloat16()
    tgt = torch.randint(0, V, (N,), device=dev)
    tgt[torch.rand(N, device=dev) < 0.4] = 0  # a padding-like hot target
    from distributed_pipeline_amd.ops._ext import get_ext
    ext = get_ext(required=True)
    _, lse = ext.lxent_fwd(x, W, b, tgt)
    g = torch.randn(N, device=dev)
    base_w, base_b = torch.randn(V, E, device=dev), torch.randn(V, device=dev)
    outs = []
    for _ in range(2):
        gw, gb = base_w.clone(), base_b.clone()
        ext.lxent_bwd(g, x, W, b, tgt, lse, False, True, True, dw_acc=gw, db_acc=gb)
        outs.append((gw, gb))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    ref_loss, _, Wr, br = _ref(x, W, b, tgt)
    ref_loss.backward(g)
    torch.testing.assert_close(outs[0][0] - base_w, Wr.grad, rtol=2e-2, atol=1e-2 * Wr.grad.abs().max().item())
    torch.testing.assert_close(outs[0][1] - base_b, br.grad, rtol=2e-2, atol=1e-2 * br.grad.abs().max().item())
